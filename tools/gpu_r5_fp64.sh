#!/bin/bash
# Round 5: tools/fp64bench (the check row's fp64 work without memory traffic).
set -o pipefail
T=${1:-r5fp64}; out=gpurun_out/$T; mkdir -p $out
timeout -k 10 120 tools/fp64bench > $out/fp64bench.txt 2>&1; rc=$?
cat $out/fp64bench.txt
exit $rc
