#!/bin/bash
# Round 5: tools/xr2probe (the L2-resident BP iteration) with the check task's parts.
set -o pipefail
T=${1:-r5xr2}; out=gpurun_out/$T; mkdir -p $out
timeout -k 10 180 tools/xr2probe tests/golden/decode_n18432_m2048_final.pchk > $out/xr2probe.txt 2>&1; rc=$?
cat $out/xr2probe.txt
exit $rc
