#!/bin/bash
# Same-box A/B of two library builds on config 5 (1M codewords, min-sum),
# ab_lib/libldpc_amd_{old,new}.so alternating (ROUNDS, default 3; the tree
# must be the new build), then the min-sum / coded / non-finite GPU parity
# tests on the tree.
#   usage: [ROUNDS=3] tools/gpu_ab_msa.sh <tag>
set -o pipefail
out=gpurun_out/${1:-abmsa}; mkdir -p $out
ROUNDS=${ROUNDS:-3} VARIANTS="old new" bash tools/gpu_ab_lib.sh ${1:-abmsa}/c5 --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_coded_input.py -x -q --timeout 200 --timeout-method thread -k "msa or min_sum or coded or nonfinite or nan or split_syndrome" > $out/pytest_new.txt 2>&1; rc=$?
tail -2 $out/pytest_new.txt
exit $rc
