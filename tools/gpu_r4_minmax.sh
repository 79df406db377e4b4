#!/bin/bash
# Round-4 A/B: the compressed min-sum check kernel's row minimum as fp64
# min / max with the sign parity and NaN flag as lane masks (the tree,
# ab_lib/libldpc_amd_new.so; a NaN row falls back to the selects) against the
# select chain (old), config 5 at 1M codewords alternating on one box; then
# the min-sum / coded / non-finite GPU parity tests on the tree.
set -o pipefail
out=gpurun_out/minmax; mkdir -p $out
ROUNDS=3 VARIANTS="old new" bash tools/gpu_ab_lib.sh minmax/c5 --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_coded_input.py -x -q --timeout 200 --timeout-method thread -k "msa or min_sum or coded or nonfinite or nan or split_syndrome" > $out/pytest_new.txt 2>&1; rc=$?
tail -2 $out/pytest_new.txt
exit $rc
