#!/bin/bash
# Round 5: guard form v5 (the refill fault flag in a VGPR: k_var_msa_c at 96
# SGPRs, 7 waves per SIMD like no guards) against no guards (ng), same box.
set -o pipefail
T=${1:-r5guard5}; out=gpurun_out/$T; mkdir -p $out
ROUNDS=3 VARIANTS="ng v5" timeout -k 10 500 bash tools/gpu_ab_lib.sh $T/c5 --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_lane_bounds_gpu.py -x -q --timeout 200 --timeout-method thread > $out/pytest.txt 2>&1; rc=$?
tail -2 $out/pytest.txt
exit $rc
