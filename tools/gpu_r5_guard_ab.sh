#!/bin/bash
# Round 5: same-box A/B of the lane-index guards (ab_lib old = built with
# -DLDPC_AB_NO_LANE_GUARD, new = the tree) on config 5 and config 3, then the
# guard tests and the min-sum / coded parity tests on the tree.  Each step
# under its own limit.
set -o pipefail
T=${1:-r5guard}; out=gpurun_out/$T; mkdir -p $out
ROUNDS=3 VARIANTS="old new" timeout -k 10 400 bash tools/gpu_ab_lib.sh $T/c5 --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
ROUNDS=2 VARIANTS="old new" timeout -k 10 300 bash tools/gpu_ab_lib.sh $T/c3 --secondary 0 --steps 3 --warmup 1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_lane_bounds_gpu.py tests/test_gpu_parity.py tests/test_coded_input.py tests/test_engine_guard_gpu.py -x -q --timeout 200 --timeout-method thread > $out/pytest.txt 2>&1; rc=$?
tail -2 $out/pytest.txt
exit $rc
