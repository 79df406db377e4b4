#!/bin/bash
# Round 5: the kept guard form (v4: plain compares, faults reported at the
# kernel's end) against no guards (ng), same box, alternating; then the guard
# and bench tests and one default bench line (with the HBM-streaming leg).
set -o pipefail
T=${1:-r5guard4}; out=gpurun_out/$T; mkdir -p $out
ROUNDS=3 VARIANTS="ng v4" timeout -k 10 500 bash tools/gpu_ab_lib.sh $T/c5 --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
ROUNDS=1 VARIANTS="ng v4" timeout -k 10 200 bash tools/gpu_ab_lib.sh $T/c3 --secondary 0 --steps 3 --warmup 1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_lane_bounds_gpu.py tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1; rc=$?
tail -3 $out/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err; rc=$?
tail -c 600 $out/bench_default.json
exit $rc
