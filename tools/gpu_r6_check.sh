#!/bin/bash
# Round 6 targeted check: the GPU tests touched this round (fault words,
# pipeline codes, DNA LLR codes, CLI) and one default bench line.
set -u
TAG=${1:-r6check}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_touched 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_lane_bounds_gpu.py tests/test_dna_pipeline.py tests/test_dna_llr_gpu.py tests/test_cli_gpu.py
run bench_default 400 python -u bench.py --steps 5 --warmup 2
exit 0
