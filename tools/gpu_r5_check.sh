#!/bin/bash
# Round 5: the new GPU tests first (lane-index bounds checks, the N > 1 bench
# line's cpu_baseline + config-4 leg), then the whole GPU suite and a short
# default bench.  Each step under its own limit; the first failure ends the call.
set -u
TAG=${1:-r5check}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_new 400 python -u -m pytest tests/test_lane_bounds_gpu.py tests/test_sharded_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
run pytest_all 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15
run bench 300 python -u bench.py --steps 5 --warmup 1
exit 0
