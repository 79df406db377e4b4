#!/bin/bash
# End-of-round validation on HEAD: the whole GPU suite, smoke, the default
# bench line (as the driver runs it: --steps 20 --warmup 5), and a rocprofv3
# kernel trace of the default bench command.  Each step under its own limit.
set -u
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_all 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=30
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 400 python -u bench.py --steps 20 --warmup 5
run trace_default 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o run --output-format csv -- python3 "$R/bench.py"
rm -f "$OUT"/trace_default/*kernel_trace.csv
exit 0
