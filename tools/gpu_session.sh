#!/bin/bash
# One GPU-box session: parity tests, a short bench, a rocprofv3 kernel-trace
# profile.  Every GPU step has its own time limit; a fault / abort / timeout
# (exit >= 124) ends the session immediately.  A plain test failure (exit 1)
# does not stop the bench.
#   usage: tools/gpu_session.sh <tag> [bench args...]
set -u
TAG=${1:-r1}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if fatal $rc; then echo "fatal after pytest"; exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
if fatal $rc; then exit $rc; fi

timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
if fatal $rc; then exit $rc; fi
exit 0
