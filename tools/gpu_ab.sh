#!/bin/bash
# Selected GPU tests (-k expression, may be empty), then an in-process A/B of
# engine variants (tools/ab_engines.py arguments).
#   usage: tools/gpu_ab.sh <tag> "<pytest -k expr>" <ab_engines.py args...>
set -u
TAG=${1:-ab}; K=${2:-}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u tools/ab_engines.py "$@" > "$OUT/ab.json" 2> "$OUT/ab.err"
  rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.json"; tail -3 "$OUT/ab.err"; exit $rc
fi
exit 0
