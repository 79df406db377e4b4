#!/bin/bash
# parity tests + schedule sweep.   usage: tools/gpu_sweep.sh <tag> [sweep args...]
set -u
TAG=${1:-sweep}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
  if fatal $rc; then exit $rc; fi
fi
timeout -k 10 900 python tools/sweep.py "$@" > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
rc=$?; echo "sweep rc=$rc"; cat "$OUT/sweep.jsonl"; tail -5 "$OUT/sweep.err"
exit 0
