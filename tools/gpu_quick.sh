#!/bin/bash
# Quick check: selected GPU parity tests (-k expression), then bench lines.
#   usage: tools/gpu_quick.sh <tag> "<pytest -k expr>" [bench arg sets separated by ';']
set -u
TAG=${1:-quick}; K=${2:-resident}; BENCHES=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
i=0
IFS=';' read -ra SETS <<< "$BENCHES"
for b in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py $b > "$OUT/bench$i.json" 2> "$OUT/bench$i.err"
  rc=$?; echo "bench$i ($b) rc=$rc"; cat "$OUT/bench$i.json"; tail -2 "$OUT/bench$i.err"
  if fatal $rc; then exit $rc; fi
done
exit 0
