#!/bin/bash
# Validation session: targeted parity tests first (MSA-C, goldens,
# schedules), then the whole GPU suite with per-test durations, then smoke.
# Each step has its own limit and writes to gpurun_out/<tag>/; a failing
# step ends the session.
#   usage: tools/gpu_r3_check.sh <tag> [pytest -k expression for the first step]
set -u
TAG=${1:-check}
K=${2:-"min_sum or golden or single_codeword"}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 25 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_quick 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" --durations=10
run pytest_all 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=50
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
