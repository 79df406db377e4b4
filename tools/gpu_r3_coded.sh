#!/bin/bash
# Coded-input session: the coded-input tests, the parity tests that now take
# the host API's code path, then the default bench (codes) and the fp64-input
# bench for comparison.  Each step has its own limit; a failing step ends it.
#   usage: tools/gpu_r3_coded.sh <tag> [pytest -k expression]
set -u
TAG=${1:-r3coded}
K=${2:-"coded or dna_batch or lr_table or single_fill or min_sum_compressed or resident_pool or golden"}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 25 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_coded 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" --durations=10
run bench_code 400 python -u bench.py
run bench_fp64 300 python -u bench.py --input fp64 --cpu-baseline 0
exit 0
