#!/bin/bash
# Upper bound of a code-free compressed min-sum check phase: the same bench
# with the check kernel's per-edge code stores skipped (LDPC_FULL_LANES bit 64;
# results are NOT valid then -- only the per-launch kernel times are compared).
set -u
TAG=${1:-exp_nocodes}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 600 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
ARGS="--algo msa --p 0.02 --batch-per-gpu 131072 --max-iter 20 --steps 2 --warmup 1 --cpu-baseline 0"
for r in 1 2; do
  run base_$r 200 env LDPC_FULL_LANES=1 python bench.py $ARGS
  run nocodes_$r 200 env LDPC_FULL_LANES=65 python bench.py $ARGS
done
exit 0
