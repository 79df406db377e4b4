#!/bin/bash
# Compressed min-sum with / without per-edge code bytes (LDPC_MSA_META): the
# MSA-C parity tests, then config 5 (BSC p = 0.002, 1M codewords, min-sum)
# alternating meta on / off on one box, then the default line with its oracle
# check.
set -u
TAG=${1:-ab_meta}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 700 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_msa 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 150 --timeout-method thread -k "min_sum or msa or split_syndrome or fused_syndrome"
ARGS="--algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1 --cpu-baseline 0"
for r in 1 2; do
  run meta1_$r 200 env LDPC_MSA_META=1 python bench.py $ARGS
  run meta0_$r 200 env LDPC_MSA_META=0 python bench.py $ARGS
done
run bench_msa 300 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1
exit 0
