#!/bin/bash
# Columns per variable wave, tile groups and pool size with coded input
# (tools/ab_engines.py --input code): config 5 (min-sum, 1024-lane pool) and
# config 3 (BP resident pool).
set -u
TAG=${1:-r3cpw}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_engines.py --input code --algo msa --p 0.002 --batch 262144 --chunk 1024 \
  --var c4:var_cpw=4 --var c3:var_cpw=3 --var c2:var_cpw=2 --var g8:group_tiles=8 --var p2048:chunk=2048 --reps 3 --profile 16 \
  > $OUT/msa.out 2> $OUT/msa.err || exit 1
cat $OUT/msa.out
timeout -k 10 400 python tools/ab_engines.py --input code --algo bp --p 0.02 --batch 32768 --chunk 0 \
  --var c4:var_cpw=4 --var c2:var_cpw=2 --var c8:var_cpw=8 --reps 3 --profile 16 > $OUT/bp.out 2> $OUT/bp.err || exit 1
cat $OUT/bp.out
exit 0
