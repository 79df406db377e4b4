#!/bin/bash
# One column per variable wave with coded input (config 5, config 3) and the
# resident schedule for the DNA batch's host-API call with coded input.
set -u
TAG=${1:-r3probe2}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_engines.py --input code --algo msa --p 0.002 --batch 262144 --chunk 1024 \
  --var c2:var_cpw=2 --var c1:var_cpw=1 --reps 3 --profile 16 > $OUT/msa.out 2> $OUT/msa.err || exit 1
cat $OUT/msa.out | tail -2
timeout -k 10 300 python tools/ab_engines.py --input code --algo bp --p 0.02 --batch 32768 --chunk 0 \
  --var c2:var_cpw=2 --var c1:var_cpw=1 --reps 3 --profile 16 > $OUT/bp.out 2> $OUT/bp.err || exit 1
cat $OUT/bp.out | tail -2
timeout -k 10 300 python tools/api_timing.py default: res:resident=1 res2:resident=1,var_cpw=2 default2: \
  > $OUT/api.out 2> $OUT/api.err || exit 1
cat $OUT/api.out
exit 0
