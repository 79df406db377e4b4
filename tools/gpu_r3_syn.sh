#!/bin/bash
# Syndrome blocks per tile (ldpc_schedule.syn_blocks) for config 5 (1024-lane
# pool, 16 tiles) and for the DNA batch's host-API call (5 tiles).
set -u
TAG=${1:-r3syn2}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_engines.py --algo msa --p 0.002 --batch 262144 --chunk 1024 --var s16:syn_blocks=16 \
  --var s8:syn_blocks=8 --var s12:syn_blocks=12 --var s24:syn_blocks=24 --var s32:syn_blocks=32 --reps 4 --profile 16 \
  > $OUT/ab.out 2> $OUT/ab.err || exit 1
cat $OUT/ab.out
timeout -k 10 200 python tools/api_timing.py s32:syn_blocks=32 s16:syn_blocks=16 s64:syn_blocks=64 s8:syn_blocks=8 s32b:syn_blocks=32 \
  > $OUT/api.out 2> $OUT/api.err || exit 1
cat $OUT/api.out
exit 0
