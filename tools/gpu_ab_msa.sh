#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/abmsa; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_engines.py --algo msa --p 0.002 --batch 131072 --reps 3 --profile 50 \
  --var A: --var B:LDPC_FULL_LANES=5 --var C:LDPC_GROUP_TILES=4 --var D:LDPC_VAR_CPW=2 --var E:LDPC_MSA_C=0 > "$OUT/ab_p002.txt" 2>&1
rc=$?; cat "$OUT/ab_p002.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_engines.py --algo msa --p 0.03 --max-iter 20 --batch 32768 --reps 2 --profile 50 \
  --var A: --var E:LDPC_MSA_C=0 > "$OUT/ab_p03.txt" 2>&1
rc=$?; cat "$OUT/ab_p03.txt"; exit $rc
