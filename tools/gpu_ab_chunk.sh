#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/abchunk3; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
for ch in 1024 16384; do
  timeout -k 10 200 python tools/ab_engines.py --algo msa --p 0.03 --max-iter 20 --batch 32768 --reps 1 --chunk $ch --profile 7 \
    --var G4:LDPC_GROUP_TILES=4 --var F64:LDPC_MSA_C=0 > "$OUT/msa_$ch.txt" 2>&1
  rc=$?; echo "chunk $ch"; grep -E "median|kernels" "$OUT/msa_$ch.txt"; [ $rc -ne 0 ] && exit $rc
done
exit 0
