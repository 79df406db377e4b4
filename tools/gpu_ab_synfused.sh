#!/bin/bash
# Fused syndrome in the grouped continuous schedule: GPU parity tests, then
# in-process A/B against the defaults (min-sum config 5 input, BP config 3).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/synf${1:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fused_syndrome" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/ab_engines.py --algo msa --p 0.002 --batch 131072 --reps 3 --chunk 0 --profile 50 \
  --var A: --var F:LDPC_SYN_FUSED=1 --var F2k:LDPC_SYN_FUSED=1,LDPC_MSA_POOL=2048 \
  --var F512:LDPC_SYN_FUSED=1,LDPC_MSA_POOL=512 > "$OUT/ab_msa.txt" 2>&1
rc=$?; cat "$OUT/ab_msa.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/ab_engines.py --algo bp --p 0.02 --batch 32768 --reps 3 --chunk 0 --profile 50 \
  --var RES: --var G:LDPC_RES=0 --var GF:LDPC_RES=0,LDPC_SYN_FUSED=1 > "$OUT/ab_bp.txt" 2>&1
rc=$?; cat "$OUT/ab_bp.txt"; exit $rc
