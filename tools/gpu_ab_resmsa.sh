#!/bin/bash
# Resident pool for compressed min-sum: GPU parity tests, then in-process A/B
# of pool sizes against the default 1024-lane MSA-C pool (config 5 input).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/resmsa${1:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "compressed or resident" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python tools/ab_engines.py --algo msa --p 0.002 --batch 131072 --reps 3 --chunk 0 --profile 50 \
  --var A: --var R2:LDPC_RES_MSA_C=1,LDPC_RES_TILES_MSA_C=2 --var R3:LDPC_RES_MSA_C=1,LDPC_RES_TILES_MSA_C=3 \
  --var R4:LDPC_RES_MSA_C=1,LDPC_RES_TILES_MSA_C=4 --var R8:LDPC_RES_MSA_C=1,LDPC_RES_TILES_MSA_C=8 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; exit $rc
