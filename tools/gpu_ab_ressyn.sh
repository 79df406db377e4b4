#!/bin/bash
# Resident pool: fused vs separate multi-block syndrome (BP config 3 input).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/ressyn${1:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "resident_pool_split" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python tools/ab_engines.py --algo bp --p 0.02 --batch 32768 --reps 3 --chunk 0 --profile 50 \
  --var F: --var S16:LDPC_RES_SYN=16 --var S32:LDPC_RES_SYN=32 --var S96:LDPC_RES_SYN=96 > "$OUT/ab_bp.txt" 2>&1
rc=$?; cat "$OUT/ab_bp.txt"; exit $rc
