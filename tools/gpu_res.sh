#!/bin/bash
# Resident-pool session: its GPU parity tests, then in-process A/B (fresh
# engines per round, rotated creation order) of the resident pool against
# the default schedule on the BP config 3 shape.
set -u
TAG=${1:-res}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "resident" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/ab_engines.py --algo bp --p 0.02 --batch 32768 --chunk 0 --fresh 4 \
  --var A: --var R3:LDPC_RES=1 --var R3NP:LDPC_RES=1,LDPC_C2V_PROBE=1 --var R2:LDPC_RES=1,LDPC_RES_TILES=2 \
  > "$OUT/ab_bp.txt" 2>&1
rc=$?; cat "$OUT/ab_bp.txt"; exit $rc
