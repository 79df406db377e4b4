#!/bin/bash
# Resident pool with one stream per pool tile: parity tests, then a
# fresh-rotation A/B against the single-stream pool (BP config 3 input).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/tstreams${1:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "tile_streams or resident_pool_in_place" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/ab_engines.py --algo bp --p 0.02 --batch 32768 --chunk 0 --fresh 6 \
  --var S1: --var TS2:LDPC_RES_STREAMS=2 --var TS3:LDPC_RES_STREAMS=3 --var TS1:LDPC_RES_STREAMS=1 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; exit $rc
