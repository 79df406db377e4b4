#!/bin/bash
# Resident pool with one stream per pool tile: parity tests, a fresh-rotation
# A/B of the stream modes (BP config 3 input), then bench.py per mode.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/tstreams${1:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "tile_streams" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/ab_engines.py --algo bp --p 0.02 --batch 32768 --chunk 0 --fresh 4 \
  --var S0:LDPC_RES_STREAMS=0 --var TS1:LDPC_RES_STREAMS=1 --var TS4:LDPC_RES_STREAMS=4 > "$OUT/ab.txt" 2>&1
rc=$?; tail -3 "$OUT/ab.txt"; [ $rc -ne 0 ] && exit $rc
for m in 0 1 4; do
  LDPC_RES_STREAMS=$m timeout -k 10 200 python bench.py --cpu-baseline 0 > "$OUT/bench$m.json" 2> "$OUT/bench$m.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/bench$m.json'));print('bench streams=$m', d['value'], d['roofline']['frac'])"
done
