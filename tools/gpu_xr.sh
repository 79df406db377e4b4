#!/bin/bash
# XCD-resident decoder session: its parity tests, then a fresh-engine A/B
# against the resident pool (and the ping-pong schedule) on config 3 input.
#   usage: tools/gpu_xr.sh <tag> [extra ab_engines args]
set -u
TAG=${1:-xr}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_xr_gpu.py -x -v --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_engines.py --chunk 0 --fresh 3 --batch 16384 --var res: --var pp:LDPC_PINGPONG=1 \
  --var xr3:LDPC_XR=1,LDPC_XR_K=3 --var xr2:LDPC_XR=1,LDPC_XR_K=2 --var xr4:LDPC_XR=1,LDPC_XR_K=4 "$@" > "$OUT/ab.json" 2> "$OUT/ab.err"
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.json"; tail -3 "$OUT/ab.err"; exit $rc
