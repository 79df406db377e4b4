#!/bin/bash
# Multi-block continuous-mode syndrome: GPU parity tests, then in-process A/B
# against the one-block-per-tile syndrome (min-sum config 5 input).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/synsplit${1:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "split_syndrome or fused_syndrome or resident or compressed or device_resident" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/ab_engines.py --algo msa --p 0.002 --batch 131072 --reps 3 --chunk 0 --profile 50 \
  --var A: --var S32:LDPC_SYN_SPLIT=32 --var S64:LDPC_SYN_SPLIT=64 --var S128:LDPC_SYN_SPLIT=128 \
  --var S64P512:LDPC_SYN_SPLIT=64,LDPC_MSA_POOL=512 > "$OUT/ab_msa.txt" 2>&1
rc=$?; cat "$OUT/ab_msa.txt"; exit $rc
