#!/bin/bash
# 32-bit meta MSA-C (edge id of min1): the min-sum parity tests, then the config-5 A/B over
# meta on / off and columns per wave (tools/gpu_ab_env.sh).
set -u
TAG=${1:-meta32}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 150 --timeout-method thread \
  -k "min_sum or msa or split_syndrome or fused_syndrome" > "$OUT/pytest.out" 2> "$OUT/pytest.err"
rc=$?; tail -3 "$OUT/pytest.out"; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "$OUT/pytest.out" | head -20; exit $rc; fi
bash tools/gpu_ab_env.sh "$TAG/ab" "--algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1" \
  "LDPC_MSA_META=1" "LDPC_MSA_META=0"
