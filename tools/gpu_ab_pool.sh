#!/bin/bash
# Schedule choice for explicit pools: DNA batch bench (cap 320) and the host
# API's 4096-codeword chunks (config 3 input), grouped vs resident in-place.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/pool${1:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
for v in "X=0" "LDPC_RES=1"; do
  env $v timeout -k 10 120 python bench.py --workload dna272 --cpu-baseline 0 --steps 10 > "$OUT/dna.json" 2> "$OUT/dna.err" || exit 1
  echo "dna272 $v: $(python -c "import json;d=json.load(open('$OUT/dna.json'));print(d['value'],d['ms_per_step'],d['config']['host_api_ms_median'])")"
done
timeout -k 10 400 python tools/ab_engines.py --algo bp --p 0.02 --batch 32768 --reps 2 --chunk 4096 --profile 50 \
  --var G4096: --var R4096:LDPC_RES=1 > "$OUT/ab_bp.txt" 2>&1
rc=$?; cat "$OUT/ab_bp.txt"; exit $rc
