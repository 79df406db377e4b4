#!/bin/bash
# Alternating bench A/B over environment settings on one box:
#   tools/gpu_ab_env.sh TAG "BENCH ARGS" "ENV_A" "ENV_B" [...]
# each setting runs twice, interleaved (A B C A B C); results in gpurun_out/TAG.
set -u
TAG=$1; ARGS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
for r in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    timeout -k 10 200 env $e python bench.py $ARGS --cpu-baseline 0 > "$OUT/v${i}_$r.out" 2> "$OUT/v${i}_$r.err"
    rc=$?; echo "v$i ($e) run $r rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/v${i}_$r.err"; exit $rc; fi
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['roofline']['avg_ms'])" "$OUT/v${i}_$r.out"
  done
done
exit 0
