#!/bin/bash
# L2 request counters per decode kernel, min-sum (compressed records) vs BP,
# on non-converging inputs (every codeword runs max_iter = 50): TCC hits /
# misses and TCP->TCC read / write requests, one rocprofv3 --pmc pass each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${1:-l2req}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
pass() {
  local name=$1 algo=$2 p=$3; shift 3
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$R/bench.py" \
    --algo $algo --p $p --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu 1024 \
    > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass msa_tcc msa 0.03 TCC_HIT_sum TCC_MISS_sum
pass msa_tcp msa 0.03 TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
pass bp_tcc bp 0.02 TCC_HIT_sum TCC_MISS_sum
pass bp_tcp bp 0.02 TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
exit 0
