#!/bin/bash
# Session-2 measurements: same-box A/B of two library builds on config 5
# (ab_lib/libldpc_amd_{old,new}.so), then the DNA batch's host-API split per
# host-thread count with the coded path (LDPC_API_TIMING=1).
set -u
TAG=${1:-r3s2}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
VARIANTS="old new" ROUNDS=3 tools/gpu_ab_lib.sh $TAG/ab --algo msa --p 0.002 --batch-per-gpu 262144 --secondary 0 --steps 2 --warmup 1 || exit 1
LDPC_API_TIMING=1 timeout -k 10 200 python tools/api_timing.py default: t8:host_threads=8 t12:host_threads=12 t24:host_threads=24 default2: > $OUT/api.out 2> $OUT/api.err || exit 1
cat $OUT/api.out
exit 0
