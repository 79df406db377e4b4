#!/bin/bash
# Round-3 micro-measurements: v2c write/read shapes (tools/wrbench) and the
# host-leg split of the DNA batch through ldpc_decode (LDPC_API_TIMING=1).
set -u
TAG=${1:-r3micro}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -n 20 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run wrbench_1208 120 tools/wrbench 1208
run wrbench_302 120 tools/wrbench 302
LDPC_API_TIMING=1 run api_timing 200 python tools/api_timing.py default: t8:host_threads=8 t4:host_threads=4
exit 0
