#!/bin/bash
# Host-API DNA-batch timeline: the host-leg split (LDPC_API_TIMING=1) and a
# rocprofv3 kernel + memory-copy trace of the same calls (tools/trace_decode.py).
set -u
TAG=${1:-r3api}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -n 8 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
LDPC_API_TIMING=1 run api_timing 200 python tools/api_timing.py default:
run api_trace 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/api_trace" -o run --output-format csv -- python3 tools/api_timing.py default:
exit 0
