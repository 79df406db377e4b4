#!/bin/bash
# Profile session: full default bench, rocprofv3 kernel-trace --stats, and the
# HBM PMC counters in separate passes (FETCH_SIZE, WRITE_SIZE).
#   usage: tools/gpu_profile.sh <tag> [extra bench args for the profiled runs]
set -u
TAG=${1:-r1}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 1500 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if fatal $rc; then exit $rc; fi; }

run bench_default 900 python bench.py
run trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 "$@"
# the per-dispatch trace (~190k rows) is too large to bring back; keep the stats
rm -f "$OUT"/trace/*kernel_trace.csv
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu ${PMC_BATCH:-1024}
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu ${PMC_BATCH:-1024}
run pmc_dram 600 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum -d "$OUT/pmc_dram" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu ${PMC_BATCH:-1024}
exit 0
