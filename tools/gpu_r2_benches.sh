#!/bin/bash
# Bench lines on HEAD (default config 3, config 5, DNA batch) and the default
# bench under rocprofv3 kernel-trace stats; the per-dispatch trace CSV is
# deleted on the box (only the stats travel back, gpurun_out/ is capped).
set -u
TAG=${1:-r2benches}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 300 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench_default 300 python bench.py
run bench_msa 400 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1
run bench_dna272 200 python bench.py --workload dna272
run bench_rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py
rm -f "$OUT"/prof/*kernel_trace.csv
exit 0
