#!/bin/bash
# Round-2 evidence on HEAD: default bench line, rocprofv3 kernel-trace stats
# of the same command, config 5 and DNA-batch lines.  Each step has its own
# limit and writes to gpurun_out/<tag>/; a failing step ends the session.
set -u
TAG=${1:-r2final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 600 "$OUT/$name.out"; echo; tail -2 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench_default 300 python bench.py
run rocprof_default 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py
run bench_msa 400 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1
run bench_dna272 200 python bench.py --workload dna272
exit 0
