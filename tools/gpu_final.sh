#!/bin/bash
# End-of-round GPU session: full parity suite + smoke, the default bench,
# rocprofv3 trace stats and HBM PMC passes of the same command, the config 5
# and DNA-batch bench lines, and a 2-rank rehearsal of the multi-GPU bench
# path (both ranks on the box's one GPU).
set -u
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 1200 "$OUT/$name.out"; tail -2 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest 800 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 600 python bench.py
run trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0
rm -f "$OUT"/trace/*kernel_trace.csv
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu 1024
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu 1024
run bench_msa 400 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1
run bench_dna272 200 python bench.py --workload dna272
run bench_2rank 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch-per-gpu 8192
exit 0
