#!/bin/bash
# Full GPU-box session: all GPU parity tests, smoke, the default bench
# (config 3), config 5 (min-sum 1M) and config 2 (DNA 272) bench lines, a
# rocprofv3 kernel-trace --stats profile of the default bench, and the HBM PMC
# passes (FETCH_SIZE / WRITE_SIZE / DRAM requests, one counter group per
# pass) for BP (config 3 shape) and compressed min-sum (BSC p=0.03, never
# converges).  Every GPU step has its own time limit; a fault / abort /
# timeout ends the session.
#   usage: tools/gpu_full.sh <tag> [skip_tests]
set -u
TAG=${1:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 1600 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if fatal $rc; then exit $rc; fi; }

if [ "${2:-}" != "skip_tests" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench_default 600 python bench.py
run bench_msa1m 600 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1
run bench_dna272 300 python bench.py --workload dna272
run trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0
rm -f "$OUT"/trace/*kernel_trace.csv
PB=${PMC_BATCH:-1024}
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu $PB
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu $PB
run pmc_dram 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum -d "$OUT/pmc_dram" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu $PB
run pmc_msa_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_msa_fetch" -o run --output-format csv -- python3 "$R/bench.py" --algo msa --p 0.03 --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu $PB
run pmc_msa_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_msa_write" -o run --output-format csv -- python3 "$R/bench.py" --algo msa --p 0.03 --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu $PB
exit 0
