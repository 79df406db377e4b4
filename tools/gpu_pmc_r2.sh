#!/bin/bash
# Round-2 roofline evidence: rocprofv3 kernel-trace stats of the default
# bench, then PMC passes (one counter group per pass) on
#   - a known-bytes calibration (tools/cachebench calib: the check kernel's
#     access shape, in place, over 2048 MB and 64 MB),
#   - bench.py at a bench-representative size (8192 codewords of config 3
#     through the same 3-tile resident pool as the 100k bench),
# counting fabric requests (FETCH_SIZE / WRITE_SIZE, TCC_EA0_*REQ) and the
# DRAM share of them (TCC_EA0_*REQ_DRAM).
#   usage: tools/gpu_pmc_r2.sh <tag>
set -u
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -s KILL "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 600 "$OUT/$name.out"; tail -2 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0
rm -f "$OUT"/trace/*kernel_trace.csv
B="python3 $R/bench.py --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu 8192"
C="$R/tools/cachebench calib"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum"; do
  tagg=$(echo "$grp" | tr ' ' '+')
  run "calib_$tagg" 60 rocprofv3 --pmc $grp -d "$OUT/calib/pmc_$tagg" -o run --output-format csv -- $C
  run "bench_$tagg" 120 rocprofv3 --pmc $grp -d "$OUT/bench/pmc_$tagg" -o run --output-format csv -- $B
done
exit 0
