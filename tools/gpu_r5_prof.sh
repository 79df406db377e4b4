#!/bin/bash
# Round-5 profiling session:
#   1. an 8-rank rehearsal of `bench.py --gpus 8` on the box's one GPU (small
#      shards; the N > 1 line's cpu_baseline and a forced 16 384-codeword
#      config-4 leg);
#   2. PMC passes (TCC_EA0_RDREQ/WRREQ, FETCH_SIZE, WRITE_SIZE) of config 3
#      (8 192 codewords, resident pool), of the headline's kernels streaming
#      from HBM (16 384 codewords in one grouped pass) and of config 5
#      (262 144 codewords), each its own rocprofv3 run;
#   3. rocprofv3 kernel-trace stats of the HBM-streaming run.
# tools/pmc_summary.py turns each PMC directory into per-kernel bytes.
#   usage: tools/gpu_r5_prof.sh [tag]
set -u
TAG=${1:-r5prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 8 --batch-per-gpu 2048 --steps 2 --warmup 1 --config4 16384 --cpu-seconds 4 \
  > "$OUT/gpus8_rehearsal.json" 2> "$OUT/gpus8_rehearsal.err" || { echo "rehearsal rc=$?"; tail -20 "$OUT/gpus8_rehearsal.err"; exit 1; }
echo "rehearsal ok"; tail -c 300 "$OUT/gpus8_rehearsal.json"; echo
pmc() {  # pmc <name> <bench args...>
  local name=$1; shift
  local B="python3 $R/bench.py --cpu-baseline 0 --secondary 0 --no-profile --steps 1 --warmup 0 $*"
  for grp in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    local tagg=$(echo "$grp" | tr ' ' '+')
    timeout -s KILL 150 rocprofv3 --pmc $grp -d "$OUT/$name/pmc_$tagg" -o run --output-format csv -- $B \
      > "$OUT/${name}_$tagg.out" 2> "$OUT/${name}_$tagg.err" || { echo "pmc $name $tagg failed"; exit 1; }
  done
  echo "pmc $name ok"
}
pmc bp8192 --batch-per-gpu 8192
pmc hbm16k --batch-per-gpu 16384 --chunk 16384 --res 0 --group-tiles -1
pmc msa262k --algo msa --p 0.002 --batch-per-gpu 262144
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_hbm16k" -o run --output-format csv -- python3 "$R/bench.py" \
  --batch-per-gpu 16384 --chunk 16384 --res 0 --group-tiles -1 --cpu-baseline 0 --secondary 0 --steps 3 --warmup 1 \
  > "$OUT/trace_hbm16k.out" 2> "$OUT/trace_hbm16k.err" || { echo "trace failed"; exit 1; }
rm -f "$OUT"/trace_hbm16k/*kernel_trace.csv
echo done
