#!/bin/bash
# Round-4 profiling session: an 8-rank rehearsal of `bench.py --gpus 8` on the
# box's one GPU (small shards), then tools/gpu_prof.sh: rocprofv3 kernel-trace
# stats of the config-5 and config-3 bench and the PMC passes (16 384 codewords
# of config 5, 8 192 of config 3), then the config-5 EA / FETCH / WRITE passes
# again at 262 144 codewords (the pool's drain amortised).
#   usage: [REHEARSAL=0] tools/gpu_r4_prof.sh [tag] [msa|bp|both]
set -u
TAG=${1:-r4prof}
WHICH=${2:-both}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
if [ "${REHEARSAL:-1}" != 0 ]; then
timeout -k 10 300 python bench.py --gpus 8 --batch-per-gpu 2048 --steps 2 --warmup 1 --max-iter 50 \
  > "$OUT/gpus8_rehearsal.json" 2> "$OUT/gpus8_rehearsal.err" || { echo "rehearsal rc=$?"; tail -20 "$OUT/gpus8_rehearsal.err"; exit 1; }
echo "rehearsal ok"; tail -c 400 "$OUT/gpus8_rehearsal.json"; echo
fi
NOBENCH=1 bash tools/gpu_prof.sh "$TAG/prof" "" "$WHICH" || exit 1
[ "$WHICH" = bp ] && exit 0
B="python3 $R/bench.py --algo msa --p 0.002 --cpu-baseline 0 --secondary 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu 262144"
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  tagg=$(echo "$grp" | tr ' ' '+')
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/msa262k/pmc_$tagg" -o run --output-format csv -- $B \
    > "$OUT/msa262k_$tagg.out" 2> "$OUT/msa262k_$tagg.err" || { echo "pmc $tagg failed"; exit 1; }
done
echo done
