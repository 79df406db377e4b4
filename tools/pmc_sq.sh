# SQ wave-state counters for the decode kernels (one rocprofv3 --pmc pass per
# counter group; no traces combined with --pmc).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_sq
mkdir -p $OUT
B=${PMC_BATCH:-4096}
run() {
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/p$1 -o run --output-format csv -- \
    python3 bench.py --batch-per-gpu $B --steps 1 --warmup 0 --cpu-baseline 0 --no-profile > $OUT/bench_$1.log 2>&1
}
run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
run SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR && \
run GRBM_GUI_ACTIVE SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum
