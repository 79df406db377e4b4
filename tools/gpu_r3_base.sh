#!/bin/bash
# Round-3 baseline of the min-sum (config 5) kernels before any change:
# host CPU share, rocprofv3 kernel-trace stats of the config-5 bench, and
# one PMC pass per counter group on a 16 384-codeword config-5 decode.
#   usage: tools/gpu_r3_base.sh <tag>
set -u
TAG=${1:-r3base}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -s KILL "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 400 "$OUT/$name.out"; echo; tail -2 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
{
  echo "nproc $(nproc)"
  python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'
  cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cgroup v2 cpu.max"
  cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us 2>/dev/null || true
} > "$OUT/host.txt" 2>&1
cat "$OUT/host.txt"
run trace_msa 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_msa" -o run --output-format csv -- python3 "$R/bench.py" \
  --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1 --cpu-baseline 0
rm -f "$OUT"/trace_msa/*kernel_trace.csv
B="python3 $R/bench.py --algo msa --p 0.002 --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu 16384"
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  tagg=$(echo "$grp" | tr ' ' '+')
  run "msa_$tagg" 120 rocprofv3 --pmc $grp -d "$OUT/msa/pmc_$tagg" -o run --output-format csv -- $B
done
exit 0
