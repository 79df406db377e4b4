#!/bin/bash
# Measurement session: selected GPU tests, the default bench line
# (with its secondary legs), rocprofv3 kernel-trace stats of the config-5
# bench, and one PMC pass per counter group on a 16 384-codeword config-5
# decode (tools/pmc_summary.py summarises them).  Each step has its own limit.
#   usage: [AB="<ab_engines.py args>"] tools/gpu_prof.sh <tag> [pytest -k expression ("" = skip)] [msa|bp|both|none]
set -u
TAG=${1:-prof}
K=${2-"config4 or two_rank"}
WHICH=${3:-msa}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 300 "$OUT/$name.out"; echo; tail -3 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ -n "$K" ]; then
  run pytest 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" --durations=10
fi
if [ -z "${NOBENCH:-}" ]; then run bench_default 400 python bench.py; fi
if [ -n "${AB:-}" ]; then
  run ab 400 python -u tools/ab_engines.py $AB
fi
if [ "$WHICH" = msa ] || [ "$WHICH" = both ]; then
  run trace_msa 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_msa" -o run --output-format csv -- python3 "$R/bench.py" \
    --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1 --cpu-baseline 0 --secondary 0
  rm -f "$OUT"/trace_msa/*kernel_trace.csv
  B="python3 $R/bench.py --algo msa --p 0.002 --cpu-baseline 0 --secondary 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu ${MSA_B:-16384}"
  for grp in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
             "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    tagg=$(echo "$grp" | tr ' ' '+')
    run "msa_$tagg" 120 rocprofv3 --pmc $grp -d "$OUT/msa/pmc_$tagg" -o run --output-format csv -- $B
  done
fi
if [ "$WHICH" = bp ] || [ "$WHICH" = both ]; then
  run trace_bp 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_bp" -o run --output-format csv -- python3 "$R/bench.py" \
    --cpu-baseline 0 --secondary 0
  rm -f "$OUT"/trace_bp/*kernel_trace.csv
  B="python3 $R/bench.py --cpu-baseline 0 --secondary 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu ${BP_B:-8192}"
  for grp in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    tagg=$(echo "$grp" | tr ' ' '+')
    run "bp_$tagg" 120 rocprofv3 --pmc $grp -d "$OUT/bp/pmc_$tagg" -o run --output-format csv -- $B
  done
fi
exit 0
