#!/bin/bash
# Validation of the coded CPW-2 default: targeted parity tests, the default
# bench line, then the rocprofv3 traces and PMC passes of the new default
# instantiations (tools/gpu_r3_prof.sh with both workloads).
set -u
TAG=${1:-r3cpw2}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "coded or columns_per_wave or resident_pool or min_sum_compressed or dna_batch or split_syndrome or bench_secondary or config4"
run bench 400 python -u bench.py
NOBENCH=1 tools/gpu_r3_prof.sh "$TAG/prof" "" both || exit 1
exit 0
