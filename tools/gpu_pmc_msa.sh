#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes for the min-sum kernels on a non-converging
# workload (BSC p=0.03: every codeword runs max_iter = 50), so executed
# codeword-iterations are exactly batch x 50.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r1msa}
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- python3 "$R/bench.py" \
    --algo msa --p 0.03 --cpu-baseline 0 --no-profile --steps 1 --warmup 0 --batch-per-gpu ${PMC_BATCH:-1024} \
    > "$OUT/pmc_$c.out" 2> "$OUT/pmc_$c.err" || exit $?
done
