#!/bin/bash
# Min-sum session: MSA GPU parity tests, then config 5 (1M codewords, BSC
# p=0.002, early exit) with compressed c2v (default) and the fp64 c2v path.
set -u
TAG=${1:-msa}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "min_sum or grouped or nan or variable_columns or continuous or extreme" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1 --cpu-baseline 0 > "$OUT/bench_msa_c.json" 2> "$OUT/bench_msa_c.err"
rc=$?; echo "bench msa_c rc=$rc"; cat "$OUT/bench_msa_c.json"; tail -3 "$OUT/bench_msa_c.err"
if fatal $rc; then exit $rc; fi
LDPC_MSA_C=0 timeout -k 10 300 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 1 --cpu-baseline 0 > "$OUT/bench_msa_fp64.json" 2> "$OUT/bench_msa_fp64.err"
rc=$?; echo "bench msa fp64 rc=$rc"; cat "$OUT/bench_msa_fp64.json"; tail -3 "$OUT/bench_msa_fp64.err"
exit $rc
