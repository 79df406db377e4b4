#!/bin/bash
# Round-4 A/B: the compressed min-sum's v2c row-block-major (edge s of column
# j at s * N + j, ab_lib/libldpc_amd_rb.so) against plain column order (j * 8
# + s, ab_lib/libldpc_amd_csc.so), config 5, then the min-sum tests on rb.
set -o pipefail
out=gpurun_out/rb; mkdir -p $out
ROUNDS=3 VARIANTS="csc rb" bash tools/gpu_ab_lib.sh rb --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
lib=dna-ldpc-codes_amd/lib/libldpc_amd.so
cp $lib $out/keep2.so
cp ab_lib/libldpc_amd_rb.so $lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_coded_input.py -x -q --timeout 200 --timeout-method thread -k "msa or min_sum or coded or nonfinite" > $out/pytest_rb.txt 2>&1; rc=$?
cp $out/keep2.so $lib
tail -3 $out/pytest_rb.txt
exit $rc
