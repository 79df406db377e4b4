#!/bin/bash
# Round-4 A/B: the compressed min-sum's v2c in CSC order (-DLDPC_MSA_CSC=1,
# ab_lib/libldpc_amd_new.so) against CSR order (ab_lib/libldpc_amd_old.so) on
# config 5, then the min-sum parity tests on the CSC build.
set -o pipefail
out=gpurun_out/csc; mkdir -p $out
ROUNDS=2 VARIANTS="old new" bash tools/gpu_ab_lib.sh csc --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
lib=dna-ldpc-codes_amd/lib/libldpc_amd.so
cp $lib $out/keep2.so
cp ab_lib/libldpc_amd_new.so $lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_coded_input.py tests/test_int_decoders.py -x -q --timeout 200 --timeout-method thread -k "msa or min_sum or coded or nonfinite" > $out/pytest_new.txt 2>&1; rc=$?
cp $out/keep2.so $lib
tail -3 $out/pytest_new.txt
exit $rc
