#!/bin/bash
# Round 5: k_var_msa_c at 8 waves per SIMD (amdgpu_waves_per_eu(8): 64 VGPRs,
# 78 SGPRs, 8 B of scratch) against the tree (7 waves: 96 SGPRs), config 5,
# same box, alternating; then the min-sum parity tests on the w8 build.
set -o pipefail
T=${1:-r5occ}; out=gpurun_out/$T; mkdir -p $out
ROUNDS=3 VARIANTS="base w8" timeout -k 10 500 bash tools/gpu_ab_lib.sh $T/c5 --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 || exit 1
