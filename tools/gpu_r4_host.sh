#!/bin/bash
# Round-4 A/B of the host leg of the DNA batch (config 2): library builds
# ab_lib/libldpc_amd_<v>.so swapped into the product path, alternating
# `bench.py --workload dna272` runs with the host-leg split printed
# (LDPC_API_TIMING=1); the in-tree library is restored at the end.
#   usage: [VARIANTS="a b"] [ROUNDS=3] tools/gpu_r4_host.sh <tag>
set -o pipefail
out=gpurun_out/${1:-host}; mkdir -p $out
lib=dna-ldpc-codes_amd/lib/libldpc_amd.so
cp $lib $out/keep.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-pieces slices}; do
    cp ab_lib/libldpc_amd_$v.so $lib
    LDPC_API_TIMING=1 timeout -k 10 200 python bench.py --workload dna272 --steps 3 > $out/$v$r.json 2> $out/$v$r.err || { cp $out/keep.so $lib; exit 1; }
    python -c "import json;d=json.load(open('$out/$v$r.json'))['config'];print('$v', d['ms_per_decode_device'], d['host_api_ms_median'], d['host_api_ms_min'], d['host_api_llr_ms_median'], d['host_api_llr_ms_min'])"
  done
done
cp $out/keep.so $lib
