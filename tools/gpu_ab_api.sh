#!/bin/bash
# Same-box A/B of library builds (ab_lib/libldpc_amd_<v>.so, VARIANTS) on the
# host-API DNA-batch call (tools/api_timing.py): alternating processes, each
# build swapped into the product path; the in-tree build restored at the end.
#   usage: VARIANTS="a b" [ROUNDS=3] tools/gpu_ab_api.sh <tag>
set -o pipefail
out=gpurun_out/${1:-abapi}
mkdir -p $out
lib=dna-ldpc-codes_amd/lib/libldpc_amd.so
cp $lib $out/keep.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-old new}; do
    cp ab_lib/libldpc_amd_$v.so $lib
    timeout -k 10 120 python tools/api_timing.py "$v:" > $out/$v$r.out 2> $out/$v$r.err || { cp $out/keep.so $lib; exit 1; }
    cat $out/$v$r.out
  done
done
cp $out/keep.so $lib
