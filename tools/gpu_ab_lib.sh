#!/bin/bash
# Same-box A/B of two library builds (ab_lib/libldpc_amd_{old,new}.so):
# alternating default bench runs, each library swapped into the product path.
set -o pipefail
out=gpurun_out/${1:-ablib}
shift
mkdir -p $out
lib=dna-ldpc-codes_amd/lib/libldpc_amd.so
cp $lib $out/keep.so
for r in 1 2 3; do
  for v in old new; do
    cp ab_lib/libldpc_amd_$v.so $lib
    timeout -k 10 200 python bench.py --cpu-baseline 0 "$@" > $out/$v$r.json 2> $out/$v$r.err || { cp $out/keep.so $lib; exit 1; }
    python -c "import json;d=json.load(open('$out/$v$r.json'));r=d['roofline'];print('$v', d['value'], r['frac'], r['avg_ms']['check'], r['avg_ms']['variable'], r['avg_ms']['syndrome'])"
  done
done
cp $out/keep.so $lib
