#!/bin/bash
# Same-box A/B of library builds ab_lib/libldpc_amd_<variant>.so (VARIANTS,
# default "old new"): alternating bench runs, each library swapped into the
# product path; the in-tree library is restored at the end.
#   usage: [VARIANTS="a b c"] [ROUNDS=3] tools/gpu_ab_lib.sh <tag> [bench.py args]
set -o pipefail
out=gpurun_out/${1:-ablib}
shift
mkdir -p $out
lib=dna-ldpc-codes_amd/lib/libldpc_amd.so
cp $lib $out/keep.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-old new}; do
    cp ab_lib/libldpc_amd_$v.so $lib
    timeout -k 10 200 python bench.py --cpu-baseline 0 "$@" > $out/$v$r.json 2> $out/$v$r.err; brc=$?
    if [ $brc -ne 0 ] && { [ -z "${ABIGNORE:-}" ] || [ ! -s $out/$v$r.json ]; }; then cp $out/keep.so $lib; exit 1; fi
    python -c "import json;d=json.load(open('$out/$v$r.json'));r=d['roofline'];print('$v', d['value'], r['frac'], r['avg_ms']['check'], r['avg_ms']['variable'], r['avg_ms']['syndrome'])"
  done
done
cp $out/keep.so $lib
