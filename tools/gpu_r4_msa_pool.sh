#!/bin/bash
# Round-4 probe: compressed min-sum with a lane pool small enough for its
# column-ordered v2c to stay in the 256 MB Infinity Cache (2-4 tiles, one
# group per step) against the default 1024-lane pool in groups of 8.
set -o pipefail
out=gpurun_out/${1:-msapool}; mkdir -p $out
B="--algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 --cpu-baseline 0"
i=0
for r in 1 2; do
  for v in "" "--chunk 192 --group-tiles 3" "--chunk 128 --group-tiles 2" "--chunk 256 --group-tiles 4" "--chunk 384 --group-tiles 3"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py $B $v > $out/p$i.json 2> $out/p$i.err || exit 1
    python -c "import json;d=json.load(open('$out/p$i.json'));r=d['roofline'];c=d['config'];print('[$v]', d['value'], c['resident_per_pass'], c['group_tiles'], r['avg_ms']['check'], r['avg_ms']['variable'], r['avg_ms']['syndrome'], r['launches']['check'], d['check']['mismatches'])"
  done
done
