#!/bin/bash
# Round-4 probe of the compressed min-sum's schedule knobs with its v2c in
# column order (config 5, 1M codewords): columns per variable wave, tile
# group, lane pool.  Two alternating rounds, one bench line per setting.
set -o pipefail
out=gpurun_out/${1:-msaprobe}; mkdir -p $out
B="--algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 --cpu-baseline 0"
i=0
for r in 1 2; do
  for v in "" "--var-cpw 4" "--var-cpw 1" "--group-tiles 8" "--chunk 2048" "--chunk 2048 --group-tiles 8"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py $B $v > $out/p$i.json 2> $out/p$i.err || exit 1
    python -c "import json;d=json.load(open('$out/p$i.json'));r=d['roofline'];c=d['config'];print('[$v]', d['value'], c['resident_per_pass'], c['group_tiles'], r['kernels']['variable'], r['avg_ms']['check'], r['avg_ms']['variable'], r['avg_ms']['syndrome'], d['check']['mismatches'])"
  done
done
