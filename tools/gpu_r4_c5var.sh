#!/bin/bash
# Round-4 check: config 5 standalone vs as bench.py's secondary leg (after the
# headline's engines were freed), on the same box, twice each.
set -o pipefail
out=gpurun_out/${1:-c5var}; mkdir -p $out
for r in 1 2; do
  timeout -k 10 200 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 --cpu-baseline 0 > $out/alone$r.json 2> $out/alone$r.err || exit 1
  python -c "import json;d=json.load(open('$out/alone$r.json'));r=d['roofline'];print('alone', d['value'], r['avg_ms']['check'], r['avg_ms']['variable'])"
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 2 > $out/leg$r.json 2> $out/leg$r.err || exit 1
  python -c "import json;d=json.load(open('$out/leg$r.json'));m=d['secondary']['config5_msa_1m'];r=m['roofline'];print('leg', m['value'], r['avg_ms']['check'], r['avg_ms']['variable'])"
done
