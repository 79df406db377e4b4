#!/bin/bash
# Process-to-process spread of the default bench (same library), then the
# in-process placement diagnostic at the bench's batch size.
set -o pipefail
out=gpurun_out/${1:-spread}
mkdir -p $out
for r in 1 2 3 4; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 > $out/b$r.json 2> $out/b$r.err || exit 1
  python -c "import json;d=json.load(open('$out/b$r.json'));r=d['roofline'];print('bench', d['value'], r['avg_ms']['check'], r['avg_ms']['variable'])"
done
timeout -k 10 300 python tools/placement_diag.py 4 100000 || exit 1
