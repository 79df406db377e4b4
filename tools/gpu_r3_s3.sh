#!/bin/bash
# Pool / group size probes with the coded kernels: config 3 at resident pools
# of 2, 3 (default) and 4 tiles; the DNA batch's host-API call with tile
# groups of 1-5.
set -u
TAG=${1:-r3s3}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
for r in 1 2; do
  for c in 0 128 256; do
    timeout -k 10 200 python bench.py --cpu-baseline 0 --secondary 0 --chunk $c > $OUT/bp_chunk$c.$r.json 2> $OUT/bp_chunk$c.$r.err || exit 1
    python -c "import json;d=json.load(open('$OUT/bp_chunk$c.$r.json'));r=d['roofline'];print('chunk $c', d['value'], d['config']['resident_per_pass'], r['avg_ms']['check'], r['avg_ms']['variable'])"
  done
done
timeout -k 10 200 python tools/api_timing.py default: g1:group_tiles=1 g2:group_tiles=2 g4:group_tiles=4 g5:group_tiles=5 default2: > $OUT/api.out 2> $OUT/api.err || exit 1
cat $OUT/api.out
exit 0
