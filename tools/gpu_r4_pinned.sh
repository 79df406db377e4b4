#!/bin/bash
# Round-4 session: the pinned-input host path (tests + the DNA batch's host legs).
set -o pipefail
out=gpurun_out/${1:-pinned}; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_coded_input.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for r in 1 2; do
  LDPC_API_TIMING=1 timeout -k 10 200 python bench.py --workload dna272 --steps 3 > $out/dna272_$r.json 2> $out/dna272_$r.err || exit 1
  python -c "import json;d=json.load(open('$out/dna272_$r.json'))['config'];print(d['ms_per_decode_device'], d['host_api_ms_median'], d['host_api_pinned_ms_median'], d['host_api_pinned_ms_min'], d['host_api_llr_ms_median'])"
done
