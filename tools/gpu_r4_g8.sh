#!/bin/bash
# Round-4 session: write/read shape ceilings for the compressed min-sum's
# column-ordered v2c (tools/wrbench at the 4- and 8-tile group sizes), the
# min-sum parity tests with groups of 8 tiles, and the default bench line.
set -o pipefail
out=gpurun_out/${1:-g8}; mkdir -p $out
for mb in 302 604; do timeout -k 10 120 tools/wrbench $mb > $out/wrbench_${mb}MB.txt 2>&1 || exit 1; done
cat $out/wrbench_604MB.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_coded_input.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread -k "msa or min_sum or coded or nonfinite or config5" > $out/pytest_msa.txt 2>&1 || { tail -20 $out/pytest_msa.txt; exit 1; }
tail -2 $out/pytest_msa.txt
timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 1
python -c "import json;d=json.load(open('$out/bench_default.json'));s=d['secondary'];m=s['config5_msa_1m'];print(d['value'], m['value'], m['group_tiles'], m['roofline']['avg_ms'], s['config2_dna272']['host_api_ms_median'])"
