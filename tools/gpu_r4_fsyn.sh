#!/bin/bash
# Round-4 A/B: compressed min-sum with the step's syndrome fused into the
# check kernel (default) against the separate k_syndrome_split launch
# (LDPC_MSA_SPLIT_SYN=1), config 5 at 1M codewords, alternating on one box;
# then the min-sum / coded / split-syndrome GPU tests on the fused default.
# (The fused build lost, 4.5 %, and is not in the tree: profiles/r4/README.md.)
set -o pipefail
out=gpurun_out/fsyn; mkdir -p $out
A="--algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --steps 2 --warmup 1 --cpu-baseline 0"
for r in 1 2 3; do
  for v in split fused; do
    if [ $v = split ]; then export LDPC_MSA_SPLIT_SYN=1; else unset LDPC_MSA_SPLIT_SYN; fi
    timeout -k 10 200 python bench.py $A > $out/$v$r.json 2> $out/$v$r.err || exit 1
    python -c "import json;d=json.load(open('$out/$v$r.json'));r=d['roofline'];c=d.get('check',{});print('$v', d['value'], r['frac'], r['avg_ms']['check'], r['avg_ms']['variable'], r['avg_ms'].get('syndrome'), c.get('mismatches'))"
  done
done
unset LDPC_MSA_SPLIT_SYN
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_coded_input.py -x -q --timeout 200 --timeout-method thread -k "msa or min_sum or coded or nonfinite or split_syndrome" > $out/pytest_fused.txt 2>&1; rc=$?
tail -3 $out/pytest_fused.txt
exit $rc
