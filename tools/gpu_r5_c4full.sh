#!/bin/bash
# Round 5: the N = 8 line's config-4 leg at its full size (1 000 000 codewords,
# 125 000 per rank) rehearsed with 8 ranks on the box's one GPU.
set -o pipefail
T=${1:-r5c4}; out=gpurun_out/$T; mkdir -p $out
timeout -k 10 900 python -u bench.py --gpus 8 --batch-per-gpu 2048 --steps 1 --warmup 0 --config4 1000000 --cpu-seconds 4 \
  > $out/gpus8_config4_1m.json 2> $out/gpus8_config4_1m.err; rc=$?
tail -c 400 $out/gpus8_config4_1m.json; tail -3 $out/gpus8_config4_1m.err
exit $rc
