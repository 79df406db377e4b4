#!/bin/bash
# Kernel trace of the DNA-batch bench (config 2): per-launch durations and the
# gaps between them inside one 272-codeword decode.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-dna_trace}
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- \
    python3 bench.py --workload dna272 --steps 10 --warmup 2 > $out/bench.out 2> $out/bench.err
rc=$?
echo "trace rc=$rc"
tail -3 $out/bench.out
exit $rc
