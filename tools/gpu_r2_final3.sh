#!/bin/bash
# End-of-round validation on HEAD: tools/gpu_r2_final.sh (whole -m gpu suite,
# smoke, default / config 5 / DNA batch bench lines), then the default bench
# under rocprofv3 kernel-trace stats.  A failing step ends the session.
set -u
TAG=${1:-r2final3}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
bash tools/gpu_r2_final.sh "$TAG" || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py > "$OUT/bench_rocprof.out" 2> "$OUT/bench_rocprof.err"
rc=$?; echo "bench_rocprof rc=$rc"; tail -c 600 "$OUT/bench_rocprof.out"; tail -3 "$OUT/bench_rocprof.err"
rm -f "$OUT"/prof/*kernel_trace.csv  # per-dispatch trace: too large for gpurun_out (64 MiB)
exit $rc
