#!/bin/bash
# Full GPU parity suite (verbose log under gpurun_out/<tag>/), then optional
# extra commands; stops at the first failure.
set -o pipefail
tag=${1:-check}
shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -4 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
for cmd in "$@"; do
    echo "== $cmd"
    eval "$cmd" || exit $?
done
