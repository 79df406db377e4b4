#!/bin/bash
# Round 6 diagnosis: bisect the ASan-build failure by translation unit
#   vC = ASan on capi.cpp only; vD = ASan on engine.hip only (all -O3 -g)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r6abi5; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
P=tests/golden/decode_n18432_m2048_final.pchk
for v in ${VARIANTS:-vC vD}; do
  mkdir -p /tmp/a_$v; ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 timeout -k 10 200 tests/asan/build/$v/abi_check $P /tmp/a_$v > "$OUT/$v.log" 2>&1; echo "== $v rc=$?"; grep -v "^$" "$OUT/$v.log" | head -8
done
exit 0
