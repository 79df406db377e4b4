#!/bin/bash
# Round 6 diagnosis of the ASan build on the GPU: ASan runtime options.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r6abi4; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
P=tests/golden/decode_n18432_m2048_final.pchk
export LSAN_OPTIONS=suppressions=$R/tests/asan/lsan.supp
for opt in detect_stack_use_after_return=0 protect_shadow_gap=0 "detect_stack_use_after_return=0:protect_shadow_gap=0"; do
  mkdir -p /tmp/a_$$; ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:$opt timeout -k 10 200 tests/asan/build/abi_check $P /tmp/a_$$ > "$OUT/o.log" 2>&1; echo "== $opt rc=$?"; grep -v "^$" "$OUT/o.log" | grep -v "Suppress\|count\|libhsa\|----" | head -6
done
exit 0
