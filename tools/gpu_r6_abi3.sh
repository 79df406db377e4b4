#!/bin/bash
# Round 6 diagnosis: does the sanitized build fail because ASan fills fresh
# heap memory (malloc_fill_byte) -- i.e. does the library read uninitialized
# host heap memory?  plain + MALLOC_PERTURB_ (glibc fills new allocations),
# and the ASan build with its malloc fill turned off.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r6abi3; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
P=tests/golden/decode_n18432_m2048_final.pchk
mkdir -p /tmp/a1 /tmp/a2
MALLOC_PERTURB_=165 timeout -k 10 120 tests/asan/build/abi_check_plain $P /tmp/a1 > "$OUT/plain_perturb.log" 2>&1; echo "plain+perturb rc=$?"; head -20 "$OUT/plain_perturb.log"
LSAN_OPTIONS=suppressions=$R/tests/asan/lsan.supp ASAN_OPTIONS=detect_leaks=1:halt_on_error=1:max_malloc_fill_size=0 timeout -k 10 200 tests/asan/build/abi_check $P /tmp/a2 > "$OUT/asan_nofill.log" 2>&1; echo "asan nofill rc=$?"; grep -v "^$" "$OUT/asan_nofill.log" | head -20
exit 0
