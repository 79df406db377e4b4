#!/bin/bash
# Round 6 diagnosis: which build difference breaks the sanitized library on the GPU.
#   vA = host ASan + UBSan, -O3 everywhere;  vB = no sanitizer, -O1 everywhere
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r6abi2; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
P=tests/golden/decode_n18432_m2048_final.pchk
mkdir -p /tmp/a1 /tmp/a2
LSAN_OPTIONS=suppressions=$R/tests/asan/lsan.supp ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 timeout -k 10 200 tests/asan/build/vA/abi_check $P /tmp/a1 > "$OUT/vA.log" 2>&1; echo "vA rc=$?"; grep -v "^$" "$OUT/vA.log" | head -20
timeout -k 10 120 tests/asan/build/vB/abi_check $P /tmp/a2 > "$OUT/vB.log" 2>&1; echo "vB rc=$?"; head -20 "$OUT/vB.log"
exit 0
