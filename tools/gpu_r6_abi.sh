#!/bin/bash
# Round 6: the C-ABI driver over the product library and over its host-ASan build, on the GPU.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r6abi; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
P=tests/golden/decode_n18432_m2048_final.pchk
mkdir -p /tmp/abi1 /tmp/abi2
timeout -k 10 120 tests/asan/build/abi_check_plain $P /tmp/abi1 > "$OUT/plain.log" 2>&1; echo "plain rc=$?"; cat "$OUT/plain.log" | head -30
rc=$(tail -1 "$OUT/plain.log" | grep -c "ok abi")
LSAN_OPTIONS=suppressions=$R/tests/asan/lsan.supp ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 timeout -k 10 200 tests/asan/build/abi_check $P /tmp/abi2 > "$OUT/asan.log" 2>&1; echo "asan rc=$?"; grep -v "^$" "$OUT/asan.log" | head -40
exit 0
