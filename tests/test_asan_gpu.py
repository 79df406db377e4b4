"""The host ASan/UBSan build of the C ABI (tests/asan/Makefile `abi`, built on
the CPU by __graft_entry__.build()) on an MI355X: with a device present,
abi_check also decodes for real -- staging copies, the next-chunk helper
thread, packed hard bits into aligned and unaligned outputs, posteriors,
pageable and pinned coded input, two shards on one device, the integer
decoders, an irregular graph (N = 13, an empty column), the engine with
device-generated codes, the DNA LLR and edit-distance kernels -- and checks
valid <=> zero syndrome and fp64 == coded results.  No sanitizer report is
allowed in this library's host code; leaks the uninstrumented ROCm runtime
keeps until exit are suppressed (tests/asan/lsan.supp)."""
import os
import subprocess

import pytest

from conftest import PCHK, ROOT

pytestmark = pytest.mark.gpu
ASAN = os.path.join(ROOT, "tests", "asan")
BIN = os.path.join(ASAN, "build", "abi_check")


@pytest.mark.timeout(300)
def test_c_abi_sanitized_on_gpu(gpu, tmp_path):
    assert os.access(BIN, os.X_OK), f"{BIN} not built (make -C tests/asan abi)"
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0:exitcode=97",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=98",
               LSAN_OPTIONS="suppressions=" + os.path.join(ASAN, "lsan.supp"))
    r = subprocess.run([BIN, PCHK, str(tmp_path)], capture_output=True, text=True, env=env, timeout=280)
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr \
        and "ERROR: LeakSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    out = r.stdout.strip()
    assert out.startswith("ok abi ") and "device(s)" in out and not out.endswith(" 0 device(s)"), out
