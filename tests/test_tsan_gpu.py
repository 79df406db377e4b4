"""Race detection on the C ABI's host side, on an
MI355X: tests/tsan/build/tsan_check over a ThreadSanitizer build of the
library's host code (tests/tsan/Makefile; built on the CPU by
__graft_entry__.build()).  Eight threads share one graph -- BP and min-sum
host decodes (two of them over two PCIe chunks), coded input, the device-resident engine, graph loads and
per-thread errors -- plus a two-shard call's per-device worker threads;
results must equal the single-thread calls and ThreadSanitizer must report
nothing.  Uninstrumented libraries (the HIP runtime) are ignored
(ignore_noninstrumented_modules), so a report names a race in this
library's own host code."""
import os
import subprocess

import pytest

from conftest import PCHK, ROOT

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "tests", "tsan", "build", "tsan_check")


@pytest.mark.timeout(300)
def test_c_abi_threads_race_free(gpu):
    assert os.access(BIN, os.X_OK), f"{BIN} not built (make -C tests/tsan)"
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 ignore_noninstrumented_modules=1 exitcode=66 "
                                        "second_deadlock_stack=1")
    r = subprocess.run([BIN, PCHK], capture_output=True, text=True, env=env, timeout=280)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.strip().startswith("ok tsan") and "MISMATCH" not in r.stdout
    # the detector is live here: a deliberate race in the driver is reported
    s = subprocess.run([BIN, "--selftest"], capture_output=True, text=True, env=env, timeout=60)
    assert s.returncode == 66 and "WARNING: ThreadSanitizer: data race" in s.stderr, (s.returncode, s.stderr[-2000:])
