import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dna-ldpc-codes_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
PCHK = os.path.join(GOLDEN, "decode_n18432_m2048_final.pchk")

for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # noqa: E402  (test infrastructure)
    if not os.path.exists(os.path.join(ORACLE, "liboracle.so")):
        import subprocess
        subprocess.check_call(["make", "-C", ORACLE, "liboracle.so"])
    return oracle


@pytest.fixture(scope="session")
def og(oracle_mod):
    return oracle_mod.OracleGraph(PCHK)


@pytest.fixture(scope="session")
def codewords():
    import synth
    return synth.load_codewords()


@pytest.fixture(scope="session")
def L():
    import ldpc_amd
    ldpc_amd.lib()  # fail loudly if the library is missing
    return ldpc_amd


@pytest.fixture(scope="session")
def gpu(L):
    n = L.device_count()
    if n < 1:
        pytest.fail("no GPU visible to the HIP runtime (gpu tests must run on an MI355X)")
    return L


@pytest.fixture(scope="session")
def G(gpu):
    return gpu.Graph(PCHK)


def pack(a):
    return np.packbits(np.asarray(a, dtype=np.uint8), axis=-1)
