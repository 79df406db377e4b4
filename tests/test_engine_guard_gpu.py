"""The host step loop of a continuous decode is bounded (engine.hip
run_cont): a decode whose pool never reports drained -- forced here with the
LDPC_DEBUG_NO_DRAIN knob, standing in for broken device lane bookkeeping --
ends with LDPC_ERR_DEVICE and a message after ceil(B / lanes) + 1 windows of
max_iter + 2 steps (plus the poll lag), instead of enqueueing steps forever.
The device stays usable afterwards."""
import numpy as np
import pytest

import synth
from conftest import PCHK
from test_gpu_parity import _cmp

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(120)
@pytest.mark.parametrize("algo,env", [("bp", {}), ("bp", {"LDPC_RES": "0"}), ("msa", {}),
                                      ("bp", {"LDPC_RES_STREAMS": "1"}), ("msa", {"LDPC_MSA_C": "0"}),
                                      ("bp", {"LDPC_PINGPONG": "1"})])
def test_undrained_decode_is_bounded(gpu, og, codewords, monkeypatch, algo, env):
    L = gpu
    monkeypatch.setenv("LDPC_DEBUG_NO_DRAIN", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    G2 = L.Graph(PCHK)  # fresh graph -> fresh engines read the env
    llr = synth.bsc_llrs(codewords, 0, 150, seed=3, p=0.003)
    with pytest.raises(L.LdpcError) as e:
        G2.decode(llr, max_iter=5, algo=algo, post=None)
    assert e.value.code == L.LDPC_ERR_DEVICE and "did not drain" in str(e.value)
    monkeypatch.delenv("LDPC_DEBUG_NO_DRAIN")
    G3 = L.Graph(PCHK)
    _cmp(G3, og, llr, 5, algo=algo)
