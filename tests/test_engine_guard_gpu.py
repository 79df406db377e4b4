"""The host step loop of a continuous decode is bounded (engine.hip
run_cont): a decode whose pool never reports drained -- forced here with the
LDPC_SCHED_DEBUG_NO_DRAIN schedule flag, standing in for broken device lane bookkeeping --
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
@pytest.mark.parametrize("algo,sch", [("bp", {}), ("bp", {"resident": False}), ("msa", {}),
                                      ("msa", {"msa_compressed": False})])
def test_undrained_decode_is_bounded(gpu, og, codewords, algo, sch):
    L = gpu
    G2 = L.Graph(PCHK)
    llr = synth.bsc_llrs(codewords, 0, 150, seed=3, p=0.003)
    with pytest.raises(L.LdpcError) as e:
        G2.decode(llr, max_iter=5, algo=algo, post=None, schedule=dict(sch, debug_no_drain=True))
    assert e.value.code == L.LDPC_ERR_DEVICE and "did not drain" in str(e.value)
    _cmp(G2, og, llr, 5, algo=algo, schedule=sch)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("algo", ["bp", "msa"])
def test_all_bits_flags_set_is_resolved(gpu, G, og, codewords, algo):
    """A caller's schedule with every flags_set bit on (-1: 'take every flag
    from flags') is still resolved: bits outside LDPC_SCHED_* are dropped, so
    it cannot pose as an already-resolved schedule and skip the defaults of
    poll_every / syn_blocks / pool_tiles (which would divide by zero or launch
    an empty grid).  Through ldpc_decode and ldpc_engine_create_ex; a batch
    larger than 8 pools exercises the resident pool's polling cadence."""
    L = gpu
    s = L.Schedule()
    s.flags_set = -1
    s.flags = L.SCHED_FLAGS["continuous"] | L.SCHED_FLAGS["resident"] | L.SCHED_FLAGS["msa_compressed"]
    llr = synth.bsc_llrs(codewords, 0, 8 * 192 + 70, seed=4, p=0.004)
    _cmp(G, og, llr, 6, algo=algo, schedule=s)
    eng = L.Engine(G, 0, algo, schedule=s)
    assert eng.continuous and eng.flags & ~0x7FFF == 0
    eng.close()
