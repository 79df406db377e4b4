"""Every store (and input read) a kernel addresses through a lane's codeword
index is bounds-checked (kernels.hpp lane_index_ok): the finished codeword's
iteration count / valid flag (cont_lanes), its hard bits and posterior
(k_var_m / k_var_msa_c), and a refilled lane's input row (the variable
kernels, k_fill_codes).  An index outside [0, B) skips the access and writes
the engine's fault words; the host reports LDPC_ERR_DEVICE naming the
index (the bookkeeping's check) or the pool slot (the variable kernels').

The LDPC_SCHED_DEBUG_BAD_LANE schedule bit stands in for broken lane
bookkeeping (round 4's illegal-address fault came from a stale lane index):
the lane that claims codeword 0 records B + 4096 instead.  Each continuous
schedule must end in LDPC_ERR_DEVICE -- never in a device fault -- and the
next clean decode on the same graph equals the oracle."""
import numpy as np
import pytest

import synth
from conftest import PCHK
from test_gpu_parity import _cmp

pytestmark = pytest.mark.gpu

def _fault_message(msg, B):
    """The report names the planted index (the bookkeeping's check) or the
    pool slot whose refill / output access the variable kernel skipped."""
    assert "lane bookkeeping fault" in msg and "out of range" in msg, msg
    assert str(B + 4096) in msg or "pool slot" in msg, msg


SCHEDULES = [
    ("bp", {}),                          # resident pool (check kernel's bookkeeping, k_var_m in place)
    ("bp", {"resident": False}),         # grouped: k_syndrome_split + k_var_m
    ("msa", {}),                         # compressed min-sum: k_var_msa_c
    ("msa", {"msa_compressed": False}),  # fp64 min-sum, resident pool
]


@pytest.mark.timeout(120)
@pytest.mark.parametrize("algo,sch", SCHEDULES)
def test_bad_lane_index_is_reported_not_written(gpu, og, codewords, algo, sch):
    L = gpu
    G2 = L.Graph(PCHK)
    B = 150
    llr = synth.bsc_llrs(codewords, 0, B, seed=5, p=0.003)
    with pytest.raises(L.LdpcError) as e:
        G2.decode(llr, max_iter=6, algo=algo, post="llr", schedule=dict(sch, debug_bad_lane=True))
    assert e.value.code == L.LDPC_ERR_DEVICE, str(e.value)
    _fault_message(str(e.value), B)
    _cmp(G2, og, llr, 6, algo=algo, schedule=sch)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("algo,sch", [("bp", {}), ("msa", {}), ("bp", {"resident": False}),
                                      ("msa", {"resident": False})])
def test_bad_lane_index_generic_code(gpu, oracle_mod, tmp_path, algo, sch):
    """A code other than the (8, 72)-regular one in the continuous pool
    (the bookkeeping of k_check_gr_res (resident) or k_syndrome_split_gen
    (grouped), k_var_gr_cont's guarded refill and output accesses), fp64 and
    coded input."""
    L = gpu
    G2 = L.Graph.rs_ldpc(6, 32, 4)
    path = tmp_path / "rs.pchk"
    G2.save_pchk(str(path))
    og2 = oracle_mod.OracleGraph(str(path))
    rng = np.random.default_rng(11)
    B = 700
    codes = np.where(rng.random((B, G2.N)) < 0.004, -1, 1).astype(np.int8)
    table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT
    llr = np.ascontiguousarray(table[codes.astype(np.int64) + 128])
    for run in (lambda sch: G2.decode(llr, max_iter=8, algo=algo, post="llr", chunk=256, schedule=sch),
                lambda sch: G2.decode_codes(codes, table, max_iter=8, algo=algo, post="llr", chunk=256,
                                            schedule=sch)):
        with pytest.raises(L.LdpcError) as e:
            run(dict(sch, debug_bad_lane=True))
        assert e.value.code == L.LDPC_ERR_DEVICE, str(e.value)
        _fault_message(str(e.value), B)
        h, _, it, v = run(sch)
        rh, _, rit, rv = og2.decode_batch(llr, 8, algo=0 if algo == "bp" else 1, threads=8, want_post=False)
        assert np.array_equal(h, rh) and np.array_equal(it, rit) and np.array_equal(v, rv.astype(bool))


@pytest.mark.timeout(120)
def test_bad_lane_index_single_fill_codes(gpu, og, codewords):
    """The DNA batch's path: one fill of the lane pool from int8 codes, whose
    step 0 is k_fill_codes' transpose of the claimed rows."""
    L = gpu
    G2 = L.Graph(PCHK)
    llr = synth.dna_like_llrs(codewords, seed=1)  # 272 codewords: one grouped fill of 5 tiles
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    assert np.array_equal(k * synth.LLR_UNIT, llr)
    table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT
    with pytest.raises(L.LdpcError) as e:
        G2.decode_codes(k, table, max_iter=20, post=None, schedule={"debug_bad_lane": True})
    assert e.value.code == L.LDPC_ERR_DEVICE, str(e.value)
    _fault_message(str(e.value), len(k))
    h, _, it, v = G2.decode_codes(k, table, max_iter=20, post=None)
    rh, _, rit, rv = og.decode_batch(llr, 20, threads=8, want_post=False)
    assert np.array_equal(h, rh) and np.array_equal(it, rit) and np.array_equal(v, rv.astype(bool))


@pytest.mark.timeout(120)
def test_bad_lane_index_engine_api(gpu, codewords):
    """Through the device-resident engine: the fault surfaces at the next
    occupancy poll or at ldpc_engine_sync, and the engine decodes cleanly
    afterwards."""
    L = gpu
    G2 = L.Graph(PCHK)
    B, N = 300, G2.N
    llr = synth.bsc_llrs(codewords, 0, B, seed=6, p=0.003)
    d_in = L.DeviceBuffer(0, B * N * 8)
    d_in.upload(np.ascontiguousarray(llr))
    d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    bad = L.Engine(G2, 0, "bp", debug_bad_lane=True)
    with pytest.raises(L.LdpcError) as e:
        bad.decode(d_in.at(0), L.IN_LLR, B, 6, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
        bad.sync()
    assert e.value.code == L.LDPC_ERR_DEVICE, str(e.value)
    _fault_message(str(e.value), B)
    # reported once: the steps enqueued before the report were drained and the
    # fault words cleared (engine.hip run_cont), so the engine syncs clean
    bad.sync()
    bad.sync()
    bad.close()
    ok = L.Engine(G2, 0, "bp")
    ok.decode(d_in.at(0), L.IN_LLR, B, 6, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
    ok.sync()
    h, _, it, v = G2.decode(llr, max_iter=6, post=None)
    assert np.array_equal(d_h.download(np.empty((B, N), np.uint8)), h)
    assert np.array_equal(d_i.download(np.empty(B, np.int32)), it)
    ok.close()
    for b in (d_in, d_h, d_i, d_v):
        b.free()
