"""GPU parity of the XCD-resident BP decoder (kernels_xr.hpp, LDPC_XR=1)
against the oracle: one persistent launch, each codeword held by one slot
whose messages stay in one XCD's L2, check / variable tasks claimed by the
XCD's workgroups.  Same bar as test_gpu_parity.py: hard bits, iteration
counts, valid flags and the BP posterior ratio bit-exact."""
import numpy as np
import pytest

import synth
from conftest import PCHK

pytestmark = pytest.mark.gpu


def _cmp(G, og, llr, max_iter, post="ratio"):
    ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, max_iter, algo=0, post_mode=1 if post == "ratio" else 0,
                                                  threads=8)
    h, p, it, v = G.decode(llr, max_iter=max_iter, algo="bp", post=post)
    assert np.array_equal(it, ref_it), (np.nonzero(it != ref_it)[0][:8], it[:8], ref_it[:8])
    assert np.array_equal(v, ref_v.astype(bool))
    assert np.array_equal(h, ref_h)
    nan = np.isnan(ref_p)
    assert np.array_equal(np.isnan(p), nan)
    if post == "ratio":
        assert np.array_equal(p[~nan].view(np.uint64), ref_p[~nan].view(np.uint64))
    else:
        fin = np.isfinite(ref_p)
        np.testing.assert_allclose(p[fin], ref_p[fin], rtol=0, atol=1e-5)
    return h, p, it, v


@pytest.fixture
def xr(monkeypatch):
    monkeypatch.setenv("LDPC_XR", "1")
    return monkeypatch


def test_xr_engine_selected(gpu, xr):
    G = gpu.Graph(PCHK)
    assert gpu.Engine(G, 0, "bp").xcd_resident
    assert not gpu.Engine(G, 0, "msa").xcd_resident


@pytest.mark.parametrize("k", [1, 3])
def test_xr_bitexact(gpu, og, codewords, xr, k):
    """DNA batch (all converge), near-threshold inputs (mixed exits, failures),
    BSC p = 0.02 (exactly 50 iterations), converging and non-converging
    codewords in one batch, max_iter 0, batches smaller than the slot count,
    NaN / inf inputs, LLR posterior."""
    xr.setenv("LDPC_XR_K", str(k))
    G = gpu.Graph(PCHK)
    llr = synth.dna_like_llrs(codewords, seed=0)
    h, _, _, v = _cmp(G, og, llr, 50)
    assert v.all() and np.array_equal(h, codewords)
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)[:96]
    _, _, it, v = _cmp(G, og, llr, 200)
    assert (it > 10).any() and not v.all()
    llr = np.concatenate([synth.bsc_llrs(codewords, 0, 150, seed=3, p=0.003),
                          synth.bsc_llrs(codewords, 150, 70, seed=2026, p=0.02)])
    _, _, it, v = _cmp(G, og, llr, 50)
    assert (it[150:] == 50).all() and not v[150:].any() and len(np.unique(it[:150])) > 2
    _cmp(G, og, llr[:70], 0)
    _cmp(G, og, llr[148:149], 50)
    _cmp(G, og, llr[140:156], 70000) if k == 1 else None  # beyond the slots' 16-bit counts: the tiled state
    _cmp(G, og, llr[:5], 50)
    rng = np.random.default_rng(21)
    llr = synth.dna_like_llrs(codewords, seed=2, reads=60000)[:100]
    llr[rng.random(llr.shape) < 0.002] = np.nan
    llr[rng.random(llr.shape) < 0.002] = np.inf
    llr[rng.random(llr.shape) < 0.002] = -np.inf
    llr[:2] = np.nan
    _cmp(G, og, llr, 40)
    _cmp(G, og, synth.dna_like_llrs(codewords, seed=3, reads=60000)[:40], 50, post="llr")


def test_xr_rs_code_q128(gpu, oracle_mod, xr, tmp_path):
    """RS-LDPC(7, 72, 8): blocks of Q = 128 in natural column order (two
    waves per task)."""
    R = gpu.Graph.rs_ldpc(7, 72, 8)
    assert R.blocks()[0] == 128
    path = str(tmp_path / "rs7.pchk")
    R.save_pchk(path)
    G = gpu.Graph(path)
    ogr = oracle_mod.OracleGraph(path)
    rng = np.random.default_rng(5)
    B = 90
    flip = rng.random((B, G.N)) < np.linspace(0.001, 0.03, B)[:, None]  # all-zero codeword over a BSC
    llr = np.where(flip, -np.log(49.0), np.log(49.0))
    _, _, it, v = _cmp(G, ogr, llr, 40)
    assert v.any() and not v.all()


def test_xr_device_exp_engine(gpu, og, codewords, xr):
    """Device-resident engine with LLR input (ocml exp in the refill) on the
    DNA alphabet, where it equals the host libm exp the oracle uses."""
    L = gpu
    G = L.Graph(PCHK)
    eng = L.Engine(G, 0, "bp")
    assert eng.xcd_resident
    llr = synth.dna_like_llrs(codewords, seed=4, reads=58000)[:120]
    B, N = llr.shape
    d_in = L.DeviceBuffer(0, B * N * 8)
    d_in.upload(np.ascontiguousarray(llr))
    d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    eng.decode(d_in.at(0), L.IN_LLR, B, 100, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
    eng.sync()
    h = d_h.download(np.empty((B, N), np.uint8))
    it = d_i.download(np.empty(B, np.int32))
    v = d_v.download(np.empty(B, np.uint8))
    ref_h, _, ref_it, ref_v = og.decode_batch(llr, 100, algo=0, threads=8, want_post=False)
    assert np.array_equal(it, ref_it) and np.array_equal(v, ref_v) and np.array_equal(h, ref_h)
