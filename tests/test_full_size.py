"""Full-size GPU runs (SURVEY 8(d) configs 3 and 5 at 100 000 codewords)
checked through size-independent properties, plus an oracle sample:

* every codeword the decoder reports valid has H x = 0 (scipy sparse product
  over GF(2), independent of the decoder) and, at these noise levels, equals
  the transmitted codeword;
* codewords reported invalid ran exactly max_iter iterations;
* a random sample of 48 codewords equals the oracle bit for bit (hard
  decisions, iteration count, valid flag) -- the inputs come from the device
  BSC generator, replicated on the host by synth.bsc_llrs.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _H(G):
    rp, ci, _, _ = G.edges()
    return sp.csr_matrix((np.ones(len(ci), np.int32), ci, rp), shape=(G.M, G.N))


@pytest.mark.parametrize("algo,p,seed", [("bp", 0.004, 31), ("msa", 0.002, 32)])
def test_full_size_properties(gpu, G, og, codewords, algo, p, seed):
    L = gpu
    B, N, max_iter = 100_000, G.N, 50
    eng = L.Engine(G, 0, algo)
    cwbuf = L.DeviceBuffer(0, codewords.nbytes)
    cwbuf.upload(codewords)
    kind = L.IN_LR if algo == "bp" else L.IN_LLR
    din = L.DeviceBuffer(0, B * N * 8)
    eng.gen_bsc(din.at(0), kind, 0, B, cwbuf.at(0), 272, seed, p, synth.LLR_UNIT)
    dh, dit, dv = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    eng.decode(din.at(0), kind, B, max_iter, dh.at(0), None, L.POST_LLR, dit.at(0), dv.at(0))
    eng.sync()
    it = dit.download(np.empty(B, np.int32))
    v = dv.download(np.empty(B, np.uint8)).astype(bool)
    assert v.mean() > 0.9, v.mean()
    assert (it[~v] == max_iter).all()
    assert (it[v] <= max_iter).all() and (it >= 0).all()
    H = _H(G)
    chunk = 10_000
    for b0 in range(0, B, chunk):
        h = np.empty((chunk, N), np.uint8)
        dh.download(h, offset=b0 * N)
        syn = (H @ h.T.astype(np.int32)) % 2  # [M][chunk]
        vv = v[b0:b0 + chunk]
        assert not syn[:, vv].any(), "a codeword reported valid has a nonzero syndrome"
        assert syn[:, ~vv].any(axis=0).all(), "an invalid codeword has a zero syndrome"
        sent = codewords[np.arange(b0, b0 + chunk) % 272]
        assert (h[vv] == sent[vv]).all(), "valid but not the transmitted codeword"
    # oracle sample, bit-exact
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(B, 48, replace=False))
    llr = np.concatenate([synth.bsc_llrs(codewords, int(b), 1, seed=seed, p=p) for b in idx])
    rh, _, rit, rv = og.decode_batch(llr, max_iter, algo=0 if algo == "bp" else 1, threads=8, want_post=False)
    for k, b in enumerate(idx):
        h = np.empty((1, N), np.uint8)
        dh.download(h, offset=int(b) * N)
        assert np.array_equal(h[0], rh[k]) and it[b] == rit[k] and v[b] == bool(rv[k]), int(b)


def test_config3_exact_workload(gpu, G, og, codewords):
    """SURVEY 8(d) config 3 exactly as bench.py times it: 100 000 codewords of
    BSC p = 0.02 from the device generator with seed 2026, BP, 50 iterations,
    the engine's default schedule.  Nothing converges at p = 0.02, so every
    codeword must run all 50 iterations and end invalid; a random sample of
    64 codewords equals the oracle bit for bit."""
    L = gpu
    B, N, max_iter, seed, p = 100_000, G.N, 50, 2026, 0.02
    eng = L.Engine(G, 0, "bp")
    cwbuf = L.DeviceBuffer(0, codewords.nbytes)
    cwbuf.upload(codewords)
    din = L.DeviceBuffer(0, B * N * 8)
    eng.gen_bsc(din.at(0), L.IN_LR, 0, B, cwbuf.at(0), 272, seed, p, synth.LLR_UNIT)
    dh, dit, dv = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    eng.decode(din.at(0), L.IN_LR, B, max_iter, dh.at(0), None, L.POST_LLR, dit.at(0), dv.at(0))
    eng.sync()
    it = dit.download(np.empty(B, np.int32))
    v = dv.download(np.empty(B, np.uint8))
    assert (it == max_iter).all() and not v.any()
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(B, 64, replace=False))
    llr = np.concatenate([synth.bsc_llrs(codewords, int(b), 1, seed=seed, p=p) for b in idx])
    rh, _, rit, rv = og.decode_batch(llr, max_iter, algo=0, threads=8, want_post=False)
    assert (rit == max_iter).all() and not rv.any()
    for k, b in enumerate(idx):
        h = np.empty((1, N), np.uint8)
        dh.download(h, offset=int(b) * N)
        assert np.array_equal(h[0], rh[k]), int(b)


@pytest.mark.timeout(300)
def test_config5_exact_workload(gpu, G, og, codewords):
    """SURVEY 8(d) config 5 exactly as bench.py's secondary leg times it: 1M
    codewords of BSC p = 0.002 (seed 2026) as int8 channel codes, float
    min-sum with early termination (Run_MSA_Decoder_INF, dec.cpp:1216-1250),
    50 iterations, the engine's default schedule (compressed messages,
    1024-lane refill pool).  Properties over the whole batch (iteration
    counts, valid flags), GF(2) syndromes of hard rows from both ends and the
    interior, and 64 codewords (both ends of the batch + random interior
    ones) equal to the oracle bit for bit."""
    L = gpu
    B, N, max_iter, seed, p = 1_000_000, G.N, 50, 2026, 0.002
    eng = L.Engine(G, 0, "msa")
    assert eng.msa_compressed and eng.continuous
    cwbuf = L.DeviceBuffer(0, codewords.nbytes)
    cwbuf.upload(codewords)
    table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT
    din = L.DeviceBuffer(0, B * N)
    dh, dit, dv = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    eng.gen_bsc_codes(din.at(0), 0, B, cwbuf.at(0), 272, seed, p)
    eng.decode_codes(din.at(0), table, L.IN_LLR, B, max_iter, dh.at(0), None, L.POST_LLR, dit.at(0), dv.at(0))
    eng.sync()
    it = dit.download(np.empty(B, np.int32))
    v = dv.download(np.empty(B, np.uint8)).astype(bool)
    assert (it >= 0).all() and (it <= max_iter).all()
    assert (it[~v] == max_iter).all(), "an invalid codeword stopped early"
    assert 0.93 < v.mean() < 0.97, v.mean()  # the oracle: 0.9515 on codewords 0..3999
    assert 10 < it.mean() < 16, it.mean()
    H = _H(G)
    for b0 in (0, B // 2 - 2048, B - 4096):
        h = dh.download(np.empty((4096, N), np.uint8), offset=b0 * N)
        syn = (H @ h.T.astype(np.int32)) % 2
        vv = v[b0:b0 + 4096]
        assert not syn[:, vv].any(), "a codeword reported valid has a nonzero syndrome"
        assert syn[:, ~vv].any(axis=0).all(), "an invalid codeword has a zero syndrome"
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([np.arange(16), np.arange(B - 16, B), rng.choice(B, 32, replace=False)]))
    llr = np.concatenate([synth.bsc_llrs(codewords, int(b), 1, seed=seed, p=p) for b in idx])
    rh, _, rit, rv = og.decode_batch(llr, max_iter, algo=1, threads=8, want_post=False)
    for k, b in enumerate(idx):
        h = dh.download(np.empty((1, N), np.uint8), offset=int(b) * N)
        assert np.array_equal(h[0], rh[k]) and it[b] == rit[k] and v[b] == bool(rv[k]), int(b)
    for b in (din, dh, dit, dv, cwbuf):
        b.free()
    eng.close()
