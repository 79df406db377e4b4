"""Coded channel input (ldpc_engine_decode_codes, the host API's code table path).

The DNA pipeline's soft input is a per-bit count difference k with LLR =
k * ln 49 (decoder.py:314); a BSC's is +-1 * ln 49.  Decoding the int8 codes
with a 256-entry table must give exactly what decoding the fp64 values
table[k + 128] gives -- BP's LR being the host exp of the LLR
(DNA_main.cpp:1344) -- on every schedule: the continuous ones keep each lane's
prior as its code (kernels.hpp prior_at / Refill::pcode), the others expand the
codes to fp64 first.
"""
import numpy as np
import pytest

import synth
from conftest import PCHK

pytestmark = pytest.mark.gpu


def _table(unit=synth.LLR_UNIT):
    return np.arange(-128, 128, dtype=np.float64) * unit


def _run(L, eng, B, N, fn):
    dh, dit, dv = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    dp = L.DeviceBuffer(0, B * N * 8)
    fn(dh.at(0), dp.at(0), dit.at(0), dv.at(0))
    eng.sync()
    return (dh.download(np.empty((B, N), np.uint8)), dp.download(np.empty((B, N), np.float64)),
            dit.download(np.empty(B, np.int32)), dv.download(np.empty(B, np.uint8)))


def _same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def test_device_bsc_codes_match_llrs(gpu, G, codewords):
    L = gpu
    eng = L.Engine(G, 0, "bp", chunk=64)
    B, N = 90, G.N
    cw = L.DeviceBuffer(0, codewords.nbytes)
    cw.upload(codewords)
    out = L.DeviceBuffer(0, B * N)
    eng.gen_bsc_codes(out.at(0), 4321, B, cw.at(0), 272, 2026, 0.02)
    eng.sync()
    codes = out.download(np.empty((B, N), np.int8))
    assert set(np.unique(codes)) <= {-1, 1}
    exp = synth.bsc_llrs(codewords, 4321, B, seed=2026, p=0.02)
    assert np.array_equal(_table()[codes.astype(np.int64) + 128], exp)


# (algo, schedule, chunk): the resident BP pool, the grouped continuous BP
# schedule with a single fill (first check from the prior), fixed passes, the
# compressed and the fp64 continuous min-sum, and the quantized min-sum
CASES = [("bp", {}, 0), ("bp", dict(resident=False), 0), ("bp", dict(resident=False), 320),
         ("bp", dict(continuous=False), 128), ("msa", {}, 0), ("msa", dict(msa_compressed=False), 0),
         ("msa", dict(continuous=False), 0), ("qmsa", {}, 128)]


@pytest.mark.parametrize("algo,sch,chunk", CASES)
def test_coded_equals_fp64_input(gpu, G, codewords, algo, sch, chunk):
    """decode_codes == decode on the expanded fp64 input, bit for bit: hard
    bits, posterior, iterations, valid flags (BSC codes generated on the device,
    and DNA count differences with erasures uploaded from the host)."""
    L = gpu
    N = G.N
    cw = L.DeviceBuffer(0, codewords.nbytes)
    cw.upload(codewords)
    p = 0.004 if algo == "bp" else 0.002
    B = 300
    eng = L.Engine(G, 0, algo, chunk=chunk, schedule=sch)
    codes = L.DeviceBuffer(0, B * N)
    eng.gen_bsc_codes(codes.at(0), 0, B, cw.at(0), 272, 2026, p)
    fp = L.DeviceBuffer(0, B * N * 8)
    bp = algo == "bp"
    kind = L.IN_LR if bp else L.IN_LLR
    eng.gen_bsc(fp.at(0), kind, 0, B, cw.at(0), 272, 2026, p, synth.LLR_UNIT)
    tab = _table()
    post = L.POST_RATIO if bp else L.POST_LLR
    a = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode_codes(codes.at(0), tab, L.IN_LLR, B, 40, h, pp, post, it, v))
    b = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode(fp.at(0), kind, B, 40, h, pp, post, it, v))
    _same(a, b)
    assert len(np.unique(a[2])) > 2
    # DNA count differences (erasures k = 0 included), one fill of the pool
    llr = synth.dna_like_llrs(codewords, seed=4, reads=58000)[:150]
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    assert np.array_equal(k.astype(np.float64) * synth.LLR_UNIT, llr)
    B = len(k)
    codes.upload(k)
    fp.upload(np.exp(llr) if bp else llr)
    a = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode_codes(codes.at(0), tab, L.IN_LLR, B, 60, h, pp, post, it, v))
    b = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode(fp.at(0), kind, B, 60, h, pp, post, it, v))
    _same(a, b)


def test_coded_lr_table_and_oracle(gpu, G, og, codewords):
    """An LR table (BP) equals the LLR table's host exp, and the coded decode
    equals the oracle; a min-sum engine refuses an LR table."""
    L = gpu
    N = G.N
    llr = synth.dna_like_llrs(codewords, seed=9, reads=56000)[:130]
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    B = len(k)
    codes = L.DeviceBuffer(0, B * N)
    codes.upload(k)
    eng = L.Engine(G, 0, "bp")
    a = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode_codes(codes.at(0), _table(), L.IN_LLR, B, 60, h, pp,
                                                                 L.POST_RATIO, it, v))
    b = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode_codes(codes.at(0), np.exp(_table()), L.IN_LR, B, 60, h,
                                                                 pp, L.POST_RATIO, it, v))
    _same(a, b)
    rh, rp, rit, rv = og.decode_batch(llr, 60, algo=0, post_mode=1, threads=8)
    assert np.array_equal(a[0], rh) and np.array_equal(a[2], rit) and np.array_equal(a[3], rv)
    assert np.array_equal(a[1].view(np.uint64), rp.view(np.uint64))
    em = L.Engine(G, 0, "msa")
    with pytest.raises(L.LdpcError):
        em.decode_codes(codes.at(0), np.exp(_table()), L.IN_LR, B, 10)


def test_host_api_min_sum_code_path(G, og, codewords):
    """ldpc_decode sends lattice LLR batches as codes for min-sum too (capi.cpp
    code table path): equal to the oracle and to the fp64 path (lr_table off)."""
    llr = synth.bsc_llrs(codewords, 0, 200, seed=2026, p=0.002)
    ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, 50, algo=1, post_mode=0, threads=8)
    for lt in (True, False):
        h, p, it, v = G.decode(llr, max_iter=50, algo="msa", post="llr", schedule=dict(lr_table=lt))
        assert np.array_equal(it, ref_it) and np.array_equal(v, ref_v.astype(bool)) and np.array_equal(h, ref_h)
        assert np.array_equal(p.view(np.uint64), ref_p.view(np.uint64))


def test_changing_tables_between_decodes(gpu, codewords):
    """Back-to-back coded decodes with different tables on one engine: each
    sees its own table (the upload waits for the decodes that read the last)."""
    L = gpu
    G2 = L.Graph(PCHK)
    N = G2.N
    llr = synth.dna_like_llrs(codewords, seed=10, reads=57000)[:64]
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    codes = L.DeviceBuffer(0, k.nbytes)
    codes.upload(k)
    eng = L.Engine(G2, 0, "bp")
    outs = []
    for unit in (synth.LLR_UNIT, 0.7, synth.LLR_UNIT):
        outs.append(_run(L, eng, 64, N, lambda h, pp, it, v: eng.decode_codes(
            codes.at(0), _table(unit), L.IN_LLR, 64, 30, h, pp, L.POST_RATIO, it, v)))
    _same(outs[0], outs[2])
    assert not np.array_equal(outs[0][1], outs[1][1])
    ref = G2.decode(k.astype(np.float64) * 0.7, max_iter=30, post="ratio", schedule=dict(lr_table=False))
    assert np.array_equal(outs[1][0], ref[0]) and np.array_equal(outs[1][2], ref[2])
    assert np.array_equal(outs[1][1].view(np.uint64), ref[1].view(np.uint64))


@pytest.mark.parametrize("algo", ["bp", "msa"])
def test_coded_nonfinite_table_entries(gpu, G, codewords, algo):
    """Table entries NaN / +-inf / -0.0 (the NaN guards of dec.cpp:676-687 and
    the min-sum sign / NaN rules): the coded decode equals the fp64 decode of
    table[code + 128] bit for bit, posterior NaN positions included."""
    L = gpu
    N = G.N
    rng = np.random.default_rng(5)
    k = rng.integers(-3, 4, size=(130, N)).astype(np.int8)
    k[rng.random(k.shape) < 0.6] = 1  # mostly a confident 0
    table = _table()
    table[128 + 2] = np.nan
    table[128 - 3] = -np.inf
    table[128 + 3] = np.inf
    table[128] = -0.0
    bp = algo == "bp"
    vals = table[k.astype(np.int64) + 128]
    B = len(k)
    codes = L.DeviceBuffer(0, B * N)
    codes.upload(k)
    fp = L.DeviceBuffer(0, B * N * 8)
    with np.errstate(over="ignore", invalid="ignore"):
        fp.upload(np.ascontiguousarray(np.exp(vals) if bp else vals))
    eng = L.Engine(G, 0, algo)
    kind = L.IN_LR if bp else L.IN_LLR
    post = L.POST_RATIO if bp else L.POST_LLR
    a = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode_codes(codes.at(0), table, L.IN_LLR, B, 20, h, pp, post, it, v))
    b = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode(fp.at(0), kind, B, 20, h, pp, post, it, v))
    _same(a, b)


@pytest.mark.parametrize("algo", ["bp", "msa"])
def test_host_api_negative_zero_and_off_lattice(G, og, codewords, algo):
    """ldpc_decode's code table path takes only exact lattice batches: for
    min-sum a -0.0 LLR (equal to 0 * unit, other bits; min-sum sums keep a
    zero's sign) and for both an off-lattice value send the batch through the
    fp64 path (BP keeps -0.0 on the code path: exp(-0.0) == exp(0.0)); results
    equal the oracle bit for bit, posterior included."""
    a = 0 if algo == "bp" else 1
    llr = synth.dna_like_llrs(codewords, seed=12, reads=57000)[:96].copy()
    zeros = np.argwhere(llr == 0)
    assert len(zeros) > 10
    r, c = zeros[:10].T
    llr[r, c] = -0.0
    # max_iter 0: the posterior is the input itself (a -0.0 must come back as -0.0)
    for case, mi in ((llr, 0), (llr, 40), (np.where(np.arange(llr.shape[1]) == 7, llr * 1.0000001, llr), 40)):
        ref_h, ref_p, ref_it, ref_v = og.decode_batch(case, mi, algo=a, post_mode=1 if a == 0 else 0, threads=8)
        h, p, it, v = G.decode(case, max_iter=mi, algo=algo, post="ratio" if a == 0 else "llr")
        assert np.array_equal(it, ref_it) and np.array_equal(v, ref_v.astype(bool)) and np.array_equal(h, ref_h)
        assert np.array_equal(p.view(np.uint64), ref_p.view(np.uint64))


@pytest.mark.timeout(180)
@pytest.mark.parametrize("max_iter", [1, 2, 50])
def test_msa_coded_refills_over_several_fills(gpu, G, og, codewords, max_iter):
    """The compressed min-sum's coded refills over several pool fills (2500
    codewords through the 1024-lane pool, so refills land in tiles with live
    lanes), with noiseless rows (iteration-0 exits) and max_iter 1 / 2 / 50:
    identical hard bits, posterior, iterations and valid flags to the fp64
    input, and a sample from both ends and the middle equal to the oracle."""
    L = gpu
    N, B = G.N, 2500
    llr = synth.bsc_llrs(codewords, 0, B, seed=77, p=0.002)
    llr[::7] = np.where(codewords[np.arange(0, B, 7) % 272] == 1, -synth.LLR_UNIT, synth.LLR_UNIT)
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    codes = L.DeviceBuffer(0, B * N)
    codes.upload(k)
    fp = L.DeviceBuffer(0, B * N * 8)
    fp.upload(llr)
    eng = L.Engine(G, 0, "msa")
    assert eng.msa_compressed and eng.continuous and eng.cap < B
    a = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode_codes(codes.at(0), _table(), L.IN_LLR, B, max_iter, h, pp,
                                                                 L.POST_LLR, it, v))
    b = _run(L, eng, B, N, lambda h, pp, it, v: eng.decode(fp.at(0), L.IN_LLR, B, max_iter, h, pp, L.POST_LLR, it, v))
    _same(a, b)
    it = a[2]
    assert (it[::7] == 0).all() and a[3][::7].all()
    if max_iter == 50:
        assert len(np.unique(it)) > 5
    idx = np.unique(np.concatenate([np.arange(0, 21), np.arange(B - 20, B), np.arange(1000, 1030)]))
    rh, rp, rit, rv = og.decode_batch(llr[idx], max_iter, algo=1, post_mode=0, threads=8)
    assert np.array_equal(a[0][idx], rh) and np.array_equal(a[2][idx], rit) and np.array_equal(a[3][idx], rv)
    assert np.array_equal(a[1][idx].view(np.uint64), rp.view(np.uint64))
    eng.close()


@pytest.mark.parametrize("algo,kw", [("bp", {}), ("bp", dict(chunk=64, devices=[0, 0])), ("msa", {}),
                                     ("qmsa", {}), ("gallager_b1", {})])
def test_host_decode_codes_equals_llr_decode(G, og, codewords, algo, kw):
    """ldpc_decode_codes (the DNA stage's count differences k + the table
    k * ln49, no fp64 matrix) == ldpc_decode on the LLRs table[k + 128], bit
    for bit -- one fill, several chunks and devices, every decoder family --
    and BP also equals the oracle and the LR-table form."""
    llr = synth.dna_like_llrs(codewords, seed=21, reads=58000)[:200]
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    assert np.array_equal(k * synth.LLR_UNIT, llr)
    post = "ratio" if algo == "bp" else "llr"
    a = G.decode_codes(k, _table(), max_iter=60, algo=algo, post=post, **kw)
    b = G.decode(llr, max_iter=60, algo=algo, post=post, schedule=dict(lr_table=False), **kw)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    if algo == "bp":
        rh, rp, rit, rv = og.decode_batch(llr, 60, algo=0, post_mode=1, threads=8)
        assert np.array_equal(a[0], rh) and np.array_equal(a[2], rit) and np.array_equal(a[3], rv.astype(bool))
        assert np.array_equal(a[1].view(np.uint64), rp.view(np.uint64))
        import ldpc_amd as L
        c = G.decode_codes(k, np.exp(_table()), table_kind=L.IN_LR, max_iter=60, post=post, **kw)
        for x, y in zip(a, c):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def test_host_decode_codes_errors(G):
    import ldpc_amd as L
    k = np.zeros((3, G.N), np.int8)
    with pytest.raises(L.LdpcError):
        G.decode_codes(k, np.exp(_table()), table_kind=L.IN_LR, algo="msa", max_iter=5)
    with pytest.raises(ValueError):
        G.decode_codes(k, _table()[:100], max_iter=5)
    h, p, it, v = G.decode_codes(k[0], _table(), max_iter=5, post=None)  # 1-D: one codeword
    assert h.shape == (G.N,) and p is None


def test_host_decode_codes_pinned_input(G, codewords):
    """Codes in pinned host memory (ldpc_amd.host_empty / ldpc_host_alloc)
    cross PCIe straight from the caller's array: the same results as from
    pageable memory, over several chunks and devices too."""
    import ldpc_amd as L
    llr = synth.dna_like_llrs(codewords, seed=22, reads=58000)[:200]
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    kp = L.host_empty(k.shape, np.int8)
    kp[...] = k
    for kw in ({}, dict(chunk=64, devices=[0, 0])):
        a = G.decode_codes(k, _table(), max_iter=60, post="ratio", **kw)
        b = G.decode_codes(kp, _table(), max_iter=60, post="ratio", **kw)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    del kp


@pytest.mark.timeout(200)
def test_host_decode_codes_several_transfer_chunks(G, codewords):
    """More codewords than one PCIe transfer chunk (4096): the codes go
    through the double-buffered chunk pipeline (the next chunk copied while
    the previous decodes), pageable and pinned, BP and min-sum -- equal to
    ldpc_decode on the LLRs."""
    import ldpc_amd as L
    B = 4096 + 300
    llr = synth.bsc_llrs(codewords, 0, B, seed=31, p=0.004)
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    kp = L.host_empty(k.shape, np.int8)
    kp[...] = k
    for algo in ("bp", "msa"):
        ref = G.decode(llr, max_iter=20, algo=algo, post=None, schedule=dict(lr_table=False))
        for src in (k, kp):
            out = G.decode_codes(src, _table(), max_iter=20, algo=algo, post=None)
            assert np.array_equal(out[0], ref[0]) and np.array_equal(out[2], ref[2]) and np.array_equal(out[3], ref[3])
    del kp
