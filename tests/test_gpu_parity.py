"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): hard decisions, iteration counts and valid
flags bit-exact; BP posterior likelihood ratio bit-exact (fp64 bytes), the
posterior LLR within 1e-5 (log differs only by device vs host libm).
"""
import hashlib

import numpy as np
import pytest

import golden_cases
import synth
from conftest import GOLDEN, PCHK, pack

pytestmark = pytest.mark.gpu
POST_TOL = 1e-5


def _cmp(G, og, llr, max_iter, algo="bp", **kw):
    a = 0 if algo == "bp" else 1
    ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, max_iter, algo=a, post_mode=1 if a == 0 else 0, threads=8)
    post = "ratio" if a == 0 else "llr"
    h, p, it, v = G.decode(llr, max_iter=max_iter, algo=algo, post=post, **kw)
    assert np.array_equal(it, ref_it), (it, ref_it)
    assert np.array_equal(v, ref_v.astype(bool))
    assert np.array_equal(h, ref_h)
    # posterior bit-exact (ratio for BP, L for min-sum) incl. inf; NaN never occurs here
    assert np.array_equal(p.view(np.uint64), ref_p.view(np.uint64))
    return h, p, it, v


def test_dna_batch_272_bitexact_50_and_200(G, og, codewords):
    """Config 2: the 272-codeword DNA batch, 50 and 200 iterations."""
    llr = synth.dna_like_llrs(codewords, seed=0)
    for it in (50, 200):
        h, _, iters, v = _cmp(G, og, llr, it)
        assert v.all() and np.array_equal(h, codewords)  # decoder.py:575-581 genie check


def test_dna_near_threshold_bitexact(G, og, codewords):
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)[:96]
    _, _, it, v = _cmp(G, og, llr, 200)
    assert (it > 10).any() and not v.all()  # mixed early exits and a failure


def test_posterior_llr_tolerance(G, og, codewords):
    llr = synth.dna_like_llrs(codewords, seed=3, reads=60000)[:40]
    _, ref_p, _, _ = og.decode_batch(llr, 50, post_mode=0, threads=8)
    _, p, _, _ = G.decode(llr, max_iter=50, post="llr")
    fin = np.isfinite(ref_p)
    assert np.array_equal(fin, np.isfinite(p))
    np.testing.assert_allclose(p[fin], ref_p[fin], rtol=0, atol=POST_TOL)


def test_bsc_nonconverging_ragged(G, og, codewords):
    """Config 3 shape at small B: p=0.02 never converges (exactly 50 iterations);
    B = 70 -> one full tile + a ragged 6-codeword tile."""
    llr = synth.bsc_llrs(codewords, 0, 70, seed=2026, p=0.02)
    _, _, it, v = _cmp(G, og, llr, 50)
    assert (it == 50).all() and not v.any()


def test_bsc_converging(G, og, codewords):
    llr = synth.bsc_llrs(codewords, 100, 64, seed=2026, p=0.004)
    _, _, it, v = _cmp(G, og, llr, 50)
    assert v.all()


def test_min_sum_early_exit(G, og, codewords):
    """Config 5 shape: min-sum with mixed early termination."""
    llr = synth.bsc_llrs(codewords, 0, 130, seed=2026, p=0.002)
    _, _, it, v = _cmp(G, og, llr, 50, algo="msa")
    assert len(np.unique(it)) > 2


def test_min_sum_nonconverging(G, og, codewords):
    llr = synth.bsc_llrs(codewords, 0, 8, seed=7, p=0.01)
    _cmp(G, og, llr, 20, algo="msa")


def test_single_codeword_and_max_iter_zero(G, og, codewords):
    llr = synth.bsc_llrs(codewords, 5, 1, seed=1, p=0.02)
    _cmp(G, og, llr, 50)
    _cmp(G, og, llr, 0)
    _cmp(G, og, llr, 0, algo="msa")
    h, p, it, v = G.decode(llr[0], max_iter=3)
    assert h.shape == (18432,) and it == 3 and v is False


def test_erasures_and_extreme_llrs(G, og, codewords):
    """LLR 0 erasures (decoder.py:514-517), huge LLRs (LR overflow -> inf,
    the NaN -> 1 guards of dec.cpp:676-677, 687-690) and -0.0."""
    rng = np.random.default_rng(11)
    llr = synth.bsc_llrs(codewords, 0, 64, seed=9, p=0.01)
    llr[rng.random(llr.shape) < 0.05] = 0.0
    llr[rng.random(llr.shape) < 0.01] *= 300.0  # exp(+-1167) -> inf / 0
    llr[rng.random(llr.shape) < 0.01] = -0.0
    _cmp(G, og, llr, 30)
    _cmp(G, og, llr, 30, algo="msa")


def test_nan_and_infinite_llrs(G, og, codewords):
    """NaN and +-inf channel LLRs: BP's LR = exp(x) becomes NaN / inf / 0 and
    runs into the NaN -> 1 guards; min-sum's |v2c| NaN exercises the
    reference's first-other-edge semantics.  Hard bits, iterations and valid
    flags bit-exact; posteriors equal bit for bit except that any NaN only
    has to be matched by a NaN (payload and sign of a NaN are not part of the
    contract)."""
    rng = np.random.default_rng(12)
    llr = synth.bsc_llrs(codewords, 0, 64, seed=10, p=0.005)
    llr[rng.random(llr.shape) < 0.002] = np.nan
    llr[rng.random(llr.shape) < 0.002] = np.inf
    llr[rng.random(llr.shape) < 0.002] = -np.inf
    llr[:4] = np.nan  # whole codewords of NaN
    for algo, a in (("bp", 0), ("msa", 1)):
        ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, 30, algo=a, post_mode=1 if a == 0 else 0, threads=8)
        h, p, it, v = G.decode(llr, max_iter=30, algo=algo, post="ratio" if a == 0 else "llr")
        assert np.array_equal(it, ref_it), algo
        assert np.array_equal(v, ref_v.astype(bool)), algo
        assert np.array_equal(h, ref_h), algo
        nan = np.isnan(ref_p)
        assert np.array_equal(np.isnan(p), nan), algo
        assert np.array_equal(p[~nan].view(np.uint64), ref_p[~nan].view(np.uint64)), algo


def test_multi_pass_chunking(G, og, codewords):
    """B larger than the resident chunk: passes of 64 codewords."""
    llr = synth.bsc_llrs(codewords, 0, 150, seed=4, p=0.006)
    _cmp(G, og, llr, 25, chunk=64)


def test_golden_vectors(G):
    z = np.load(f"{GOLDEN}/oracle_goldens.npz", allow_pickle=False)
    for case in golden_cases.CASES:
        llr, max_iter, algo = golden_cases.inputs(case, z)
        h, p, it, v = G.decode(llr, max_iter=max_iter, algo="bp" if algo == 0 else "msa",
                               post="ratio" if algo == 0 else "llr")
        assert np.array_equal(pack(h), z[case + "_hard"]), case
        assert np.array_equal(it, z[case + "_iters"]), case
        assert np.array_equal(v, z[case + "_valid"].astype(bool)), case
        assert hashlib.sha256(p.tobytes()).hexdigest() == str(z[case + "_post_sha"]), case


def test_irregular_graph_generic_kernels(gpu, oracle_mod, tmp_path):
    """Irregular degrees exercise the generic (non-template) kernels, incl.
    a degree-1 row, an empty row and an empty column."""
    rng = np.random.default_rng(3)
    M, N = 40, 120
    rows, cols = [], []
    for j in range(N - 1):  # column N-1 stays empty
        for i in rng.choice(M - 1, size=int(rng.integers(1, 5)), replace=False):  # row M-1 stays empty
            rows.append(int(i)); cols.append(j)
    rows.append(5); cols.append(7)  # duplicate entry: ignored (mod2sparse.cpp:521-524)
    # write a .pchk so both sides load the same file
    path = tmp_path / "irr.pchk"
    _write_pchk(path, M, N, rows, cols)
    og = oracle_mod.OracleGraph(str(path))
    G = gpu.Graph(str(path))
    assert (G.M, G.N, G.E) == (og.M, og.N, og.E)
    llr = rng.normal(2.0, 2.5, size=(70, N))
    llr[:, :5] = 0.0
    _cmp(G, og, llr, 40)
    _cmp(G, og, llr, 40, algo="msa")


@pytest.mark.parametrize("code", [(5, 16, 4), (6, 32, 6), (7, 64, 8)])
def test_rs_ldpc_codes_bitexact(gpu, oracle_mod, tmp_path, code):
    """Codes from the native RS-LDPC constructor (RS_LDPC.c), written as
    .pchk by the mod2sparse_write restatement and decoded on both sides."""
    s, rho, gamma = code
    g = gpu.Graph.rs_ldpc(s, rho, gamma)
    path = tmp_path / f"rs_{s}_{rho}_{gamma}.pchk"
    g.save_pchk(str(path))
    og = oracle_mod.OracleGraph(str(path))
    G = gpu.Graph(str(path))
    assert (G.M, G.N, G.E, G.dc, G.dv) == (og.M, og.N, og.E, rho, gamma)
    rng = np.random.default_rng(s)
    # all-zero codeword through a BSC (p = 4%) plus a few erasures
    flips = rng.random((96, G.N)) < 0.04
    llr = np.where(flips, -synth.LLR_UNIT, synth.LLR_UNIT)
    llr[:, ::97] = 0.0
    _cmp(G, og, llr, 30)
    _cmp(G, og, llr, 30, algo="msa")


def _write_pchk(path, M, N, rows, cols):
    by_row = {}
    for r, c in zip(rows, cols):
        by_row.setdefault(r, []).append(c)
    ints = [(ord("P") << 8) + 0x80, M, N]
    for r in sorted(by_row):
        ints.append(-(r + 1))
        ints.extend(c + 1 for c in by_row[r])
    ints.append(0)
    np.array(ints, dtype="<i4").tofile(str(path))


def test_device_bsc_generator_matches_host(gpu, G, codewords):
    L = gpu
    eng = L.Engine(G, 0, "bp", chunk=64)
    B, N = 100, G.N
    cwbuf = L.DeviceBuffer(0, codewords.nbytes)
    cwbuf.upload(codewords)
    out = L.DeviceBuffer(0, B * N * 8)
    for kind, as_lr in ((L.IN_LLR, False), (L.IN_LR, True)):
        eng.gen_bsc(out.at(0), kind, 12345, B, cwbuf.at(0), 272, 2026, 0.02, synth.LLR_UNIT)
        eng.sync()
        got = out.download(np.empty((B, N), np.float64))
        exp = synth.bsc_llrs(codewords, 12345, B, seed=2026, p=0.02, as_lr=as_lr)
        assert np.array_equal(got, exp)


def test_engine_device_resident_matches_host_api(gpu, G, og, codewords):
    """ldpc_engine_decode on device-resident LR input == ldpc_decode == oracle,
    including hard/iters/valid outputs and profiling counters."""
    L = gpu
    B, N = 130, G.N
    eng = L.Engine(G, 0, "bp", chunk=128)  # 2 passes
    cwbuf = L.DeviceBuffer(0, codewords.nbytes)
    cwbuf.upload(codewords)
    din = L.DeviceBuffer(0, B * N * 8)
    eng.gen_bsc(din.at(0), L.IN_LR, 0, B, cwbuf.at(0), 272, 77, 0.005, synth.LLR_UNIT)
    dh, dit, dv = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    eng.profile(1)
    eng.decode(din.at(0), L.IN_LR, B, 50, dh.at(0), None, L.POST_LLR, dit.at(0), dv.at(0))
    eng.sync()
    st = eng.stats()
    assert st["check"]["launches"] > 0 and st["check"]["sampled"] == st["check"]["launches"] and st["check"]["ms"] > 0
    h = dh.download(np.empty((B, N), np.uint8))
    it = dit.download(np.empty(B, np.int32))
    v = dv.download(np.empty(B, np.uint8))
    llr = synth.bsc_llrs(codewords, 0, B, seed=77, p=0.005)
    rh, _, rit, rv = og.decode_batch(llr, 50, threads=8, want_post=False)
    assert np.array_equal(it, rit) and np.array_equal(v, rv) and np.array_equal(h, rh)
    # hard output at an odd device address: the finished-lane hard-bit stores
    # of the variable kernels fall back from packed to byte stores
    for algo, kind in (("bp", L.IN_LR), ("msa", L.IN_LLR)):
        e2 = L.Engine(G, 0, algo)
        if algo == "msa":
            e2.gen_bsc(din.at(0), L.IN_LLR, 0, B, cwbuf.at(0), 272, 77, 0.002, synth.LLR_UNIT)
        dh2 = L.DeviceBuffer(0, B * N + 8)
        e2.decode(din.at(0), kind, B, 50, dh2.at(3), None, L.POST_LLR, dit.at(0), dv.at(0))
        e2.sync()
        h2 = dh2.download(np.empty(B * N + 8, np.uint8))[3:3 + B * N].reshape(B, N)
        it2 = dit.download(np.empty(B, np.int32))
        llr2 = synth.bsc_llrs(codewords, 0, B, seed=77, p=0.005 if algo == "bp" else 0.002)
        rh2, _, rit2, _ = og.decode_batch(llr2, 50, algo=0 if algo == "bp" else 1, threads=8, want_post=False)
        assert np.array_equal(it2, rit2) and np.array_equal(h2, rh2)


def test_device_exp_matches_host_on_dna_alphabet(gpu, G, codewords):
    """LLR input with exp on the device (ocml) vs the host libm: on the DNA
    alphabet k*ln49 the decode is identical (the survey's exhaustive exp check)."""
    llr = synth.dna_like_llrs(codewords, seed=0, reads=60000)[:64]
    a = G.decode(llr, max_iter=50, post="ratio", exp_on_host=True)
    b = G.decode(llr, max_iter=50, post="ratio", exp_on_host=False)
    ks = np.unique(np.rint(llr / synth.LLR_UNIT))
    assert len(ks) > 5
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y))


def test_multi_device_api_single_gpu_box(G, og, codewords):
    """devices=[0,0]: two host threads sharing one GPU exercise the sharded path."""
    llr = synth.bsc_llrs(codewords, 0, 100, seed=8, p=0.006)
    _cmp(G, og, llr, 20, devices=[0, 0])


@pytest.mark.parametrize("group,nt,cont", [(1, 0, 0), (3, 1, 0), (2, 0, 0), (-1, 1, 0), (-1, 0, 0), (3, 1, 1),
                                           (1, 0, 1), (-1, 1, 1)])
def test_grouped_schedules_bitexact(gpu, og, codewords, group, nt, cont):
    """The Infinity-Cache-resident schedule (check->variable messages of one
    tile group at a time; group -1 = the whole pass), the nontemporal
    d-stream and continuous batching change only the launch order across
    codewords, never a codeword's arithmetic."""
    sch = dict(group_tiles=group, nontemporal=bool(nt), continuous=bool(cont), resident=False)
    G2 = gpu.Graph(PCHK)
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)[:200]
    _cmp(G2, og, llr, 60, schedule=sch)
    llr = synth.bsc_llrs(codewords, 0, 200, seed=2026, p=0.002)
    _cmp(G2, og, llr, 30, algo="msa", schedule=sch)


@pytest.mark.parametrize("cpw,cont", [(1, 1), (2, 0), (4, 1), (8, 0), (2, 1)])
def test_variable_columns_per_wave_bitexact(gpu, og, codewords, cpw, cont):
    """k_var_m (CPW columns per wave, BP and min-sum) changes only which
    wave handles a column, never a column's arithmetic; with continuous
    batching its refill path initialises fresh lanes."""
    sch = dict(var_cpw=cpw, continuous=bool(cont), resident=False, msa_compressed=False)
    G2 = gpu.Graph(PCHK)
    llr = synth.dna_like_llrs(codewords, seed=3, reads=57000)[:200]
    _cmp(G2, og, llr, 60, schedule=sch)
    llr = synth.bsc_llrs(codewords, 0, 150, seed=7, p=0.004)
    _cmp(G2, og, llr, 40, schedule=sch)
    llr = synth.bsc_llrs(codewords, 0, 200, seed=8, p=0.002)
    _cmp(G2, og, llr, 30, algo="msa", schedule=sch)


@pytest.mark.parametrize("tiles,poll,cpw", [(2, 4, 4), (1, 1, 4), (3, 2, 2), (2, 7, 1)])
def test_resident_pool_in_place_bitexact(gpu, og, codewords, tiles, poll, cpw):
    """Resident pool (engine.hip run_cont `res`, k_check_bp / k_check_msa with
    RES): a pool of 1-3 tiles iterated in place (check->variable messages
    written over the variable->check messages of the same edges), the
    syndrome fused into the check kernel with last-block lane bookkeeping,
    occupancy polled every `poll` steps.  BP and fp64 min-sum stay bit-exact
    across mixed early exits, all lanes finishing at once (p = 0.02, exactly
    50 iterations), max_iter 0, batches smaller than the pool, NaN / inf."""
    sch = dict(resident=True, pool_tiles=tiles, poll_every=poll, var_cpw=cpw, msa_compressed=False)
    G2 = gpu.Graph(PCHK)
    kw = dict(chunk=64 * tiles, schedule=sch)
    e = gpu.Engine(G2, 0, "bp", **kw)
    assert e.resident and not e.syndrome_split
    del e
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)[:200]
    _cmp(G2, og, llr, 60, **kw)
    llr = np.concatenate([synth.bsc_llrs(codewords, 0, 150, seed=3, p=0.003),
                          synth.bsc_llrs(codewords, 150, 130, seed=2026, p=0.02)])
    _, _, it, _ = _cmp(G2, og, llr, 50, **kw)
    assert (it[150:] == 50).all() and len(np.unique(it[:150])) > 2
    _cmp(G2, og, llr[:70], 0, **kw)
    _cmp(G2, og, llr[:5], 50, **kw)
    _cmp(G2, og, synth.bsc_llrs(codewords, 0, 200, seed=8, p=0.002), 30, algo="msa", **kw)
    rng = np.random.default_rng(21)
    llr = synth.dna_like_llrs(codewords, seed=2, reads=60000)[:100]
    llr[rng.random(llr.shape) < 0.002] = np.nan
    llr[rng.random(llr.shape) < 0.002] = np.inf
    llr[rng.random(llr.shape) < 0.002] = -np.inf
    ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, 40, algo=0, post_mode=1, threads=8)
    h, p, it, v = G2.decode(llr, max_iter=40, algo="bp", post="ratio", **kw)
    assert np.array_equal(it, ref_it) and np.array_equal(v, ref_v.astype(bool)) and np.array_equal(h, ref_h)
    nan = np.isnan(ref_p)
    assert np.array_equal(np.isnan(p), nan)
    assert np.array_equal(p[~nan].view(np.uint64), ref_p[~nan].view(np.uint64))


@pytest.mark.parametrize("chunk", [64, 128])
def test_continuous_batching_edge_cases(gpu, og, codewords, chunk):
    """Continuous mode with a pool smaller than the batch (lanes are refilled
    many times), mixed early exits, max_iter 0, B not a multiple of 64, and
    the posterior written at each codeword's own exit."""
    G2 = gpu.Graph(PCHK)
    sch = dict(continuous=True)
    llr = np.concatenate([synth.bsc_llrs(codewords, 0, 150, seed=3, p=0.003),
                          synth.bsc_llrs(codewords, 150, 50, seed=3, p=0.02)])
    _cmp(G2, og, llr, 25, chunk=chunk, schedule=sch)
    _cmp(G2, og, llr[:70], 0, chunk=chunk, schedule=sch)
    _cmp(G2, og, llr[:130], 12, algo="msa", chunk=chunk, schedule=sch)


@pytest.mark.parametrize("msa_c,group,cont,cpw", [(0, 3, 1, 4), (1, 1, 0, 1), (1, 2, 1, 2), (1, 8, 1, 4),
                                                  (1, -1, 0, 2), (1, 4, 1, 4), (1, 5, 1, 1), (1, 4, 1, 3)])
def test_min_sum_compressed_messages_bitexact(gpu, og, codewords, msa_c, group, cont, cpw):
    """MSA-C (kernels.hpp k_check_msa_c / k_var_msa_c): the check phase stores
    per row the min1 / min2 planes, a 16-bit meta word (sign parity, NaN at
    x_0 / x_1, position of min1) and the NaN planes when needed; the variable
    phase rebuilds each c2v from them and the sign bits of the v2c it stored,
    so hard bits, iterations, valid flags and the posterior L stay bit-exact
    -- across group sizes (XCD-affine tile order, groups that do not divide
    8), continuous batching, columns per wave, and the NaN / inf / -0.0
    first-other-edge cases."""
    sch = dict(msa_compressed=bool(msa_c), group_tiles=group, continuous=bool(cont), var_cpw=cpw)
    G2 = gpu.Graph(PCHK)
    e = gpu.Engine(G2, 0, "msa", schedule=sch)
    assert e.msa_compressed == bool(msa_c)
    del e
    llr = synth.bsc_llrs(codewords, 0, 300, seed=2026, p=0.002)
    _, _, it, _ = _cmp(G2, og, llr, 50, algo="msa", schedule=sch)
    assert len(np.unique(it)) > 2
    _cmp(G2, og, synth.bsc_llrs(codewords, 0, 70, seed=5, p=0.01), 12, algo="msa", schedule=sch)
    rng = np.random.default_rng(13)
    llr = synth.bsc_llrs(codewords, 0, 130, seed=11, p=0.004)
    llr[rng.random(llr.shape) < 0.003] = np.nan
    llr[rng.random(llr.shape) < 0.002] = np.inf
    llr[rng.random(llr.shape) < 0.002] = -np.inf
    llr[rng.random(llr.shape) < 0.01] = -0.0
    llr[:2] = np.nan
    ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, 20, algo=1, post_mode=0, threads=8)
    h, p, it, v = G2.decode(llr, max_iter=20, algo="msa", post="llr", schedule=sch)
    assert np.array_equal(it, ref_it) and np.array_equal(v, ref_v.astype(bool)) and np.array_equal(h, ref_h)
    nan = np.isnan(ref_p)
    assert np.array_equal(np.isnan(p), nan)
    assert np.array_equal(p[~nan].view(np.uint64), ref_p[~nan].view(np.uint64))


@pytest.mark.parametrize("algo,msa_c,group,chunk,blocks", [("msa", 1, 4, 1024, 16), ("msa", 1, 2, 128, 3),
                                                           ("msa", 0, 3, 192, 64), ("bp", 0, 3, 256, 8),
                                                           ("bp", 0, 1, 128, 1)])
def test_split_syndrome_bitexact(gpu, og, codewords, algo, msa_c, group, chunk, blocks):
    """The continuous grouped schedule's syndrome (kernels.hpp
    k_syndrome_split) spread over `blocks` blocks per tile (8 rows per wave, 8
    edge parts per row), the last block per tile running the lane bookkeeping
    and the variable launch writing the finished codewords' outputs."""
    sch = dict(syn_blocks=blocks, continuous=True, resident=False, msa_compressed=bool(msa_c), group_tiles=group)
    G2 = gpu.Graph(PCHK)
    if algo == "bp":
        llr = np.concatenate([synth.bsc_llrs(codewords, 0, 300, seed=3, p=0.003),
                              synth.bsc_llrs(codewords, 300, 100, seed=2026, p=0.02)])
        _, _, it, _ = _cmp(G2, og, llr, 30, chunk=chunk, schedule=sch)
    else:
        llr = synth.bsc_llrs(codewords, 0, 400, seed=2026, p=0.002)
        _, _, it, _ = _cmp(G2, og, llr, 50, algo="msa", chunk=chunk, schedule=sch)
    assert len(np.unique(it)) > 2
    _cmp(G2, og, llr[:70], 0, algo=algo, chunk=chunk, schedule=sch)
    _cmp(G2, og, llr[:3], 20, algo=algo, chunk=chunk, schedule=sch)


def test_host_lr_table_path(G, og, codewords):
    """ldpc_decode's LR table path (capi.cpp): LLRs that are exact multiples
    k * unit (the DNA alphabet) cross PCIe as one byte each and become
    table[k] = host exp(k * unit), the same bits as exp(LLR).  Bit-exact
    against the oracle (host exp), identical to the exp path (lr_table off),
    and batches off the alphabet (several units, a non-multiple, NaN) fall
    back to the host exp."""
    llr = synth.dna_like_llrs(codewords, seed=5, reads=60000)[:150]
    h1, p1, it1, v1 = _cmp(G, og, llr, 60)
    h0, p0, it0, v0 = G.decode(llr, max_iter=60, post="ratio", schedule=dict(lr_table=False))
    assert np.array_equal(h0, h1) and np.array_equal(it0, it1) and np.array_equal(p0.view(np.uint64), p1.view(np.uint64))
    mixed = llr[:40].copy()
    mixed[7] *= 1.5  # a second unit
    mixed[9, 100] = 0.123  # off the alphabet
    mixed[11, 5] = np.nan
    _cmp(G, og, mixed, 60) if not np.isnan(mixed).any() else None
    ref_h, _, ref_it, ref_v = og.decode_batch(mixed, 60, algo=0, threads=8, want_post=False)
    h, _, it, v = G.decode(mixed, max_iter=60, post=None)
    assert np.array_equal(h, ref_h) and np.array_equal(it, ref_it) and np.array_equal(v, ref_v.astype(bool))



def test_single_fill_first_check_from_prior(gpu, G, og, codewords):
    """A batch that fits the lane pool in one fill (the DNA batch through
    ldpc_decode): the refill stores only the prior and the first check takes
    d0 = 1 - 2/(1+LR) from it (k_check_bp_first) instead of E stored copies.
    Bit-exact against the oracle and identical to the stored-copies path
    (first_from_prior off) at max_iter 0 / 1 / 2 / 60, with NaN / +-inf
    inputs, for host LR (ldpc_decode) and device exp (Engine, LLR input)."""
    rng = np.random.default_rng(33)
    nasty = synth.dna_like_llrs(codewords, seed=6, reads=57000)[:150]
    nasty[rng.random(nasty.shape) < 0.002] = np.nan
    nasty[rng.random(nasty.shape) < 0.002] = np.inf
    nasty[rng.random(nasty.shape) < 0.002] = -np.inf
    cases = [(synth.dna_like_llrs(codewords, seed=7, reads=58000), it) for it in (0, 1, 2, 60)]
    cases.append((nasty, 40))
    for llr, it in cases:
        ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, it, algo=0, post_mode=1, threads=8)
        outs = []
        for fp in (True, False):
            h, p, i, v = G.decode(llr, max_iter=it, post="ratio", schedule=dict(first_from_prior=fp))
            assert np.array_equal(i, ref_it) and np.array_equal(v, ref_v.astype(bool)) and np.array_equal(h, ref_h)
            nan = np.isnan(ref_p)
            assert np.array_equal(np.isnan(p), nan)
            assert np.array_equal(p[~nan].view(np.uint64), ref_p[~nan].view(np.uint64))
            outs.append((h, i))
        assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    # device-resident engine, LLR input (device exp in the refill), one fill of 150
    L = gpu
    llr = synth.dna_like_llrs(codewords, seed=8, reads=58000)[:150]
    B, N = llr.shape
    eng = L.Engine(G, 0, "bp", chunk=B)
    d_in = L.DeviceBuffer(0, B * N * 8)
    d_in.upload(np.ascontiguousarray(llr))
    d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    eng.decode(d_in.at(0), L.IN_LLR, B, 100, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
    eng.sync()
    ref_h, _, ref_it, ref_v = og.decode_batch(llr, 100, algo=0, threads=8, want_post=False)
    assert np.array_equal(d_i.download(np.empty(B, np.int32)), ref_it)
    assert np.array_equal(d_h.download(np.empty((B, N), np.uint8)), ref_h)


@pytest.mark.timeout(240)
def test_min_sum_compressed_on_rows_permuted(gpu, G, oracle_mod, codewords, tmp_path):
    """The DNA code with its rows permuted: still (72, 8)-regular, so the
    compressed min-sum runs, but edge s of a column no longer lies in row
    block s, so its v2c takes the plain column order instead of the
    row-block-major one (engine.hip); both layouts are exercised against the
    oracle, over several fills of the lane pool."""
    rp, ci, _, _ = G.edges()
    rows = np.repeat(np.arange(G.M), np.diff(rp))
    perm = np.random.default_rng(9).permutation(G.M)
    path = tmp_path / "dna_rows_permuted.pchk"
    _write_pchk(path, G.M, G.N, perm[rows].tolist(), ci.tolist())
    og2 = oracle_mod.OracleGraph(str(path))
    G2 = gpu.Graph(str(path))
    assert (G2.dc, G2.dv, G2.regular_dc, G2.regular_dv) == (72, 8, True, True)
    llr = synth.bsc_llrs(codewords, 0, 1500, seed=41, p=0.002)
    sel = np.r_[0:40, 700:730, 1460:1500]
    h, p, it, v = G2.decode(llr, max_iter=30, algo="msa", post="llr")
    rh, rp_, rit, rv = og2.decode_batch(llr[sel], 30, algo=1, post_mode=0, threads=8)
    assert np.array_equal(h[sel], rh) and np.array_equal(it[sel], rit) and np.array_equal(v[sel], rv.astype(bool))
    assert np.array_equal(p[sel].view(np.uint64), rp_.view(np.uint64))
    assert len(np.unique(it)) > 3
