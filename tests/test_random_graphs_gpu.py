"""GPU parity on random codes: a seeded sweep of parity-check matrices the
DNA code never exercises -- single rows, N not a multiple of 8 or 64, rows
heavier than 72, empty rows and columns, duplicate entries -- and random
(dv, dc) = (8, 72)-regular codes that are not array codes (the specialised
degree-72 kernels on an unstructured graph).  Each graph is written as a
.pchk and loaded on both sides (mod2sparse_read, mod2sparse.cpp:381-427);
BP (dec.cpp:583-694) and min-sum (dec.cpp:1216-1678) decodes must equal the
oracle bit for bit: hard decisions, iteration counts, valid flags and the
posterior (BP likelihood ratio, min-sum L), over ragged batches, max_iter 0
and erasures / -0.0 / infinities / NaN in the channel input; the integer decoders
(dec.cpp:699-832, 1174-1764) on a subset."""
import numpy as np
import pytest

from test_gpu_parity import _cmp, _write_pchk

pytestmark = pytest.mark.gpu


def _cmp_nan(G, og, llr, max_iter, algo="bp", schedule=None):
    """test_gpu_parity._cmp, with the NaN rule of test_nan_and_infinite_llrs:
    a NaN posterior only has to be matched by a NaN (payload and sign are not
    part of the contract); everything else bit for bit."""
    a = 0 if algo == "bp" else 1
    ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, max_iter, algo=a, post_mode=1 if a == 0 else 0, threads=8)
    kw = {"schedule": schedule} if schedule else {}
    h, p, it, v = G.decode(llr, max_iter=max_iter, algo=algo, post="ratio" if a == 0 else "llr", **kw)
    assert np.array_equal(it, ref_it) and np.array_equal(v, ref_v.astype(bool)) and np.array_equal(h, ref_h), algo
    nan = np.isnan(ref_p)
    assert np.array_equal(np.isnan(p), nan), algo
    assert np.array_equal(p[~nan].view(np.uint64), ref_p[~nan].view(np.uint64)), algo


def _random_graph(rng, M, N, deg_lo, deg_hi, dup=True):
    rows, cols = [], []
    for i in range(M):
        d = int(rng.integers(deg_lo, deg_hi + 1))
        for j in rng.choice(N, size=min(d, N), replace=False):
            rows.append(i)
            cols.append(int(j))
    if dup and rows:
        k = int(rng.integers(0, len(rows)))
        rows.append(rows[k])
        cols.append(cols[k])  # a duplicate entry: ignored (mod2sparse.cpp:521-524)
    return rows, cols


def _regular_graph(rng, Q, dv=8, dc=72):
    """A random (dv, dc)-regular code with M = dv * Q rows and N = dc * Q
    columns: row block b holds each column once (a random permutation per
    block), so no column repeats in a row and every degree is exact."""
    M, N = dv * Q, dc * Q
    rows, cols = [], []
    for b in range(dv):
        perm = rng.permutation(N)
        for i in range(Q):
            for j in perm[i * dc:(i + 1) * dc]:
                rows.append(b * Q + i)
                cols.append(int(j))
    return M, N, rows, cols


def _llr(rng, B, N, kind):
    if kind == "normal":
        x = rng.normal(1.5, 2.5, size=(B, N))
    else:  # lattice +-ln49 from a BSC, with erasures, -0.0, infinities and a NaN
        x = np.where(rng.random((B, N)) < 0.03, -3.8918202981106265, 3.8918202981106265)
        x[rng.random((B, N)) < 0.02] = 0.0
        x[rng.random((B, N)) < 0.01] = -0.0
        if B > 2:
            x[1, 0] = np.inf
            x[2, N - 1] = -np.inf
        if B > 4:
            x[4, N // 2] = np.nan
    return np.ascontiguousarray(x)


CASES = [  # (M, N, row degree range, B, max_iter, llr kind)
    (1, 2, (2, 2), 1, 5, "normal"),
    (1, 9, (9, 9), 3, 3, "lattice"),
    (3, 17, (1, 6), 65, 0, "normal"),
    (17, 63, (2, 9), 64, 12, "lattice"),
    (24, 64, (3, 12), 63, 20, "normal"),
    (30, 65, (1, 20), 130, 25, "lattice"),
    (40, 130, (0, 7), 7, 30, "normal"),
    (12, 500, (60, 110), 70, 15, "lattice"),   # rows heavier than 72
    (200, 500, (2, 6), 129, 40, "normal"),
    (64, 1001, (5, 30), 66, 25, "lattice"),
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", range(len(CASES)))
def test_random_graph_bitexact(gpu, oracle_mod, tmp_path, case):
    M, N, (lo, hi), B, max_iter, kind = CASES[case]
    rng = np.random.default_rng(1000 + case)
    rows, cols = _random_graph(rng, M, N, lo, hi)
    path = tmp_path / f"rand{case}.pchk"
    _write_pchk(path, M, N, rows, cols)
    og = oracle_mod.OracleGraph(str(path))
    G = gpu.Graph(str(path))
    assert (G.M, G.N, G.E) == (og.M, og.N, og.E)
    llr = _llr(rng, B, N, kind)
    for sch in (None, {"continuous": False}):  # continuous lane pool (column degree <= 16), fixed passes
        _cmp_nan(G, og, llr, max_iter, schedule=sch)
        _cmp_nan(G, og, llr, max_iter, algo="msa", schedule=sch)
    if case % 3 == 0:  # the integer decoders: Gallager A / B1 / B2 and quantized min-sum
        for algo, name in ((3, "gallager_a"), (4, "gallager_b1"), (5, "gallager_b2"), (2, "qmsa")):
            rh, _, rit, rv = og.decode_int_batch(llr, max_iter, algo)
            h, _, it, v = G.decode(llr, max_iter=max_iter, algo=name, post=None)
            assert np.array_equal(h, rh) and np.array_equal(it, rit) and np.array_equal(v, rv.astype(bool)), name


@pytest.mark.timeout(600)
@pytest.mark.parametrize("Q", [2, 5, 16])
def test_random_regular_8_72_bitexact(gpu, oracle_mod, tmp_path, Q):
    """(8, 72)-regular codes that are not array codes: the specialised
    degree-72 check kernels and the default schedules on an unstructured
    graph (ldpc_graph_blocks finds no block layout)."""
    rng = np.random.default_rng(Q)
    M, N, rows, cols = _regular_graph(rng, Q)
    path = tmp_path / f"reg{Q}.pchk"
    _write_pchk(path, M, N, rows, cols)
    og = oracle_mod.OracleGraph(str(path))
    G = gpu.Graph(str(path))
    assert (G.dc, G.regular_dc, G.dv, G.regular_dv) == (72, True, 8, True)
    for B, p, it in ((1, 0.01, 20), (64, 0.02, 30), (200, 0.005, 25)):
        llr = np.where(rng.random((B, N)) < p, -3.8918202981106265, 3.8918202981106265)
        _cmp(G, og, np.ascontiguousarray(llr), it)
        _cmp(G, og, np.ascontiguousarray(llr), it, algo="msa")


SCHEDULES = [
    {},                                            # defaults: resident pool (BP), compressed continuous (min-sum)
    {"resident": False},                           # grouped continuous
    {"resident": False, "nontemporal": True, "var_cpw": 8},
    {"resident": False, "group_tiles": 1, "var_cpw": 1},
    {"continuous": False},                         # fixed passes
    {"msa_compressed": False},                     # fp64 min-sum messages
    {"first_from_prior": False, "split_syndrome": False},
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("sch", range(len(SCHEDULES)))
def test_random_regular_schedules_bitexact(gpu, oracle_mod, tmp_path, sch):
    """Every schedule family on a random (8, 72)-regular code with N % 64 == 0
    (the specialised kernels' fast paths), fp64 and coded input: a schedule
    decides how the batch is laid out over launches, never what it computes."""
    rng = np.random.default_rng(77)
    M, N, rows, cols = _regular_graph(rng, 16)
    path = tmp_path / "reg16.pchk"
    _write_pchk(path, M, N, rows, cols)
    og = oracle_mod.OracleGraph(str(path))
    G = gpu.Graph(str(path))
    schedule = SCHEDULES[sch]
    B = 300
    llr = np.ascontiguousarray(np.where(rng.random((B, N)) < 0.012, -3.8918202981106265, 3.8918202981106265))
    llr[rng.random((B, N)) < 0.01] = 0.0
    for algo in ("bp", "msa"):
        h, p, it, v = _cmp(G, og, llr, 30, algo=algo, schedule=schedule)
        codes = np.rint(llr / 3.8918202981106265).astype(np.int8)
        table = np.arange(-128, 128, dtype=np.float64) * 3.8918202981106265
        h2, p2, it2, v2 = G.decode_codes(codes, table, max_iter=30, algo=algo,
                                         post="ratio" if algo == "bp" else "llr", schedule=schedule)
        assert np.array_equal(h2, h) and np.array_equal(it2, it) and np.array_equal(v2, v)
        assert np.array_equal(p2.view(np.uint64), p.view(np.uint64))


def _bucket_graph(rng, M, N, dc_max, dv_max):
    """Row 0 of degree dc_max, column 0 in dv_max rows, every other row of
    random degree 1..dc_max and no column in more than dv_max rows: the
    largest degrees sit exactly on (or one past) a register bucket of the
    generic kernels (engine.hip kGenCheckBuckets / kGenVarBuckets)."""
    sets = [set() for _ in range(M)]
    cnt = np.zeros(N, np.int64)
    for i in range(dv_max):
        sets[i].add(0)
    cnt[0] = dv_max
    for i in range(M):
        want = dc_max if i == 0 else int(rng.integers(1, dc_max + 1))
        for j in rng.permutation(np.arange(1, N)):
            if len(sets[i]) >= want:
                break
            if cnt[j] < dv_max:
                sets[i].add(int(j))
                cnt[j] += 1
    rows = [i for i in range(M) for _ in sets[i]]
    cols = [j for i in range(M) for j in sorted(sets[i])]
    return rows, cols


BUCKETS = [(8, 4), (9, 5), (16, 8), (17, 9), (32, 12), (33, 13), (48, 16), (49, 17), (64, 3), (65, 2), (96, 16),
           (97, 17), (40, 24), (41, 25), (60, 32), (61, 33)]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", range(len(BUCKETS)))
def test_generic_bucket_edges_bitexact(gpu, oracle_mod, tmp_path, case):
    """Maximum row / column degrees on and just past each register bucket
    (and past the last one: the memory-staged fallback), BP and min-sum, a
    ragged batch with erasures, infinities and a NaN."""
    dc, dv = BUCKETS[case]
    rng = np.random.default_rng(500 + case)
    M, N = max(dv + 3, 20), 300
    rows, cols = _bucket_graph(rng, M, N, dc, dv)
    path = tmp_path / f"bucket{case}.pchk"
    _write_pchk(path, M, N, rows, cols)
    og = oracle_mod.OracleGraph(str(path))
    G = gpu.Graph(str(path))
    assert (G.dc, G.dv) == (dc, dv)
    llr = _llr(rng, 130, N, "lattice" if case % 2 else "normal")
    for sch in (None, {"continuous": False}):
        _cmp_nan(G, og, llr, 20, schedule=sch)
        _cmp_nan(G, og, llr, 20, algo="msa", schedule=sch)


GEN_SCHEDULES = [
    {},                                                            # resident pool (k_check_gr_res, in place)
    {"_chunk": 0},                                                 # the engine's own pool size (gen_pool_tiles)
    {"resident": True, "pool_tiles": 1, "poll_every": 3, "_chunk": 0},
    {"continuous": False},                                         # fixed passes
    {"resident": False},                                           # grouped continuous
    {"resident": False, "group_tiles": 1, "syn_blocks": 1},
    {"resident": False, "syn_blocks": 64, "group_tiles": 2},
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("sch", range(len(GEN_SCHEDULES)))
def test_generic_continuous_bitexact(gpu, oracle_mod, tmp_path, sch):
    """Codes other than the (8, 72)-regular one in the continuous lane pool
    (k_var_gr_cont; k_syndrome_split_gen or, resident, k_check_gr_res): an
    RS-LDPC code (RS_LDPC.c) and an
    irregular random code, early-exiting BSC words in a batch several times
    the pool (lanes refilled as codewords finish), fp64 and int8-coded input,
    posteriors of every finished codeword -- equal to the oracle, and to the
    fixed-pass schedule."""
    rng = np.random.default_rng(900 + sch)
    schedule = dict(GEN_SCHEDULES[sch])
    chunk = schedule.pop("_chunk", 256)
    rows, cols = _random_graph(rng, 90, 700, 4, 40)
    path = tmp_path / "irr.pchk"
    _write_pchk(path, 90, 700, rows, cols)
    graphs = [gpu.Graph.rs_ldpc(6, 32, 4), gpu.Graph(str(path))]
    ogs = [None, oracle_mod.OracleGraph(str(path))]
    rs_path = tmp_path / "rs.pchk"
    graphs[0].save_pchk(str(rs_path))
    ogs[0] = oracle_mod.OracleGraph(str(rs_path))
    unit = 3.8918202981106265
    table = np.arange(-128, 128, dtype=np.float64) * unit
    for G, og in zip(graphs, ogs):
        assert G.dv <= 16 and not (G.dc == 72 and G.dv == 8)
        B = 1000
        for algo, p in (("bp", 0.01), ("msa", 0.003)):
            codes = np.where(rng.random((B, G.N)) < p, -1, 1).astype(np.int8)
            codes[rng.random((B, G.N)) < 0.01] = 0
            codes[rng.random((B, G.N)) < 0.002] = 3
            llr = np.ascontiguousarray(table[codes.astype(np.int64) + 128])
            a = 0 if algo == "bp" else 1
            post = "ratio" if a == 0 else "llr"
            rh, rp, rit, rv = og.decode_batch(llr, 30, algo=a, post_mode=1 if a == 0 else 0, threads=8)
            eng_kw = dict(max_iter=30, algo=algo, post=post, schedule=schedule, chunk=chunk)
            h, pp, it, v = G.decode(llr, **eng_kw)
            assert np.array_equal(h, rh) and np.array_equal(it, rit) and np.array_equal(v, rv.astype(bool)), algo
            assert np.array_equal(pp.view(np.uint64), rp.view(np.uint64)), algo
            h2, p2, it2, v2 = G.decode_codes(codes, table, **eng_kw)
            assert np.array_equal(h2, h) and np.array_equal(it2, it) and np.array_equal(v2, v), algo
            assert np.array_equal(p2.view(np.uint64), pp.view(np.uint64)), algo
            assert 1 < it.mean() < 30  # early exits: the pool refills
