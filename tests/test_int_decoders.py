"""Integer-message decoders of dec.cpp: quantized /
offset min-sum (Run_MSA_Decoder dec.cpp:1174) and Gallager A/B1/B2
(Run_Gallager_Decoder dec.cpp:699).  CPU: the oracle on known answers.
GPU (marked): the HIP path bit-exact against the oracle."""
import math

import numpy as np
import pytest

import synth
from conftest import PCHK

L49 = math.log(49.0)


@pytest.fixture(scope="module")
def og_int(oracle_mod):
    return oracle_mod.OracleGraph(PCHK)


def test_oracle_noiseless_zero_iterations(og_int, codewords):
    llr = np.where(codewords[:4] == 1, -L49, L49)
    for algo in (2, 3, 4, 5):
        h, post, it, v = og_int.decode_int_batch(llr, 20, algo, precision=6, step=0.5)
        assert np.array_equal(h, codewords[:4]) and (it == 0).all() and v.all()


def test_oracle_single_flip_corrected(og_int, codewords):
    """Girth-6 RS-LDPC code, dv = 8: one flipped bit is corrected by every
    decoder in one iteration."""
    x = codewords[:3].copy()
    for b, j in enumerate((0, 9000, 18431)):
        x[b, j] ^= 1
    llr = np.where(x == 1, -L49, L49)
    for algo in (2, 3, 4, 5):
        h, post, it, v = og_int.decode_int_batch(llr, 20, algo, precision=6, step=0.5, beta=1)
        assert np.array_equal(h, codewords[:3]) and (it == 1).all() and v.all(), algo


def test_oracle_quantizer_and_posterior(og_int, codewords):
    """post at 0 iterations is the quantized prior: Cal_MSA_Q(x) with step 1,
    q = 4 (max 7): round-half-up of |x|, clipped, sign restored; -0.0 -> 0."""
    x = np.array([0.0, -0.0, 0.49, 0.5, -0.5, 1.49, -2.5, 6.6, 7.5, 100.0, -100.0])
    llr = np.tile(np.where(codewords[0] == 1, -L49, L49), (1, 1))
    llr[0, :len(x)] = x
    _, post, it, _ = og_int.decode_int_batch(llr, 0, 2, precision=4, step=1.0)
    assert post[0, :len(x)].tolist() == [0, 0, 0, 1, -1, 1, -3, 7, 7, 7, -7]


@pytest.mark.gpu
@pytest.mark.parametrize("algo,prec,step,beta,p,max_iter", [
    ("qmsa", 6, 0.5, 0, 0.002, 30), ("qmsa", 6, 0.5, 1, 0.004, 30), ("qmsa", 4, 1.0, 1, 0.01, 15),
    ("qmsa", 8, 0.25, 0, 0.02, 10), ("qmsa", 3, 2.0, 0, 0.003, 25),
    ("gallager_a", 0, 0, 0, 0.002, 20), ("gallager_b1", 0, 0, 0, 0.004, 20), ("gallager_b2", 0, 0, 0, 0.01, 20),
])
def test_int_decoders_bitexact(gpu, G, og_int, codewords, algo, prec, step, beta, p, max_iter):
    a = {"qmsa": 2, "gallager_a": 3, "gallager_b1": 4, "gallager_b2": 5}[algo]
    B = 200
    llr = synth.bsc_llrs(codewords, 0, B, seed=40 + a, p=p)
    # erasures / small LLRs quantize to 0: exercises the tie hash
    llr[::7, 100:140] = 0.0
    llr[::5, 300:320] *= 0.05
    kw = dict(msa_precision=prec, msa_step=step, msa_offset=beta, tie_seed=1234) if algo == "qmsa" else {}
    h, post, it, v = G.decode(llr, max_iter=max_iter, algo=algo, post="llr", **kw)
    rh, rpost, rit, rv = og_int.decode_int_batch(llr, max_iter, a, precision=prec or 6, step=step or 0.5, beta=beta,
                                                 seed=1234, threads=8)
    assert np.array_equal(it, rit)
    assert np.array_equal(v, rv.astype(bool))
    assert np.array_equal(h, rh)
    assert np.array_equal(post, rpost)
    # chunking does not change the tie hash (keyed by the index in the call)
    h2, post2, it2, _ = G.decode(llr, max_iter=max_iter, algo=algo, post="llr", chunk=64, **kw)
    assert np.array_equal(h2, h) and np.array_equal(it2, it) and np.array_equal(post2, post)


@pytest.mark.gpu
def test_int_decoders_irregular_graph(gpu, oracle_mod, tmp_path):
    rng = np.random.default_rng(11)
    M, N = 50, 150
    rows, cols = [], []
    for j in range(N - 1):
        for i in rng.choice(M - 1, size=int(rng.integers(1, 6)), replace=False):
            rows.append(int(i)); cols.append(j)
    G = gpu.Graph.from_edges(M, N, rows, cols)
    path = tmp_path / "irr.pchk"
    G.save_pchk(str(path))
    og = oracle_mod.OracleGraph(str(path))
    llr = rng.normal(1.5, 2.0, size=(70, N))
    llr[:, :4] = 0.0
    for a in (2, 3, 4, 5):
        name = {2: "qmsa", 3: "gallager_a", 4: "gallager_b1", 5: "gallager_b2"}[a]
        kw = dict(msa_precision=5, msa_step=0.75, msa_offset=1, tie_seed=7) if a == 2 else {}
        h, post, it, v = G.decode(llr, max_iter=25, algo=name, post="llr", **kw)
        rh, rpost, rit, rv = og.decode_int_batch(llr, 25, a, precision=5, step=0.75, beta=1, seed=7, threads=4)
        assert np.array_equal(h, rh) and np.array_equal(it, rit) and np.array_equal(post, rpost), name


@pytest.mark.gpu
def test_reference_decoder_type_ints(gpu, G, codewords):
    """algo as an int is the reference's decoder_type (DNA_main.cpp:41-53):
    1 runs Gallager A like 'gallager_a' and bin/ldpc's decoder_type 1, 20/21/22
    the float min-sum, 0 BP."""
    llr = synth.bsc_llrs(codewords, 0, 64, seed=5, p=0.004)
    for t, name in ((1, "gallager_a"), (2, "gallager_b1"), (3, "gallager_b2"), (20, "msa"), (21, "msa"), (0, "bp")):
        a = G.decode(llr, max_iter=20, algo=t, post=None)
        b = G.decode(llr, max_iter=20, algo=name, post=None)
        for x, y in zip(a, b):
            if x is not None:
                assert np.array_equal(np.asarray(x), np.asarray(y)), (t, name)


def test_oracle_quantizer_out_of_range(og_int, codewords):
    """Cal_MSA_Q (dec.cpp:1708-1746) on values outside the int range: the
    reference's x86 build converts them to INT_MIN (cvttsd2si's "integer
    indefinite"), whatever their sign, and its sign step keeps INT_MIN -- so
    an infinite, NaN or huge LLR enters quantized min-sum as a strongly
    negative prior (bit decided 1), never as +max_value.  The oracle spells
    this out (no C undefined behaviour); a 0-iteration decode shows the
    quantized priors directly."""
    llr = np.where(codewords[:1] == 1, -L49, L49)
    bad = {3: np.inf, 4: -np.inf, 5: np.nan, 6: 1e300, 7: -1e300, 8: 2.0 ** 31 * 0.5, 9: 2.0 ** 30 - 0.5}
    for j, x in bad.items():
        llr[0, j] = x
    _, post, _, _ = og_int.decode_int_batch(llr, 0, 2, precision=6, step=0.5)
    int_min = float(-2 ** 31)
    for j in (3, 4, 5, 6, 7, 8):
        assert post[0, j] == int_min, (j, post[0, j])
    assert post[0, 9] == 31.0  # in range: clipped to max_value = 2^(6-1) - 1


@pytest.mark.gpu
def test_int_decoders_out_of_range_inputs(gpu, G, og_int, codewords):
    """The same out-of-range LLRs through every integer decoder on the GPU,
    bit-exact against the oracle (quantizer + wrapping int sums,
    kernels_int.hpp)."""
    llr = synth.bsc_llrs(codewords, 0, 70, seed=33, p=0.004)
    rng = np.random.default_rng(4)
    for x in (np.inf, -np.inf, np.nan, 1e300, -1e300, 2.0 ** 31 * 0.5):
        idx = rng.integers(0, llr.size, 40)
        llr.flat[idx] = x
    for algo, name in ((2, "qmsa"), (3, "gallager_a"), (4, "gallager_b1"), (5, "gallager_b2")):
        for beta in ((0, 1) if algo == 2 else (0,)):
            rh, rpost, rit, rv = og_int.decode_int_batch(llr, 15, algo, precision=6, step=0.5, beta=beta)
            h, post, it, v = G.decode(llr, max_iter=15, algo=name, post="llr", msa_offset=beta)
            assert np.array_equal(h, rh) and np.array_equal(it, rit) and np.array_equal(v, rv.astype(bool)), name
            assert np.array_equal(post, rpost), name
