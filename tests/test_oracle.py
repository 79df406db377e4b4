"""CPU tests: the oracle against the reference's own fixtures and code.

Pins (DESIGN.md "Oracle"):
  * graph loader + syndrome: oracle == the reference's own mod2sparse.cpp /
    rcode.cpp / check.cpp, compiled unmodified into oracle/_ref (only where
    /root/reference exists -- skipped elsewhere);
  * all 272 true codewords satisfy H c = 0 (reference fixture);
  * BP / min-sum: the reference's only correctness signal is the genie check
    against the true codeword (decoder.py:575-581); converging inputs must
    decode to the true codeword;
  * regression: tests/golden/oracle_goldens.npz (made by tools/make_goldens.py).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, PCHK, pack


def test_graph_shape(og):
    assert (og.M, og.N, og.E) == (2048, 18432, 147456)
    assert og.regular() == (8, 1, 72, 1)  # CheckRegular dec.cpp:138-189


def test_graph_matches_reference_linked_lists(oracle_mod, og):
    if not oracle_mod.ref_available():
        pytest.skip("oracle/_ref not built (reference sources absent)")
    r = oracle_mod.RefGraph(PCHK)
    deg, cols = r.rows(og.E + 8)
    assert np.array_equal(deg, np.diff(og.row_ptr)) and np.array_equal(cols, og.col_idx)
    cdeg, rows = r.cols(og.E + 8)
    rowof = np.repeat(np.arange(og.M), np.diff(og.row_ptr))
    assert np.array_equal(cdeg, np.diff(og.col_ptr)) and np.array_equal(rows, rowof[og.col_edge])


def test_syndrome_matches_reference(oracle_mod, og):
    if not oracle_mod.ref_available():
        pytest.skip("oracle/_ref not built (reference sources absent)")
    r = oracle_mod.RefGraph(PCHK)
    rng = np.random.default_rng(5)
    for _ in range(8):
        x = (rng.random(og.N) < rng.random()).astype(np.uint8)
        c1, p1 = og.check(x)
        c2, p2 = r.check(x)
        assert c1 == c2 and np.array_equal(p1, p2)


def test_true_codewords_are_codewords(og, codewords):
    assert codewords.shape == (272, 18432)
    for c in codewords:
        assert og.check(c)[0] == 0


def test_noiseless_decode_is_identity(og, codewords):
    # LLR = +-ln49 with no flips: valid at n = 0 for both decoders
    import synth
    llr = np.where(codewords[:4] == 1, -synth.LLR_UNIT, synth.LLR_UNIT)
    for algo in (0, 1):
        h, _, it, v = og.decode_batch(llr, 50, algo=algo, threads=4)
        assert (it == 0).all() and v.all() and np.array_equal(h, codewords[:4])


def test_genie_dna_batch(og, codewords):
    """decoder.py:575-581 genie check on DNA-like inputs (first 32 codewords)."""
    import synth
    llr = synth.dna_like_llrs(codewords, seed=0)[:32]
    h, _, it, v = og.decode_batch(llr, 200, threads=8)
    assert v.all()
    assert np.array_equal(h, codewords[:32])
    assert it.max() <= 10


def test_bsc_low_noise_converges(og, codewords):
    import synth
    llr = synth.bsc_llrs(codewords, 0, 8, seed=2026, p=0.004)
    h, _, it, v = og.decode_batch(llr, 50, threads=8)
    assert v.all() and np.array_equal(h, codewords[np.arange(8) % 272])
    llr = synth.bsc_llrs(codewords, 0, 4, seed=2026, p=0.002)
    h, _, it, v = og.decode_batch(llr, 50, algo=1, threads=4)
    assert v.all() and np.array_equal(h, codewords[:4])


def test_bsc_high_noise_never_converges(og, codewords):
    import synth
    llr = synth.bsc_llrs(codewords, 0, 4, seed=2026, p=0.02)
    _, _, it, v = og.decode_batch(llr, 50, threads=4, want_post=False)
    assert (it == 50).all() and not v.any()


def test_max_iter_zero(og, codewords):
    import synth
    llr = synth.bsc_llrs(codewords, 0, 2, seed=1, p=0.01)
    h, post, it, v = og.decode_batch(llr, 0, threads=2)
    assert (it == 0).all()
    assert np.array_equal(h, (np.exp(llr) < 1).astype(np.uint8))  # Init: dblk = LR < 1
    np.testing.assert_allclose(post, llr, rtol=0, atol=1e-12)


def _goldens():
    path = os.path.join(GOLDEN, "oracle_goldens.npz")
    if not os.path.exists(path):
        pytest.skip("oracle_goldens.npz not generated")
    return np.load(path, allow_pickle=False)


@pytest.mark.parametrize("case", ["g1_50", "g1_200", "g2", "g3", "g4"])
def test_oracle_regression_goldens(og, case):
    import golden_cases
    z = _goldens()
    llr, max_iter, algo = golden_cases.inputs(case, z)
    h, post, it, v = og.decode_batch(llr, max_iter, algo=algo, post_mode=1 if algo == 0 else 0, threads=8)
    assert np.array_equal(pack(h), z[case + "_hard"])
    assert np.array_equal(it, z[case + "_iters"])
    assert np.array_equal(v, z[case + "_valid"])
    assert hashlib.sha256(post.tobytes()).hexdigest() == str(z[case + "_post_sha"])
