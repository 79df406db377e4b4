"""DNA soft-input construction, CPU part: the strand
index set and payload mapping against the reference's final_DNA.txt (data
fixture), the oracle restatement on hand-derived cases, and the library's
host-only soft-file writer (Python repr tokens) against the oracle's text.
GPU parity of the kernels is in test_dna_llr_gpu.py."""
import hashlib
import math
import os

import numpy as np
import pytest

import dna_llr
import synth
from conftest import GOLDEN

L49 = math.log(49.0)


@pytest.fixture(scope="module")
def dfx():
    return np.load(os.path.join(GOLDEN, "dna_fixtures.npz"), allow_pickle=False)


@pytest.fixture(scope="module")
def dorc():
    import dna_llr_oracle  # test infrastructure (oracle/)
    return dna_llr_oracle


def test_strand_indices_match_final_dna(dfx):
    s = dna_llr.strand_indices()
    assert len(s) == 18432 and np.all(np.diff(s) > 0)
    assert np.array_equal(s, dfx["strand_index"])


def test_payloads_match_final_dna(dfx, codewords):
    pay = synth.strand_payloads(codewords)
    assert pay.shape == (18432, 136)
    sha = hashlib.sha256(b"\n".join(row.tobytes() for row in pay)).hexdigest()
    assert sha == str(dfx["payload_sha256"])


def test_quality_hist(dfx):
    q = dfx["quality_hist"]
    assert q.sum() > 600000 and q[ord("C")] > q.sum() // 2


def test_oracle_edit_dist_known_answers(dorc):
    cases = [("", "", 0), ("", "ACGT", 4), ("ACGT", "", 4), ("kitten", "sitting", 3), ("ACGT", "ACGT", 0),
             ("ACGT", "TGCA", 4), ("AAAA", "AA", 2), ("GATTACA", "GCATGCU", 4)]
    for a, b, d in cases:
        assert dorc.edit_dist(a, b) == d


def test_oracle_edit_dist_against_independent_dp(dorc):
    rng = np.random.default_rng(0)
    for _ in range(40):
        a = "".join(rng.choice(list("ACGT"), int(rng.integers(0, 40))))
        b = "".join(rng.choice(list("ACGTN"), int(rng.integers(0, 40))))
        # Wagner-Fischer with numpy rows (same recurrence, different code)
        prev = np.arange(len(b) + 1)
        for i, ca in enumerate(a, 1):
            cur = np.empty_like(prev)
            cur[0] = i
            for j, cb in enumerate(b, 1):
                cur[j] = prev[j - 1] if ca == cb else 1 + min(prev[j - 1], prev[j], cur[j - 1])
            prev = cur
        assert dorc.edit_dist(a, b) == prev[-1]


def test_oracle_dna2binary(dorc):
    assert dorc.dna2binary(["ACGT"]) == ["0 0 0 1 1 0 1 1 "]
    assert dorc.dna2binary(["AN-"]) == ["0 0 2 2 2 2 "]
    assert dorc.dna2binary(["AC", "GTTT"]) == ["0 0 0 1 ", "1 0 1 1 "]  # len(cands[0]) for all


def test_oracle_strand_cases(dorc):
    L = L49
    A = "A" * 136
    # two identical reads: every bit 2 zeros -> 2L except bit 271 q-filter
    v = dorc.strand_llrs([A, A], [60, 40], L, None)
    assert v[0] == 2 * L and v[271] == 1 * L
    # single short read: only bit 271, by the low bit of the last base, if q > 63
    v = dorc.strand_llrs(["ACG"], [64], L, None)
    assert v[271] == L and all(x == 0 and type(x) is int for x in v[:271])
    v = dorc.strand_llrs(["ACT"], [64], L, None)
    assert v[271] == -L
    v = dorc.strand_llrs(["ACT"], [63], L, None)
    assert v[271] == 0 and type(v[271]) is int
    # tie at bit 271 with both reads q >= 53: int 0
    B = A[:-1] + "C"
    v = dorc.strand_llrs([A, B], [60, 66], L, None)
    assert v[271] == 0 and type(v[271]) is int and v[270] == 2 * L
    # ragged, no close pair -> dropped
    rng = np.random.default_rng(1)
    r1 = "".join(rng.choice(list("ACGT"), 136))
    r2 = "".join(rng.choice(list("ACGT"), 100))
    assert dorc.strand_llrs([r1, r2], [67, 67], L, dna_llr.pad_align) is None
    # ragged, padded alignment of length 138 -> failure path, last chars counted with q > 63
    v = dorc.strand_llrs([A + "GA", A[:-1], A[:-3] + "C"], [67, 70, 40], L, dna_llr.pad_align)
    # failed rows: "..GA" q67 -> 'A' (low 0), "A..A--" q70 -> '-' (counts as 1), q40 skipped
    assert v[271] == 0.0 and type(v[271]) is float
    assert all(x == 0 and type(x) is int for x in v[:271])


def test_pad_align():
    out = dna_llr.pad_align(["AC", "ACGT", "A"])
    assert out == [(2, "A---"), (1, "ACGT"), (0, "AC--")]


def test_py_float_repr_matches_python(L):
    rng = np.random.default_rng(2)
    vals = [0.0, -0.0, 1.0, -1.0, 0.1, 1e-4, 9.999e-5, 1e-5, 1e15, 1e16, 1.5e16, 123456789012345.6,
            float("inf"), float("-inf"), 5e-324, 1.7976931348623157e308, 2 * L49, -2 * L49, L49, 0.5,
            3.0e-7, 12345.678]
    vals += [k * L49 for k in range(-300, 301)]
    vals += list(rng.standard_normal(300) * 10.0 ** rng.integers(-20, 20, 300))
    vals += list(rng.random(200))
    for v in vals:
        assert dna_llr.py_float_repr(v) == repr(float(v)), v
    assert dna_llr.py_float_repr(float("nan")) == "nan"


def test_soft_file_writer_matches_oracle_text(L, dorc, codewords, tmp_path):
    """Writer parity on an oracle-built LLR set (no GPU): the same values
    and int pattern written by the library and by str() in the oracle."""
    reads = synth.dna_reads(codewords, seed=3, n_reads=400, sub=0.01, ins=0.004, dele=0.004, p_bad_index=0.05)
    reads = synth.dna_reads_edge_cases(codewords, reads, seed=4)
    by_strand = dorc.build_llr(*reads, dna_llr.strand_indices().tolist(), 0.02, dna_llr.pad_align)
    S = len(by_strand)
    llr = np.array([[float(v[i]) for v in by_strand] for i in range(272)])
    mask = np.array([[type(v[i]) is int for v in by_strand] for i in range(272)], np.uint8)
    res = dna_llr.LlrResult(llr=llr, int_mask=mask, kind=np.zeros(S, np.int32))
    res.write_soft_files(str(tmp_path), 400)
    for i in (0, 1, 100, 270, 271):
        got = (tmp_path / f"soft400_n18432_m1860_{i + 1}.txt").read_text()
        assert got == dorc.soft_file_text(by_strand, i), i
    assert len(os.listdir(tmp_path)) == 272
