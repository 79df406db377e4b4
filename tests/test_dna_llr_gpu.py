"""DNA soft-input construction on the GPU against the oracle restatement
(oracle/dna_llr_oracle.py): edit distances exact, LLRs bit-exact (fp64
bytes), the int-0 pattern identical, soft files byte-identical.  The
aligner is the shared `pad_align` stand-in on both sides (MUSCLE is out of
scope)."""
import math

import numpy as np
import pytest

import dna_llr
import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dorc():
    import dna_llr_oracle
    return dna_llr_oracle


def _oracle_arrays(by_strand):
    llr = np.array([[float(v[i]) for v in by_strand] for i in range(272)])
    mask = np.array([[type(v[i]) is int for v in by_strand] for i in range(272)], np.uint8)
    return llr, mask


def test_edit_distance_kernel(gpu, dorc):
    rng = np.random.default_rng(9)
    seqs = [""]
    for n in [1, 5, 60, 136, 137, 150, 300, 800]:
        seqs.append("".join(rng.choice(list("ACGT"), n)))
    base = "".join(rng.choice(list("ACGT"), 136))
    for k in range(20):  # near-duplicates of one strand
        s = list(base)
        for _ in range(int(rng.integers(0, 20))):
            op, p = int(rng.integers(0, 3)), int(rng.integers(0, len(s)))
            if op == 0:
                s[p] = "ACGTN-"[int(rng.integers(0, 6))]
            elif op == 1:
                s.insert(p, "ACGT"[int(rng.integers(0, 4))])
            else:
                del s[p]
        seqs.append("".join(s))
    n = len(seqs)
    pairs = np.array([(a, b) for a in range(n) for b in range(n) if (a + b) % 3 == 0 or a < 3], np.int32)
    got = dna_llr.edit_distance(seqs, pairs)
    for (a, b), d in zip(pairs, got):
        if len(seqs[a]) * len(seqs[b]) > 40000:
            continue  # the O(n^2) Python oracle is checked on the shorter pairs
        assert d == dorc.edit_dist(seqs[a], seqs[b]), (a, b)
    long_pairs = [(a, b) for (a, b) in pairs if len(seqs[a]) * len(seqs[b]) > 40000]
    for a, b in long_pairs[:6]:
        assert got[list(map(tuple, pairs)).index((a, b))] == dorc.edit_dist(seqs[a], seqs[b])


@pytest.mark.parametrize("case", [
    dict(seed=21, n_reads=3000, sub=0.01, ins=0.003, dele=0.003, p_bad_index=0.05),
    dict(seed=22, n_reads=20000, sub=0.02, ins=0.002, dele=0.002, p_bad_index=0.02),
])
def test_build_llr_bitexact_vs_oracle(gpu, dorc, codewords, tmp_path, case):
    reads = synth.dna_reads(codewords, **case)
    reads = synth.dna_reads_edge_cases(codewords, reads, seed=case["seed"] + 100)
    res = dna_llr.build_llr(*reads, eps=0.02, align_fn=dna_llr.pad_align)
    by_strand = dorc.build_llr(*reads, dna_llr.strand_indices().tolist(), 0.02, dna_llr.pad_align)
    llr, mask = _oracle_arrays(by_strand)
    assert np.array_equal(res.llr.view(np.uint64), llr.view(np.uint64))
    assert np.array_equal(res.int_mask, mask)
    # the kernel's int8 codes give back every LLR bit for bit through the table k * ln49
    assert res.codes is not None
    assert np.array_equal(res.code_table()[res.codes.astype(np.int64) + 128].view(np.uint64), llr.view(np.uint64))
    # every strand kind occurs
    assert set(np.unique(res.kind).tolist()) == {0, 1, 2, 3}
    assert res.n_pairs > 0 and res.n_aligned_strands > 0
    res.write_soft_files(str(tmp_path), case["n_reads"])
    for i in (0, 135, 271):
        got = (tmp_path / f"soft{case['n_reads']}_n18432_m1860_{i + 1}.txt").read_text()
        assert got == dorc.soft_file_text(by_strand, i)


def test_build_llr_without_aligner_fails_loudly(gpu, codewords):
    reads = synth.dna_reads(codewords, seed=5, n_reads=50)
    reads = synth.dna_reads_edge_cases(codewords, reads, seed=6)
    with pytest.raises(RuntimeError):
        dna_llr.build_llr(*reads, eps=0.02, align_fn=None)


def test_full_scale_reads_decode(gpu, codewords):
    """72000 reads (the reference's --rs), substitutions only, through
    reads -> GPU LLRs -> first/second decode: every codeword decodes (the
    o_72000_*_result.txt outcome "First decoding result: 272/272")."""
    import dna_pipeline
    reads = synth.dna_reads(codewords, seed=7, n_reads=72000, sub=0.01)
    res = dna_pipeline.trial_from_reads(reads, codewords, eps=0.02, align_fn=dna_llr.pad_align)
    built = res["llr"]
    assert built.llr.shape == (272, 18432)
    assert res["first_success"] == 272 and not res["fail_second"]
    # the count rule: LLR / ln49 is an integer count difference everywhere,
    # and the kernel's int8 codes are those differences (the first decode's input)
    k = built.llr / math.log(49.0)
    assert np.array_equal(k, np.rint(k))
    assert built.codes is not None and built.codes.dtype == np.int8
    assert np.array_equal(built.code_table()[built.codes.astype(np.int64) + 128], built.llr)
    assert 0 < res["n_erased_strands"] < 18432 * 0.05


def test_build_llr_codes_beyond_int8(gpu, codewords):
    """A strand read more than 127 times has count differences that no int8
    code holds: ldpc_dna_llr_codes reports exact = 0, LlrResult.codes is
    None, and the pipeline's first decode takes the fp64 entry instead."""
    import dna_pipeline
    idx, seqs, quals = synth.dna_reads(codewords, seed=31, n_reads=4000)
    pay = synth.strand_payloads(codewords)
    s0 = int(dna_llr.strand_indices()[0])
    idx += [s0] * 140
    seqs += [pay[0].tobytes().decode()] * 140
    quals += [70] * 140
    res = dna_llr.build_llr(idx, seqs, quals, eps=0.02, align_fn=dna_llr.pad_align)
    assert res.codes is None
    k = res.llr / math.log(49.0)
    assert np.abs(k).max() > 127 and np.array_equal(k, np.rint(k))
    t = dna_pipeline.trial_from_reads((idx, seqs, quals), codewords, eps=0.02, align_fn=dna_llr.pad_align)
    assert t["first_success"] + len(t["fail_first"]) == 272
