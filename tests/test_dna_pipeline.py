"""The in-process decoder.py LDPC stage (dna_pipeline.py)."""
import math

import numpy as np
import pytest

import dna_pipeline as P
import synth


def _oracle_fn(og):
    def fn(llr, max_iter):
        h, _, _, _ = og.decode_batch(llr, max_iter, threads=8, want_post=False)
        return h
    return fn


def test_rescale_matches_reference_loop():
    """decoder.py:603-609 element loop, incl. the str() round trip of the re_soft file."""
    rng = np.random.default_rng(0)
    llr = np.round(rng.normal(0, 3, 500)) * synth.LLR_UNIT
    llr[::7] = 0.0
    eps, eps2 = 0.02, 0.0185
    ref = []
    for x in llr.tolist():
        if x == 0:
            ref.append(x)
        else:
            ref.append(x * math.log((1 - eps2 + 0.0005) / (eps2 - 0.0005)) / math.log((1 - eps) / eps))
    ref = np.array([float(str(v)) for v in ref])
    assert np.array_equal(P.rescale(llr, eps, eps2), ref)


def test_trial_flow_on_oracle(og, codewords):
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)[:16]
    res = P.decode_trial(llr, codewords[:16], decode_fn=_oracle_fn(og))
    assert res["first_success"] + len(res["fail_first"]) == 16
    assert res["fail_first"] == [14]  # golden case g5: codeword 14 fails at 200 iterations
    assert res["second_iterations"] >= 1
    txt = P.report(res)
    assert "First decoding result" in txt and "Second decoding failure index" in txt


def test_faithful_vs_tracking_semantics(og, codewords):
    """With two failures the reference's per-codeword reset keeps only the last."""
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)[:16]
    bad = synth.bsc_llrs(codewords, 0, 2, seed=5, p=0.03)  # hopeless: never decodes
    llr = np.concatenate([bad, llr[2:]])
    fn = _oracle_fn(og)
    f = P.decode_trial(llr, codewords[:16], decode_fn=fn, max_iter=20)
    t = P.decode_trial(llr, codewords[:16], decode_fn=fn, max_iter=20, faithful=False)
    assert 1 in f["fail_first"] and 2 in f["fail_first"]
    assert set(t["fail_second"]) >= {1, 2}
    assert len(f["fail_second"]) <= 1


@pytest.mark.gpu
def test_trial_gpu_equals_oracle(G, og, codewords):
    """Config 2 (272-codeword DNA batch) through the full first + second decode
    flow: GPU and oracle give identical outcomes."""
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)
    a = P.decode_trial(llr, codewords, decode_fn=P.gpu_decode_fn(G))
    b = P.decode_trial(llr, codewords, decode_fn=_oracle_fn(og))
    for k in ("first_success", "second_success", "fail_first", "fail_second", "second_iterations",
              "first_errors", "second_errors", "erasure_index"):
        assert a[k] == b[k], k
    assert np.array_equal(a["hard"], b["hard"])
    assert a["first_success"] < 272  # the near-threshold batch exercises the second decode
