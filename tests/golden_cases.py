"""Golden-vector cases: inputs are regenerated deterministically
(counter-based BSC hash, or stored int8 count differences for the DNA-like
sets); expected outputs live in tests/golden/oracle_goldens.npz, produced by
tools/make_goldens.py from the oracle.

  g1_50 / g1_200  DNA-like, 72000 reads (the pipeline's coverage), codewords 1..16
  g5              DNA-like, 57000 reads (near threshold: mixed outcomes), 200 it
  g2              BSC p=0.02, 8 codewords, 50 it (never converges)
  g3              BSC p=0.004, 8 codewords, 50 it (converges in a few)
  g4              min-sum, BSC p=0.002, 8 codewords, 50 it
"""
import numpy as np

import synth

SEED = 2026
CASES = {
    # name: (kind, params, max_iter, algo)
    "g1_50": ("dna", "g1_k", 50, 0),
    "g1_200": ("dna", "g1_k", 200, 0),
    "g5": ("dna", "g5_k", 200, 0),
    "g2": ("bsc", 0.02, 50, 0),
    "g3": ("bsc", 0.004, 50, 0),
    "g4": ("bsc", 0.002, 50, 1),
}


def dna_k(reads: int, seed: int, count: int = 16) -> np.ndarray:
    cw = synth.load_codewords()
    llr = synth.dna_like_llrs(cw, seed=seed, reads=reads)[:count]
    k = np.rint(llr / synth.LLR_UNIT).astype(np.int8)
    assert np.array_equal(k.astype(np.float64) * synth.LLR_UNIT, llr)
    return k


def inputs(case: str, z=None):
    kind, prm, max_iter, algo = CASES[case]
    if kind == "dna":
        k = z[prm]
        llr = k.astype(np.float64) * synth.LLR_UNIT
    else:
        cw = synth.load_codewords()
        llr = synth.bsc_llrs(cw, 0, 8, seed=SEED, p=prm)
    return np.ascontiguousarray(llr), max_iter, algo
