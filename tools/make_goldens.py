#!/usr/bin/env python3
"""Generate tests/golden/oracle_goldens.npz from the CPU oracle.

    make -C oracle && python tools/make_goldens.py

Stored per case (tests/golden_cases.py): bit-packed hard decisions,
iteration counts, valid flags and a
SHA-256 of the fp64 posterior bytes (BP: raw likelihood ratio P; MSA: L) for
exact checks.  DNA-like inputs are stored as int8 count differences k
(LLR = k * ln49, decoder.py:314).
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "dna-ldpc-codes_amd"), os.path.join(ROOT, "oracle")]

import golden_cases  # noqa: E402
import oracle  # noqa: E402
import synth  # noqa: E402


def main():
    g = oracle.OracleGraph(synth.PCHK)
    out = {"g1_k": golden_cases.dna_k(72000, 0), "g5_k": golden_cases.dna_k(57000, 1)}
    for case in golden_cases.CASES:
        llr, max_iter, algo = golden_cases.inputs(case, out)
        h, post, it, v = g.decode_batch(llr, max_iter, algo=algo, post_mode=1 if algo == 0 else 0, threads=8)
        out[case + "_hard"] = np.packbits(h, axis=-1)
        out[case + "_iters"] = it
        out[case + "_valid"] = v
        out[case + "_post_sha"] = np.array(hashlib.sha256(post.tobytes()).hexdigest())
        print(case, "iters", it.tolist(), "valid", v.tolist())
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "oracle_goldens.npz"), **out)


if __name__ == "__main__":
    main()
