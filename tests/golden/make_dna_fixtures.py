"""Regenerate tests/golden/dna_fixtures.npz from DATA files of the reference
(read as text; nothing from the reference is imported or executed).

* quality_hist   -- counts of the per-read quality characters in
                    ex_decoder/72000_RS_Q_{0..9}.txt (the matching read files
                    72000_RS_*.txt are missing blobs).  synth.dna_reads draws
                    read qualities from it.
* strand_index   -- the 16-bit index of each of the 18432 strands, read from
                    the first 8 nt of original files/final_DNA.txt
                    (A/C/G/T = 0..3, most significant first).  Pins
                    dna_llr.strand_indices(), the restatement of
                    ex_decoder/pre_processing.py:29-89.
* payload_sha256 -- sha256 of the 18432 payloads (nt 16..151) joined by
                    "\\n".  Pins the strand <-> codeword-bit mapping
                    (strand j = bit j of codewords 1..272, DNA2binary order).

    python tests/golden/make_dna_fixtures.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "dna_fixtures.npz")


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present")
    counts = np.zeros(128, np.int64)
    for k in range(10):
        with open(os.path.join(REF, "ex_decoder", f"72000_RS_Q_{k}.txt")) as f:
            for line in f:
                line = line.rstrip("\n")
                if line:
                    counts[ord(line[0])] += 1
    strands = open(os.path.join(REF, "original files", "final_DNA.txt")).read().split()
    assert len(strands) == 18432 and all(len(s) == 152 for s in strands)
    idx = np.array([int("".join(str("ACGT".index(c)) for c in s[:8]), 4) for s in strands], np.int32)
    sha = hashlib.sha256("\n".join(s[16:] for s in strands).encode()).hexdigest()
    np.savez_compressed(OUT, quality_hist=counts, strand_index=idx,
                        payload_sha256=np.array(sha))
    print(f"wrote {OUT}: {int(counts.sum())} qualities, {len(idx)} strand indices")


if __name__ == "__main__":
    main()
