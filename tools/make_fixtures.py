#!/usr/bin/env python3
"""Copy the reference's DATA fixtures for the decode path into tests/golden/.

Run in the build container (where /root/reference exists):

    python tools/make_fixtures.py

* decode_n18432_m2048_final.pchk -- the parity-check matrix (byte copy; the
  copies in decoder/ and ex_decoder/ are identical).
* codewords_272.npz -- the 272 true codewords codeword_n18432_m1860_{1..272}.txt,
  bit-packed ([272][18432] bits).
These are data files the reference holds (inputs / known answers), not source.
"""
import os
import shutil
import sys

import numpy as np

REF = os.environ.get("LDPC_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def main():
    src = os.path.join(REF, "ex_decoder")
    if not os.path.isdir(src):
        sys.exit(f"reference data not found under {src}")
    os.makedirs(OUT, exist_ok=True)
    shutil.copyfile(os.path.join(src, "decode_n18432_m2048_final.pchk"),
                    os.path.join(OUT, "decode_n18432_m2048_final.pchk"))
    cws = []
    for i in range(1, 273):
        with open(os.path.join(src, f"codeword_n18432_m1860_{i}.txt")) as f:
            cws.append(np.array(f.read().split(), dtype=np.uint8))
    cw = np.stack(cws)
    assert cw.shape == (272, 18432) and set(np.unique(cw)) <= {0, 1}
    np.savez_compressed(os.path.join(OUT, "codewords_272.npz"), bits=np.packbits(cw, axis=1), n=cw.shape[1],
                        count=cw.shape[0])
    print("wrote", OUT)


if __name__ == "__main__":
    main()
