"""Input generators for the decode path (host side, numpy).

* ``dna_like_llrs`` -- SURVEY 8(d) config 2.  The reference's decoder input
  reads (72000_RS_*.txt) are missing blobs (.MISSING_LARGE_BLOBS:6-15), so the
  272-codeword DNA batch is rebuilt from the 272 true codewords with a seeded
  read simulator: strand j carries bit i of codeword i+1 (original
  files/final_DNA.txt payload, A/C/G/T = 00/01/10/11, def_func.DNA2binary
  def_func.py:97-117); per strand Poisson(72000/18432) reads, each nucleotide
  substituted with probability `sub` by a uniformly chosen other base; per-bit
  LLR = (count0 - count1) * ln((1-eps)/eps) exactly as decoder.py:314 computes
  it, and LLR 0 for strands without reads (decoder.py:514-517).
* ``bsc_llrs`` -- host replica of the device BSC generator
  (kernels.hpp k_gen_bsc) used for configs 3-5; tests check the device output
  against it bit for bit.
* ``load_codewords`` -- the 272 true codewords (bit-packed fixture).
"""
from __future__ import annotations

import math
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
PCHK = os.path.join(GOLDEN, "decode_n18432_m2048_final.pchk")
CODEWORDS = os.path.join(GOLDEN, "codewords_272.npz")

EPSILON = 0.02
LLR_UNIT = math.log((1 - EPSILON) / EPSILON)  # 3.8918202981106265 = ln 49 (decoder.py:314)


def load_codewords() -> np.ndarray:
    """[272][18432] uint8 -- codeword_n18432_m1860_{1..272}.txt."""
    z = np.load(CODEWORDS, allow_pickle=False)
    return np.unpackbits(z["bits"], axis=1, count=int(z["n"]))[: int(z["count"])].astype(np.uint8)


def dna_like_llrs(codewords: np.ndarray, seed: int = 0, reads: int = 72000, sub: float = 0.01,
                  eps: float = EPSILON) -> np.ndarray:
    """LLRs [n_cw][N] for the DNA batch (see module doc)."""
    n_cw, N = codewords.shape
    if n_cw % 2:
        raise ValueError("codewords come in nucleotide pairs (bits 2k, 2k+1 of a strand)")
    unit = math.log((1 - eps) / eps)
    rng = np.random.default_rng(seed)
    # strand j: nucleotides k = 0..n_cw/2-1, base = 2*bit(2k) + bit(2k+1)
    bits = codewords.T.astype(np.int64)  # [N][n_cw]
    base = 2 * bits[:, 0::2] + bits[:, 1::2]  # [N][n_nt]
    nreads = rng.poisson(reads / N, size=N)
    strand = np.repeat(np.arange(N), nreads)  # read -> strand
    rb = base[strand]  # [R][n_nt]
    mut = rng.random(rb.shape) < sub
    rb = np.where(mut, (rb + rng.integers(1, 4, size=rb.shape)) % 4, rb)
    rbits = np.empty((rb.shape[0], n_cw), np.int64)
    rbits[:, 0::2] = rb >> 1
    rbits[:, 1::2] = rb & 1
    ones = np.zeros((N, n_cw), np.int64)
    np.add.at(ones, strand, rbits)
    zeros = nreads[:, None] - ones
    k = (zeros - ones).T  # [n_cw][N] count difference
    llr = k.astype(np.float64) * unit  # int * double, as (count_0-count_1)*math.log(...)
    return np.ascontiguousarray(llr)


# --- counter-based BSC generator (bit-identical to kernels.hpp k_gen_bsc) ---
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return x ^ (x >> np.uint64(31))


def bsc_flips(b0: int, B: int, N: int, seed: int, p: float) -> np.ndarray:
    seedmix = _splitmix64(np.array([seed], np.uint64))[0]
    b = np.arange(b0, b0 + B, dtype=np.uint64)[:, None]
    j = np.arange(N, dtype=np.uint64)[None, :]
    u = _splitmix64(((b << np.uint64(24)) | j) ^ seedmix) >> np.uint64(11)
    return (u.astype(np.float64) * 2.0 ** -53) < p


def bsc_llrs(codewords: np.ndarray, b0: int, B: int, seed: int, p: float, mag: float = LLR_UNIT,
             as_lr: bool = False) -> np.ndarray:
    """[B][N] fp64: +-mag (or the host-exp'd LR) for codewords b0..b0+B-1 sent
    over a BSC(p); transmitted word = codewords[b mod n_cw]."""
    n_cw, N = codewords.shape
    idx = (np.arange(b0, b0 + B) % n_cw)
    y = codewords[idx] ^ bsc_flips(b0, B, N, seed, p).astype(np.uint8)
    if as_lr:
        return np.where(y == 1, math.exp(-mag), math.exp(mag))
    return np.where(y == 1, -mag, mag)
