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
    k = dna_like_counts(codewords, seed=seed, reads=reads, sub=sub)
    unit = math.log((1 - eps) / eps)
    llr = k.astype(np.float64) * unit  # int * double, as (count_0-count_1)*math.log(...)
    return np.ascontiguousarray(llr)


def dna_like_codes(codewords: np.ndarray, seed: int = 0, reads: int = 72000, sub: float = 0.01) -> np.ndarray:
    """The count differences of dna_like_llrs as int8 codes (dna_like_llrs ==
    codes * ln((1-eps)/eps)); ValueError if one does not fit."""
    k = dna_like_counts(codewords, seed=seed, reads=reads, sub=sub)
    if k.size and np.abs(k).max() > 127:
        raise ValueError("a count difference exceeds the int8 code range")
    return np.ascontiguousarray(k.astype(np.int8))


def dna_like_counts(codewords: np.ndarray, seed: int = 0, reads: int = 72000, sub: float = 0.01) -> np.ndarray:
    """Count differences count_0 - count_1 [n_cw][N] (int64) of the DNA batch."""
    n_cw, N = codewords.shape
    if n_cw % 2:
        raise ValueError("codewords come in nucleotide pairs (bits 2k, 2k+1 of a strand)")
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
    return np.ascontiguousarray((zeros - ones).T)  # [n_cw][N] count difference


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


# --- sequenced reads for the LLR-construction stage -----
DNA_FIXTURES = os.path.join(GOLDEN, "dna_fixtures.npz")
_BASES = np.frombuffer(b"ACGT", np.uint8)


def quality_hist() -> np.ndarray:
    """Counts of per-read quality characters (ord) from the reference's
    72000_RS_Q_{0..9}.txt (tests/golden/dna_fixtures.npz)."""
    return np.load(DNA_FIXTURES, allow_pickle=False)["quality_hist"]


def strand_payloads(codewords: np.ndarray) -> np.ndarray:
    """[N][n_cw/2] uint8 ASCII: strand j's payload, nucleotide k = bits
    (2k, 2k+1) of codewords (DNA2binary order, def_func.py:97-117)."""
    bits = codewords.T.astype(np.int64)
    return _BASES[2 * bits[:, 0::2] + bits[:, 1::2]]


def dna_reads(codewords: np.ndarray, seed: int = 0, n_reads: int = 72000, sub: float = 0.01,
              ins: float = 0.0, dele: float = 0.0, p_bad_index: float = 0.0,
              quality: np.ndarray = None):
    """Simulated random-sampled reads after index decoding: (index values,
    payload strings, qualities).  Strand uniformly at random (the reference's
    random sampling of `--rs` reads), per-base substitution / insertion /
    deletion, a fraction of reads with a random (mostly invalid) 16-bit
    index, quality = ord(char) drawn from the reference's quality histogram."""
    import dna_llr
    rng = np.random.default_rng(seed)
    pay = strand_payloads(codewords)
    N, nt = pay.shape
    sidx = dna_llr.strand_indices()
    strand = rng.integers(0, N, n_reads)
    idx = sidx[strand].copy()
    bad = rng.random(n_reads) < p_bad_index
    idx[bad] = rng.integers(0, 1 << 16, int(bad.sum()))
    qh = quality_hist() if quality is None else quality
    qvals = np.nonzero(qh)[0]
    quals = rng.choice(qvals, n_reads, p=qh[qvals] / qh[qvals].sum()).astype(np.int64)
    r = pay[strand].copy()
    m = rng.random(r.shape) < sub
    r[m] = _BASES[(np.searchsorted(_BASES, r[m]) + rng.integers(1, 4, int(m.sum()))) % 4]
    seqs = [row.tobytes().decode() for row in r]
    if ins > 0 or dele > 0:
        n_ins = rng.binomial(nt, ins, n_reads)
        n_del = rng.binomial(nt, dele, n_reads)
        for k in np.nonzero((n_ins > 0) | (n_del > 0))[0]:
            s = list(seqs[k])
            for _ in range(int(n_del[k])):
                if s:
                    del s[int(rng.integers(0, len(s)))]
            for _ in range(int(n_ins[k])):
                s.insert(int(rng.integers(0, len(s) + 1)), "ACGT"[int(rng.integers(0, 4))])
            seqs[k] = "".join(s)
    return idx.tolist(), seqs, quals.tolist()


def dna_reads_edge_cases(codewords: np.ndarray, reads, seed: int = 1):
    """Append reads that put the rarer per-strand shapes of decoder.py's loop
    on fresh strands: single short read (q > 63 and q <= 63), single long
    read, ragged strands with no close pair, ragged strands whose padded
    alignment is not payload length (alignment failure), payload-length
    ragged alignment, non-ACGT characters, and a bit-271 one-vs-one tie."""
    import dna_llr
    idx, seqs, quals = (list(x) for x in reads)
    rng = np.random.default_rng(seed)
    pay = strand_payloads(codewords)
    sidx = dna_llr.strand_indices()
    used = set(idx)
    free = [j for j in rng.permutation(len(sidx)) if int(sidx[j]) not in used]
    it = iter(free)

    def add(j, s, q):
        idx.append(int(sidx[j])); seqs.append(s); quals.append(int(q))

    for q in (70, 60, 67):  # single short read
        j = next(it); add(j, pay[j].tobytes().decode()[:100 + q % 7], q)
    j = next(it); add(j, pay[j].tobytes().decode() + "ACG", 67)  # single long read
    j = next(it)  # ragged, no close pair
    add(j, "".join(rng.choice(list("ACGT"), 136)), 67); add(j, "".join(rng.choice(list("ACGT"), 120)), 67)
    for _ in range(2):  # ragged, padded length 138 != 136 -> alignment failure (kind 3)
        j = next(it); p = pay[j].tobytes().decode()
        add(j, p + "GA", 67); add(j, p[:-1], 70); add(j, p[:-3] + "C", 40)
    for _ in range(2):  # ragged, padded length 136 -> aligned rows counted
        j = next(it); p = pay[j].tobytes().decode()
        add(j, p, 67); add(j, p[:-2], 66); add(j, p[:130], 55)
    j = next(it); p = pay[j].tobytes().decode()  # non-ACGT characters
    add(j, p[:50] + "N" + p[51:], 67); add(j, p[:10] + "-" + p[11:], 67)
    j = next(it); p = pay[j].tobytes().decode()  # tie at bit 271: one 0 vs one 1 among q >= 53
    last = "A" if p[-1] in "CT" else "C"
    add(j, p, 60); add(j, p[:-1] + last, 66); add(j, p, 40)
    return idx, seqs, quals
