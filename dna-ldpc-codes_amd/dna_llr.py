"""DNA soft-input construction: sequenced reads -> the 272 x 18432 LLR matrix
(the step before the first decode).

Host mirror of ex_decoder/decoder.py:103-519; the arithmetic runs in HIP
(csrc/dna.hip through the C ABI):

1. reads whose decoded index is not a strand index are dropped, the rest are
   grouped by strand in read order (decoder.py:103-118, a stable sort);
2. each strand is classified (decoder.py:149-497):
   * no reads                                  -> all LLRs int 0 (:507-510)
   * one read shorter than the payload         -> only the last bit (:240-263)
   * one read, or several all of payload length -> count over the reads
   * several reads of mixed length ("ragged")  -> pairwise edit distance
     (GPU, ldpc_dna_edit_distance) keeps the reads with some partner at
     distance < 15 (:171-178); none -> no LLRs; otherwise the kept reads go
     to the aligner (MUSCLE in the reference, :181-186 -- an injected
     `align_fn` here) and aligned rows of payload length are counted; if
     none survives, only the last bit is set from the failed rows (:266-282);
3. ldpc_dna_llr turns the classified rows into LLRs, bit-major
   ([codeword i][strand j] = soft file i+1, entry j), which is exactly the
   decoder's input layout, plus the int-0 mask the soft-file writer needs.

Differences from the reference (deliberate): when the LAST strand holding
reads is ragged with no close pair, or is a single short read, the reference
keeps looping past the end of decimal_index and raises IndexError; here that
strand simply gets the same LLRs as any other strand of its kind.  The
aligner is injected: MUSCLE is out of scope, so the parity tests
hand the same deterministic `pad_align` stand-in to the product and to the
oracle.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

PAYLOAD_NT = 136          # decoder.py:156 (len == 136)
N_STRANDS = 18432         # decoder.py:509 (range(18432))
ED_THRESHOLD = 15         # decoder.py:175 (temp < 15)

KIND_NONE, KIND_COUNT, KIND_SHORT, KIND_ALIGN_FAILED = 0, 1, 2, 3

AlignFn = Callable[[List[str]], List[Tuple[int, str]]]


def strand_indices() -> np.ndarray:
    """The 18432 strand index values in ascending order
    (ex_decoder/pre_processing.py:29-89): every 14-bit value i whose 7
    nucleotides satisfy nt[2] != nt[3] and nt[5] != nt[6] is kept; the r-th
    kept value yields (i << 2) | (j << 1) | ((popcount(r) + j) & 1) for
    j = 0, 1 -- the parity uses the running count r of kept values, as the
    reference's sum(index[i]) does (pre_processing.py:76-78)."""
    i = np.arange(1 << 14, dtype=np.int64)
    nt = [(i >> (12 - 2 * k)) & 3 for k in range(7)]
    kept = i[(nt[2] != nt[3]) & (nt[5] != nt[6])]
    r = np.arange(len(kept), dtype=np.int64)
    pop = np.zeros_like(r)
    x = r.copy()
    while x.any():
        pop += x & 1
        x >>= 1
    out = np.empty(2 * len(kept), np.int64)
    out[0::2] = (kept << 2) | (pop & 1)
    out[1::2] = (kept << 2) | 2 | ((pop + 1) & 1)
    return out


def pad_align(seqs: Sequence[str]) -> List[Tuple[int, str]]:
    """Deterministic stand-in for the MUSCLE call (NOT an aligner): every
    sequence right-padded with '-' to the longest length, records returned
    in reverse input order (MUSCLE also reorders its output records)."""
    n = max((len(s) for s in seqs), default=0)
    return [(k, seqs[k] + "-" * (n - len(seqs[k]))) for k in reversed(range(len(seqs)))]


@dataclass
class LlrResult:
    llr: np.ndarray                # [2*PAYLOAD_NT][S] float64 (soft file i+1 = row i)
    int_mask: np.ndarray           # same shape, uint8: 1 = int 0 in the reference
    kind: np.ndarray               # [S] int32 strand classification
    n_reads_valid: int = 0
    n_pairs: int = 0               # edit-distance pairs evaluated on the GPU
    n_aligned_strands: int = 0
    erased: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))  # strands with no LLRs
    # the count differences: llr == codes * unit exactly (decoder.py:297-314);
    # None when some |count difference| > 127 (no int8 code)
    codes: Optional[np.ndarray] = None  # [2*PAYLOAD_NT][S] int8
    unit: float = 0.0                   # ln((1-eps)/eps)

    def code_table(self) -> np.ndarray:
        """table[k + 128] = k * unit: with `codes`, the input of
        Graph.decode_codes (the same doubles as llr)."""
        return np.arange(-128, 128, dtype=np.float64) * self.unit

    def write_soft_files(self, directory: str, rs: int):
        """soft<rs>_n18432_m1860_<i>.txt, i = 1..272 (decoder.py:511-516)."""
        import ldpc_amd
        L = ldpc_amd.lib()
        llr = np.ascontiguousarray(self.llr)
        mask = np.ascontiguousarray(self.int_mask)
        ldpc_amd._check(L.ldpc_write_soft_files(os.fsencode(directory), int(rs), llr.ctypes.data_as(C.c_void_p),
                                                mask.ctypes.data_as(C.c_void_p), llr.shape[0], llr.shape[1]))


def _lib():
    import ldpc_amd
    L = ldpc_amd.lib()
    if not getattr(L, "_dna_bound", False):
        vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
        L.ldpc_dna_llr.argtypes = [i32, vp, vp, vp, vp, i32, C.c_double, vp, vp, i32]
        L.ldpc_dna_llr_codes.argtypes = [i32, vp, vp, vp, vp, i32, C.c_double, vp, vp, vp, vp, i32]
        L.ldpc_dna_edit_distance.argtypes = [vp, vp, vp, i64, vp, vp, i64, vp, i32]
        L.ldpc_write_soft_files.argtypes = [C.c_char_p, i32, vp, vp, i32, i32]
        L.ldpc_py_float_repr.argtypes = [C.c_double, C.c_char_p, i32]
        L._dna_bound = True
    return ldpc_amd, L


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def edit_distance(seqs: Sequence[str], pairs: np.ndarray, device: int = 0) -> np.ndarray:
    """Levenshtein distance of each (a, b) index pair, on the GPU
    (def_func.edit_dist, def_func.py:10-26)."""
    mod, L = _lib()
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    enc = [s.encode("latin-1") for s in seqs]
    lens = np.array([len(b) for b in enc], np.int32)
    offs = np.zeros(len(enc), np.int64)
    if len(enc) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.int64)
    buf = np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy()
    a = np.ascontiguousarray(pairs[:, 0])
    b = np.ascontiguousarray(pairs[:, 1])
    out = np.zeros(len(pairs), np.int32)
    mod._check(L.ldpc_dna_edit_distance(_p(buf), _p(offs), _p(lens), len(enc), _p(a), _p(b), len(pairs),
                                        _p(out), device))
    return out


def py_float_repr(v: float) -> str:
    """The library's Python-repr formatter (used by the soft-file writer)."""
    mod, L = _lib()
    buf = C.create_string_buffer(40)
    n = L.ldpc_py_float_repr(float(v), buf, 40)
    if n < 0:
        mod._check(n)
    return buf.value.decode()


@dataclass
class LlrPlan:
    """Host classification handed to ldpc_dna_llr."""
    kind: np.ndarray      # [S] int32
    row_ptr: np.ndarray   # [S+1] int64
    rows: np.ndarray      # [max(R,1)][PAYLOAD_NT] uint8
    row_q: np.ndarray     # [max(R,1)] int32
    n_reads_valid: int
    n_pairs: int
    n_aligned_strands: int


def plan_llr(index_vals: Sequence[int], seqs: Sequence[str], quals: Sequence[int],
             align_fn: Optional[AlignFn] = None, device: int = 0, strands: Optional[np.ndarray] = None,
             distance_fn=None) -> LlrPlan:
    """Group and classify the reads (decoder.py:103-497 control flow).
    Pairwise distances of ragged strands come from the GPU
    (`distance_fn` defaults to edit_distance on `device`)."""
    distance_fn = distance_fn or (lambda sq, pr: edit_distance(sq, pr, device))
    sidx = strand_indices() if strands is None else np.asarray(strands, np.int64)
    S = len(sidx)
    iv = np.asarray(index_vals, np.int64)
    if not (len(iv) == len(seqs) == len(quals)):
        raise ValueError("index_vals, seqs and quals must have the same length")
    pos = np.searchsorted(sidx, iv)
    ok = pos < S
    ok[ok] = sidx[pos[ok]] == iv[ok]
    read_ids = np.nonzero(ok)[0]
    read_ids = read_ids[np.argsort(pos[read_ids], kind="stable")]  # decoder.py:116
    rpos = pos[read_ids]
    q_all = np.asarray(quals, np.int64)
    lens = np.fromiter((len(seqs[r]) for r in read_ids), np.int64, len(read_ids))
    cnt = np.bincount(rpos, minlength=S)
    start = np.zeros(S + 1, np.int64)
    start[1:] = np.cumsum(cnt)

    kind = np.zeros(S, np.int32)
    all_full = np.ones(S, bool)
    np.logical_and.at(all_full, rpos, lens == PAYLOAD_NT)
    single = cnt == 1
    first_len = np.zeros(S, np.int64)
    first_len[cnt > 0] = lens[start[:-1][cnt > 0]]
    kind[single & (first_len < PAYLOAD_NT)] = KIND_SHORT
    kind[single & (first_len >= PAYLOAD_NT)] = KIND_COUNT
    multi = cnt > 1
    kind[multi & all_full] = KIND_COUNT
    ragged = np.nonzero(multi & ~all_full)[0]

    # ragged strands: all pairs i < k per strand -> one GPU batch
    pair_list, pair_strand = [], []
    for s in ragged:
        n = int(cnt[s])
        ii, kk = np.triu_indices(n, 1)
        pair_list.append(np.stack([start[s] + ii, start[s] + kk], 1))
        pair_strand.append(np.full(len(ii), s))
    rows_of = {}  # strand -> (row strings, qualities) for aligned / failed strands
    n_pairs = 0
    n_aligned = 0
    if pair_list:
        pairs = np.concatenate(pair_list)
        n_pairs = len(pairs)
        # pair indices refer to positions in the strand-sorted read list
        local = [seqs[r] for r in read_ids]
        d = distance_fn(local, pairs)
        close = d < ED_THRESHOLD
        ps = np.concatenate(pair_strand)
        for s in ragged:
            m = close & (ps == s)
            sel = np.unique(pairs[m].ravel())  # decoder.py:176-178 (np.unique: sorted)
            if len(sel) == 0:
                kind[s] = KIND_NONE  # decoder.py:179-188
                continue
            if align_fn is None:
                raise RuntimeError("ragged strands need an aligner (align_fn); MUSCLE is out of scope")
            cand = [local[i] for i in sel]
            cq = q_all[read_ids[sel]]
            aligned, aq, err, eq = [], [], [], []
            for order, a in align_fn(cand):  # decoder.py:195-214
                if len(a) != PAYLOAD_NT:
                    err.append(a[-1] if a else "")
                    eq.append(int(cq[order]))
                    continue
                aligned.append(a)
                aq.append(int(cq[order]))
            n_aligned += 1
            if aligned:
                kind[s] = KIND_COUNT
                rows_of[s] = (aligned, aq)
            else:
                kind[s] = KIND_ALIGN_FAILED
                rows_of[s] = (err, eq)

    # rows: PAYLOAD_NT bytes each (kinds 2/3: byte 0 = last base)
    row_count = np.zeros(S, np.int64)
    plain_count = (kind == KIND_COUNT) & ~np.isin(np.arange(S), list(rows_of.keys()))
    row_count[plain_count] = cnt[plain_count]
    row_count[kind == KIND_SHORT] = 1
    for s, (rws, _) in rows_of.items():
        row_count[s] = len(rws)
    row_ptr = np.zeros(S + 1, np.int64)
    row_ptr[1:] = np.cumsum(row_count)
    R = int(row_ptr[-1])
    rows = np.full((max(R, 1), PAYLOAD_NT), ord("-"), np.uint8)
    row_q = np.zeros(max(R, 1), np.int32)

    # plain count strands: the reads' first PAYLOAD_NT bases, vectorised
    pc = np.nonzero(plain_count)[0]
    if len(pc):
        sel_reads = np.concatenate([np.arange(start[s], start[s + 1]) for s in pc])
        dst = np.concatenate([np.arange(row_ptr[s], row_ptr[s + 1]) for s in pc])
        blob = np.frombuffer("".join(seqs[read_ids[r]][:PAYLOAD_NT] for r in sel_reads).encode("latin-1"),
                             np.uint8)
        rows[dst] = blob.reshape(-1, PAYLOAD_NT)
        row_q[dst] = q_all[read_ids[sel_reads]]
    for s in np.nonzero(kind == KIND_SHORT)[0]:
        r = read_ids[start[s]]
        sq = seqs[r]
        if not sq and q_all[r] > 63:
            raise ValueError(f"empty read on strand {s} with quality > 63 (the reference indexes its last bit)")
        rows[row_ptr[s], 0] = ord(sq[-1]) if sq else ord("-")
        row_q[row_ptr[s]] = q_all[r]
    for s, (rws, qs) in rows_of.items():
        for k, (txt, q) in enumerate(zip(rws, qs)):
            if kind[s] == KIND_COUNT:
                rows[row_ptr[s] + k] = np.frombuffer(txt.encode("latin-1"), np.uint8)
            else:
                rows[row_ptr[s] + k, 0] = ord(txt) if txt else ord("-")
            row_q[row_ptr[s] + k] = q

    return LlrPlan(kind=kind, row_ptr=row_ptr, rows=rows, row_q=row_q, n_reads_valid=len(read_ids),
                   n_pairs=n_pairs, n_aligned_strands=n_aligned)


def build_llr(index_vals: Sequence[int], seqs: Sequence[str], quals: Sequence[int], eps: float = 0.02,
              align_fn: Optional[AlignFn] = None, device: int = 0,
              strands: Optional[np.ndarray] = None) -> LlrResult:
    """Reads (decoded index value, payload sequence, quality) -> LlrResult.
    `strands` defaults to strand_indices(); align_fn answers the MUSCLE call
    for ragged strands (required only if such strands have close pairs)."""
    mod, L = _lib()
    plan = plan_llr(index_vals, seqs, quals, align_fn, device, strands)
    S = len(plan.kind)
    unit = math.log((1 - eps) / eps)  # decoder.py:297
    llr = np.zeros((2 * PAYLOAD_NT, S), np.float64)
    mask = np.zeros((2 * PAYLOAD_NT, S), np.uint8)
    codes = np.zeros((2 * PAYLOAD_NT, S), np.int8)
    exact = C.c_int32(0)
    mod._check(L.ldpc_dna_llr_codes(S, _p(plan.kind), _p(plan.row_ptr), _p(plan.rows), _p(plan.row_q), PAYLOAD_NT,
                                    unit, _p(llr), _p(mask), _p(codes), C.byref(exact), device))
    return LlrResult(llr=llr, int_mask=mask, kind=plan.kind, n_reads_valid=plan.n_reads_valid,
                     n_pairs=plan.n_pairs, n_aligned_strands=plan.n_aligned_strands,
                     erased=np.nonzero(plan.kind == KIND_NONE)[0], codes=codes if exact.value else None, unit=unit)
