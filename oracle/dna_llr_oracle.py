"""CPU restatement of the DNA soft-input construction -- TEST INFRASTRUCTURE
ONLY (tests/ may import it; the product never does).

Restates, with the reference's control flow, ex_decoder/decoder.py:103-519
(read filtering and sort :103-118, the strand loop :142-497, the zero fill and
sort :502-510, the soft-file tokens :511-516 via def_func.write_codeword
:54-57), def_func.edit_dist (def_func.py:10-26) and def_func.DNA2binary
(:97-117).  The external MUSCLE call (:181-186 / :356-361) is an injected
`align_fn(seqs) -> [(order, aligned)]`, exactly what the parsing loop
(:188-214) extracts from align_output.txt.

Parity status: the strand-index restatement is pinned by the reference's
final_DNA.txt (tests/golden/dna_fixtures.npz).  The loop itself is
"parity unpinned": the reference's read files (72000_RS_*.txt) are missing
blobs, its LLR outputs were never committed, and running the reference's
Python here was refused, so this restatement is checked only
against hand-derived cases (tests/test_dna_llr.py).

Returns the LLR matrix as Python values per (bit, strand): int 0 or float,
which is what str() turns into the soft-file tokens.
"""
from __future__ import annotations

import math
from typing import Callable, List, Sequence, Tuple


def edit_dist(str1: str, str2: str) -> int:
    """def_func.py:10-26 (full DP table)."""
    dp = [[0] * (len(str2) + 1) for _ in range(len(str1) + 1)]
    for i in range(1, len(str1) + 1):
        dp[i][0] = i
    for j in range(1, len(str2) + 1):
        dp[0][j] = j
    for i in range(1, len(str1) + 1):
        for j in range(1, len(str2) + 1):
            if str1[i - 1] == str2[j - 1]:
                dp[i][j] = dp[i - 1][j - 1]
            else:
                dp[i][j] = min(dp[i - 1][j - 1], dp[i - 1][j], dp[i][j - 1]) + 1
    return dp[-1][-1]


def dna2binary(cands: Sequence[str]) -> List[str]:
    """def_func.py:97-117: 'x y ' per base; the length of cands[0] is used
    for every candidate."""
    table = {"A": "0 0", "C": "0 1", "G": "1 0", "T": "1 1"}
    out = []
    for c in cands:
        b = ""
        for j in range(len(cands[0])):
            b = b + table.get(c[j], "2 2") + " "
        out.append(b)
    return out


def strand_llrs(cands: List[str], quals: List[int], L: float, align_fn, nbits: int = 272):
    """One strand (decoder.py:331-497 'else' branch).  Returns the 272 LLR
    values, or None when the strand is dropped (no close pair)."""
    llr = [0 for _ in range(nbits)]
    last = nbits - 1
    error_q = []
    if len(cands) != 1:
        if all(len(c) == nbits // 2 for c in cands):  # :340-349
            r_q = list(quals)
            llr_cand = dna2binary(cands)
        else:
            same_seq = []  # :352-358
            for i in range(len(cands)):
                for k in range(i + 1, len(cands)):
                    if edit_dist(cands[i], cands[k]) < 15:
                        same_seq.append(i)
                        same_seq.append(k)
            uniq = sorted(set(same_seq))
            r_cand = [cands[i] for i in uniq]
            q2 = [quals[i] for i in uniq]
            if not r_cand:  # :361-371
                return None
            r_q, aligned = [], []
            for order, a in align_fn(r_cand):  # :380-405
                if len(a) != nbits // 2:
                    error_q.append([q2[order], a[len(a) - 1]])
                    continue
                r_q.append(q2[order])
                aligned.append(a)
            llr_cand = dna2binary(aligned)
    else:
        r_q = list(quals)
        if len(cands[0]) < nbits // 2:  # :411-433
            b = dna2binary(cands)[0].replace(" ", "")
            if r_q[0] > 63:
                llr[last] = L if b[len(b) - 1] == "0" else -L
            return llr
        llr_cand = dna2binary(cands)
    for i in range(nbits):  # :437-485
        c0 = c1 = q0 = q1 = 0
        if len(llr_cand) == 0:
            for q, ch in error_q:
                if q > 63:
                    t = dna2binary(ch)[0].replace(" ", "")
                    if t[1] == "0":
                        c0 += 1
                    else:
                        c1 += 1
            llr[last] = (c0 - c1) * L
            break
        for j in range(len(llr_cand)):
            llr_cand[j] = llr_cand[j].replace(" ", "")
            if i == last and r_q[j] < 53:
                continue
            if llr_cand[j][i] == "0":
                c0 += 1
                q0 += r_q[j]
            else:
                c1 += 1
                q1 += r_q[j]
        if i == last and c0 == 1 and c1 == 1:
            if q0 < 53 and q1 >= 63:
                llr[i] = -2 * L
            elif q0 >= 63 and q1 < 53:
                llr[i] = 2 * L
            else:
                llr[i] = 0
        else:
            llr[i] = (c0 - c1) * L
    return llr


def build_llr(index_vals: Sequence[int], seqs: Sequence[str], quals: Sequence[int], decimal_index: Sequence[int],
              eps: float, align_fn: Callable[[List[str]], List[Tuple[int, str]]], nbits: int = 272):
    """decoder.py:103-510 -> per strand position j (ascending index value),
    the list of nbits LLR values (int 0 or float)."""
    L = math.log((1 - eps) / eps)
    valid = set(decimal_index)
    index_DNA = [(i, s, q) for i, s, q in zip(index_vals, seqs, quals) if i in valid]  # :103-112
    index_DNA = sorted(index_DNA, key=lambda x: x[0])  # :116
    by_index = {}
    for i, s, q in index_DNA:
        by_index.setdefault(i, ([], []))
        by_index[i][0].append(s)
        by_index[i][1].append(q)
    out = {}
    for i, (cands, qs) in by_index.items():
        v = strand_llrs(cands, qs, L, align_fn, nbits)
        if v is not None:
            out[i] = v
    zero = [0 for _ in range(nbits)]  # :502-505
    return [out.get(i, zero) for i in sorted(decimal_index)]


def soft_file_text(llr_by_strand, bit: int) -> str:
    """Soft file bit+1 (decoder.py:511-516 + def_func.write_codeword)."""
    return "".join(str(v[bit]) + " " for v in llr_by_strand)
