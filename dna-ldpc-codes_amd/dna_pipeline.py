"""In-process LDPC stage of the DNA-storage decoder.

Reproduces the decode loop of the reference's ex_decoder/decoder.py without
the 272+ `ldpc.exe` processes and soft/dec text files:

* first decode (decoder.py:553-581): every codeword's LLR vector decoded with
  max_iter 200; the genie check against the true codeword gives `fail_DNA`
  (1-based indices) and the per-strand `re_decode` counts (output bit !=
  input hard decision), from which `erasure_index` = strands with > 140
  (decoder.py:590, def_func.re_index);
* second decode (decoder.py:592-664): while failures remain and eps2 > 0.001,
  rescale the ORIGINAL LLRs of the failed codewords by
  ``(x * ln((1-eps2+0.0005)/(eps2-0.0005))) / ln((1-eps)/eps)`` (zeros kept),
  lower eps2 by 0.0005 and re-decode.  The reference resets ``fail_DNA2 = []``
  inside its per-codeword loop (decoder.py:659-661), so only the LAST re-decoded
  codeword's outcome survives an iteration; this module keeps that behaviour
  (``faithful=True``, the default) or tracks every failure (``faithful=False``).

All decodes of one stage go to the GPU in ONE batched call.  `decode_fn` is
injectable so tests can run the identical flow on the CPU oracle.

The first decode's LLRs are count differences times ln((1-eps)/eps)
(decoder.py:314): when the caller has them as int8 codes (dna_llr's
LlrResult.codes, made by the LLR kernel itself), the GPU decode_fn takes the
codes and the 256-entry table k * unit (Graph.decode_codes) -- the same
doubles, without the host lattice pass over the fp64 matrix that the fp64
entry needs.  The second decode's rescaled LLRs are off that lattice and keep
the fp64 entry.
"""
from __future__ import annotations

import math
import time
from typing import Callable, Dict, List, Optional

import numpy as np

DecodeFn = Callable[[np.ndarray, int], np.ndarray]  # (llr [B][N], max_iter) -> hard [B][N]
# optional attribute `codes` of a DecodeFn: (codes int8 [B][N], table [256], max_iter) -> hard [B][N],
# the decode of llr = table[codes + 128]


def code_table(unit: float) -> np.ndarray:
    """table[k + 128] = k * unit: the doubles (count_0 - count_1) * unit of decoder.py:314."""
    return np.arange(-128, 128, dtype=np.float64) * unit


def gpu_decode_fn(graph=None, algo="bp") -> DecodeFn:
    import ldpc_amd
    g = graph if graph is not None else ldpc_amd.graph(ldpc_amd.default_pchk())

    def fn(llr: np.ndarray, max_iter: int) -> np.ndarray:
        hard, _, _, _ = g.decode(llr, max_iter=max_iter, algo=algo, post=None)
        return hard

    def codes(k: np.ndarray, table: np.ndarray, max_iter: int) -> np.ndarray:
        hard, _, _, _ = g.decode_codes(k, table, max_iter=max_iter, algo=algo, post=None)
        return hard

    fn.codes = codes
    return fn


def rescale(llr: np.ndarray, eps: float, eps2: float) -> np.ndarray:
    """decoder.py:603-609: x -> x * ln((1-eps2+.0005)/(eps2-.0005)) / ln((1-eps)/eps), 0 kept."""
    num = math.log((1 - eps2 + 0.0005) / (eps2 - 0.0005))
    den = math.log((1 - eps) / eps)
    return np.where(llr == 0, llr, (llr * num) / den)


def decode_trial(llr: np.ndarray, codewords: np.ndarray, eps: float = 0.02, max_iter: int = 200,
                 decode_fn: Optional[DecodeFn] = None, faithful: bool = True,
                 codes: Optional[np.ndarray] = None) -> Dict:
    """Run the LDPC part of one decoder.py trial.  llr: [n_cw][N] (row i = soft
    file i+1), codewords: [n_cw][N] true codewords (the genie).  codes
    (optional, int8 [n_cw][N]): the count differences with llr == codes *
    ln((1-eps)/eps) exactly, as the producer guarantees (dna_llr.build_llr);
    a decode_fn with a `codes` attribute then decodes them for the first
    decode."""
    decode_fn = decode_fn or gpu_decode_fn()
    llr = np.ascontiguousarray(llr, dtype=np.float64)
    n_cw, N = llr.shape
    t0 = time.perf_counter()
    if codes is not None and hasattr(decode_fn, "codes"):
        if codes.shape != llr.shape or codes.dtype != np.int8:
            raise ValueError("codes must be int8 with the shape of llr")
        hard = decode_fn.codes(codes, code_table(math.log((1 - eps) / eps)), max_iter)
    else:
        hard = decode_fn(llr, max_iter)
    t_first = time.perf_counter() - t0
    errors = (hard != codewords).sum(axis=1)
    fail = [i + 1 for i in range(n_cw) if errors[i] != 0]
    re_decode = (hard != (llr < 0)).sum(axis=0)  # decoder.py:565-574
    erasure_index = [j for j in range(N) if re_decode[j] > 140]

    fail2: List[int] = list(fail)
    iter_sec = 0
    eps2 = eps - 0.0005
    second_errors = {}
    t1 = time.perf_counter()
    while fail2 and eps2 > 0.001:
        iter_sec += 1
        batch = np.stack([rescale(llr[i - 1], eps, eps2) for i in fail2])
        eps2 = eps2 - 0.0005
        h2 = decode_fn(batch, max_iter)
        new: List[int] = []
        for k, i in enumerate(fail2):
            v = int((h2[k] != codewords[i - 1]).sum())
            second_errors[i] = v
            if faithful:
                new = []  # decoder.py:659-661 resets the list per codeword
            if v != 0:
                new.append(i)
            if v == 0:
                hard[i - 1] = h2[k]
        fail2 = new
    t_second = time.perf_counter() - t1
    return {
        "first_success": n_cw - len(fail), "second_success": n_cw - len(fail2), "n": n_cw,
        "fail_first": fail, "fail_second": fail2, "second_iterations": iter_sec,
        "first_errors": {i: int(errors[i - 1]) for i in fail}, "second_errors": second_errors,
        "erasure_index": erasure_index, "hard": hard, "t_first_s": t_first, "t_second_s": t_second,
    }


def trial_from_reads(reads, codewords: np.ndarray, eps: float = 0.02, max_iter: int = 200, align_fn=None,
                     decode_fn: Optional[DecodeFn] = None, faithful: bool = True, device: int = 0) -> Dict:
    """decoder.py:120-664 for one trial: reads (index values, payloads,
    qualities) -> LLRs on the GPU (dna_llr.build_llr) -> first and second
    decode.  Adds the LLR stage's time and strand statistics to the result."""
    import dna_llr
    t0 = time.perf_counter()
    built = dna_llr.build_llr(*reads, eps=eps, align_fn=align_fn, device=device)
    t_llr = time.perf_counter() - t0
    res = decode_trial(built.llr, codewords, eps=eps, max_iter=max_iter, decode_fn=decode_fn, faithful=faithful,
                       codes=built.codes)
    res.update(t_llr_s=t_llr, n_erased_strands=int(len(built.erased)), n_reads_valid=built.n_reads_valid,
               llr=built)
    return res


def report(res: Dict, rs: int = 72000, total_time: Optional[float] = None, threshold: Optional[int] = None,
           newline: str = "\n") -> str:
    """The o_/x_ result-file body (decoder.py:668-727).  total_time adds the
    'Total time: %f sec' line; threshold adds the 'Re-decoding threshold
    (number): %d' line of the committed o_72000_7_*_result.txt files (written
    by a revision of decoder.py that had it, on Windows: newline='\r\n')."""
    ok = not res["fail_second"]
    fmt = lambda xs: ("None" if not xs else " ".join(str(v) for v in xs) + " ")  # noqa: E731
    n = res["n"]
    lines = ["=" * 78, " " * 31 + "Results" + " " * 40, "=" * 78]
    if total_time is not None:
        lines.append("Total time: %f sec" % total_time)
    lines.append(f"Random Sampling Number: {rs}")
    if threshold is not None:
        lines.append("Re-decoding threshold (number): %d" % threshold)
    if ok:
        lines += ["Decoding success", "", "First decoding result:   %d/%d" % (res["first_success"], n),
                  "Second decoding result:  %d/%d" % (res["second_success"], n),
                  "Second decoding iteration number:  %d" % res["second_iterations"]]
    else:
        lines += ["Decoding failure", "", "First decoding result:\t%d/%d" % (res["first_success"], n),
                  "Second decoding result:\t%d/%d" % (res["second_success"], n)]
    lines += ["First decoding failure index: " + fmt(res["fail_first"]),
              "Second decoding failure index: " + fmt(res["fail_second"])]
    return newline.join(lines) + newline


def result_file_name(res: Dict, rs: int, trial: int, eps: float, threshold: Optional[int] = None) -> str:
    """o_/x_ file name of decoder.py:668-671; with threshold, the
    o_<rs>_<threshold>_<trial>_<eps> form of the committed result files."""
    head = "o" if not res["fail_second"] else "x"
    if threshold is None:
        return head + "_%d_%d_%f_result.txt" % (rs, trial, eps)
    return head + "_%d_%d_%d_%f_result.txt" % (rs, threshold, trial, eps)
