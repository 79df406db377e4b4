#!/usr/bin/env python3
"""Benchmark: decoded codewords/s for the n=18432 / m=2048 BP decoder at 50
iterations (BASELINE.json metric), one process per GPU.

    python bench.py                       # N=1, 100k synthetic codewords per step
    python bench.py --gpus N              # N ranks: starts torch.distributed.run as a child
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Workload (SURVEY 8(d) config 3, weak-scaled per GPU by default): every
rank decodes its own contiguous shard of `--batch-per-gpu` codewords
[rank*B, (rank+1)*B) -- or, with `--global-batch G` (config 4: `--gpus 8
--global-batch 1000000`), its dist.shard of [0, G), "scaling": "strong" --
from the counter-based BSC(p=0.02) generator (transmitted word
codeword_n18432_m1860_{1 + b mod 272}, LLR = +-ln49, LR = exp(LLR) by the
host libm as DNA_main.cpp:1344 does).  The channel output sits in HBM as one
int8 code per bit (+-1, `--input code`, ldpc_engine_decode_codes with the
table code -> code * ln49), the form the DNA pipeline's count differences take
(decoder.py:314); `--input fp64` keeps fp64 LR / LLR values instead.  Both
decode the same values bit for bit.  p = 0.02 never converges, so every
codeword runs exactly 50 iterations.  Inputs are generated into HBM before the
timed region; a step = one full decode of the shard (init, 50 x [syndrome,
check, variable], final syndrome, hard-bit unpack, iteration counts).

No data-path collective: ranks only meet in a barrier, a MAX of their elapsed
times and a gather of their check counts (gloo, CPU tensors).  `value` = all
codewords of all ranks / max elapsed.

Correctness of the timed decode, on every rank: the oracle decodes a sample of
the rank's own shard -- its head (at N = 1 the cpu_baseline leg's sample, at
N > 1 about 8 codewords per host thread of the rank's share of the cores), its
last rows (the lane pool's drain) and 32 random interior rows -- and its hard
bits, iteration counts and valid flags must equal the GPU's; `check` in the
JSON line carries the per-rank counts and rows, and any mismatch exits
non-zero.

At N = 1 (unless --secondary 0) driver-timed secondary legs follow the
headline, each with its own oracle check, under "secondary": the headline on
fp64 input, the headline's kernels streaming from HBM (16384 codewords in one
pass, 38.7 GB of messages: the HBM-only roofline beside the headline's
Infinity-Cache-resident pool), config 2 (the 272-codeword DNA batch through
the host API ldpc_decode, median of 15 calls) and config 5 (1M codewords,
min-sum with early exit, 2 timed steps).

At N > 1, after the headline and every rank's check: rank 0 times the oracle
on all the host cores it may use while the other ranks wait in a barrier
(`cpu_baseline`, as at N = 1), and at N = 8 BASELINE config 4 follows as
"secondary.config4_1m_strong" -- 1M codewords split by dist.shard, 1 warm-up
+ 2 timed decodes (max over ranks), every rank's shard oracle-checked
(--config4 G forces a G-codeword leg at any N > 1).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "dna-ldpc-codes_amd")]

METRIC = "decoded codewords/sec (n=18432, m=2048, 50 BP iters) at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
# the engine's default columns per variable-phase wave (kernel instantiation
# names): 2 with coded priors in the resident pool or the compressed min-sum,
# else 4 (engine.hip var_cpw_for)
VAR_CPW, VAR_CPW_CODED = 4, 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch-per-gpu", type=int, default=100_000,
                    help="weak scaling: codewords per rank, rank r decodes [r*B, (r+1)*B)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many codewords split over the ranks by dist.shard (SURVEY 8(d) "
                         "config 4: --gpus 8 --global-batch 1000000 -> 125k per rank); 0 = weak scaling")
    ap.add_argument("--dump-dir", default="",
                    help="write each rank's outputs (shard start/size, iterations, valid flags, packed hard bits) "
                         "to <dir>/rank<r>.npz (tests)")
    ap.add_argument("--max-iter", type=int, default=50)
    ap.add_argument("--algo", default="bp", choices=["bp", "msa"])
    ap.add_argument("--p", type=float, default=0.02)
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--chunk", type=int, default=0, help="resident codewords per pass (0: auto)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--check-per-thread", type=int, default=16,
                    help="N > 1 (and --cpu-baseline 0): oracle-checked codewords per host thread of each rank")
    ap.add_argument("--group-tiles", type=int, default=None,
                    help="tiles per check/variable launch (unset or 0: engine default; < 0: the whole pass, as the ABI)")
    ap.add_argument("--nt", type=int, default=-1, help="nontemporal d-stream (-1: engine default)")
    ap.add_argument("--cont", type=int, default=-1, help="continuous batching / lane refill (-1: engine default)")
    ap.add_argument("--res", type=int, default=-1,
                    help="resident in-place pool of a few tiles (-1: engine default; BP / fp64 min-sum, continuous)")
    ap.add_argument("--var-cpw", type=int, default=0, help="columns per variable-phase wave (0: engine default 4)")
    ap.add_argument("--ffp", type=int, default=-1,
                    help="single-fill BP: first check from the prior (LDPC_SCHED_FIRST_FROM_PRIOR; -1: engine default)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-kernel HIP event timing")
    ap.add_argument("--secondary", type=int, default=1,
                    help="N = 1: also time the headline on fp64 input and streaming from HBM, config 5 (1M min-sum) "
                         "and config 2 (DNA batch, host API) after the headline")
    ap.add_argument("--msa-batch", type=int, default=1_000_000, help="config-5 secondary leg: codewords")
    ap.add_argument("--hbm-batch", type=int, default=16384,
                    help="HBM-streaming secondary leg: codewords in its one pass (0: skip the leg)")
    ap.add_argument("--input", default="code", choices=["code", "fp64"],
                    help="channel output in HBM: int8 codes + a 256-entry table (default) or fp64 LR / LLR")
    ap.add_argument("--workload", default="bsc", choices=["bsc", "dna272"],
                    help="bsc: SURVEY 8(d) configs 3-5 (default); dna272: config 2, the 272-codeword DNA batch")
    ap.add_argument("--config4", default="auto",
                    help="N > 1: BASELINE config 4 as a secondary leg after the headline -- G codewords strong-sharded "
                         "over the ranks (dist.shard), 1 warm-up + 2 timed decodes, every rank oracle-checked; "
                         "'auto' (default): G = 1000000 at N = 8 only; an integer G > 0 forces it at any N > 1; 0: off")
    return ap.parse_args()


def host_cpus() -> dict:
    """Host threads this process can run at once: the affinity mask, capped by
    a cgroup CPU quota when there is one (a one-GPU box: 16 of 256)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return {"effective": min(aff, quota) if quota else aff, "affinity": aff, "cgroup_quota_cpus": quota}


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / CPU baseline only
    return oracle


def oracle_check(og, llr_fn, gpu_out, algo, max_iter, ranges, threads):
    """Oracle vs GPU on shard rows `ranges`: (start, n) runs and / or arrays of
    row indices.  Returns (checked, mismatching rows, oracle seconds)."""
    checked, bad, el = 0, [], 0.0
    for rg in ranges:
        if isinstance(rg, tuple):
            start, n = rg
            if n <= 0:
                continue
            rows = np.arange(start, start + n)
            llr = llr_fn(start, n)
            h, it, v = gpu_out(start, n)
        else:
            rows = np.asarray(rg, dtype=np.int64)
            if rows.size == 0:
                continue
            llr = np.concatenate([llr_fn(int(r), 1) for r in rows])
            outs = [gpu_out(int(r), 1) for r in rows]
            h = np.concatenate([o[0] for o in outs])
            it = np.concatenate([np.asarray(o[1]) for o in outs])
            v = np.concatenate([np.asarray(o[2]) for o in outs])
        t = time.perf_counter()
        rh, _, rit, rv = og.decode_batch(llr, max_iter, algo=algo, threads=threads, want_post=False)
        el += time.perf_counter() - t
        for k, r in enumerate(rows):
            if not (np.array_equal(h[k], rh[k]) and it[k] == rit[k] and bool(v[k]) == bool(rv[k])):
                bad.append(int(r))
        checked += len(rows)
    return checked, bad, el


def tail_and_interior(B, lo, n_tail=32, n_interior=32, seed=0):
    """Rows of a shard [0, B) outside a checked head [0, lo): its last n_tail
    rows (the lane pool's drain) and n_interior random rows in between."""
    t0 = max(lo, B - n_tail)
    tail = np.arange(t0, B, dtype=np.int64)
    pool = np.arange(lo, t0, dtype=np.int64)
    interior = np.sort(np.random.default_rng(seed).choice(pool, min(n_interior, pool.size), replace=False)) \
        if pool.size else pool
    return tail, interior


def cpu_baseline(args, og, llr_fn, B, gpu_out, cpus):
    """The oracle (bit-exact C restatement of dec.cpp, 'port') on the host's
    cores, on a bounded sample of the same workload -- and the check of the
    timed GPU decode on every sampled codeword.  Returns (cpu_baseline, check)."""
    threads = cpus["effective"]
    algo = 0 if args.algo == "bp" else 1
    # calibrate with one codeword per thread, then size the sample for ~cpu_seconds
    n0 = min(threads, B)
    c0, bad0, t1 = oracle_check(og, llr_fn, gpu_out, algo, args.max_iter, [(0, n0)], threads)
    rounds = max(1, int(args.cpu_seconds / max(t1, 1e-3)))
    n = max(1, min(threads * rounds, B - n0))
    start = n0 if B > n0 else 0
    c1, bad1, el = oracle_check(og, llr_fn, gpu_out, algo, args.max_iter, [(start, n)], threads)
    # beyond the timed sample: the shard's drain (last rows) and its interior
    tail, inter = tail_and_interior(B, start + n, seed=args.seed)
    c2, bad2, _ = oracle_check(og, llr_fn, gpu_out, algo, args.max_iter, [tail, inter], threads)
    rows = {"head": [0, start + n], "tail": [int(tail[0]), B] if tail.size else None, "interior": inter.tolist()}
    cb = {"value": round(n / el, 3), "unit": "codewords/s", "cores": threads, "kind": "port",
          "per_core": round(n / el / threads, 3),
          "host": cpus,
          "sample": f"{n} codewords of the same BSC(p={args.p}) workload (indices {start}..{start + n - 1}), "
                    f"{args.max_iter} iters, oracle/ldpc_oracle.c on {threads} host threads: every CPU this process "
                    f"may use (the affinity mask lists {cpus['affinity']}, the cgroup CPU quota allows "
                    f"{cpus['cgroup_quota_cpus']}; more threads than the quota only time-slice it), {el:.1f} s"}
    return cb, (c0 + c1 + c2, bad0 + bad1 + bad2, rows)


def kernel_names(eng, algo, coded=False, cpw=None) -> dict:
    """Template instantiations of the check / variable kernels an engine
    launches (csrc/engine.hip launch_check / launch_var), as rocprofv3 names
    them (tools/pmc_summary.py short form); the variable kernels' last argument is
    PC, coded priors (coded input on a continuous schedule)."""
    msa = "true" if algo == "msa" else "false"
    pc = str(bool(coded) and eng.continuous).lower()
    if not cpw:  # the engine's default (an explicit --var-cpw names itself)
        cpw = VAR_CPW_CODED if pc == "true" and (eng.resident or eng.msa_compressed) else VAR_CPW
    elif eng.msa_compressed:
        cpw = min(cpw, 4)
    if eng.msa_compressed:
        nt = str(eng.nontemporal).lower()
        return {"check": f"k_check_msa_c<72,{nt}>",
                "variable": f"k_var_msa_c<72,8,{str(eng.continuous).lower()},{cpw},{nt},{pc}>"}
    chk = "k_check_msa" if algo == "msa" else "k_check_bp"
    if eng.resident:
        return {"check": f"{chk}<72,false,true>", "variable": f"k_var_m<{msa},8,false,true,{cpw},true,{pc}>"}
    nt = str(eng.nontemporal).lower()
    return {"check": f"{chk}<72,{nt},false>",
            "variable": f"k_var_m<{msa},8,{nt},{str(eng.continuous).lower()},{cpw},false,{pc}>"}


def algorithmic_bytes(eng, N, M, E) -> dict:
    """Algorithmic bytes per executed codeword-iteration, per kernel (SURVEY
    8(d))."""
    if eng.msa_compressed:
        # compressed min-sum: the check phase reads E v->c fp64 and writes per
        # row the min1 / min2 planes + a 16-bit meta word (NaN planes only when
        # NaN occurs); the variable phase reads the records and meta words,
        # N LLR and its columns' sign bytes, and writes E v->c fp64, the sign
        # bytes (N) and N/8 hard-bit ballots
        return {"check": 8.0 * E + 18.0 * M, "variable": 8.0 * E + 18.0 * M + 10.0 * N + N / 8.0}
    return {
        # check phase: read E v->c (d) + write E c->v (lr), fp64
        "check": 16.0 * E,
        # variable phase: read E lr + N LR, write E d + N/8 hard-bit ballots
        "variable": 16.0 * E + 8.0 * N + N / 8.0,
    }


def moved_bytes(eng, N, M, E, coded=False) -> dict:
    """Bytes each kernel moves per executed codeword-iteration: the
    algorithmic bytes, with the prior read as its 1-byte code instead of an
    fp64 value where the continuous schedules keep coded priors (DESIGN.md
    sec. 4.3)."""
    b = dict(algorithmic_bytes(eng, N, M, E))
    if coded and eng.continuous:
        b["variable"] -= 7.0 * N
    return b


MALL_BYTES = 256 * 2 ** 20  # MI355X Infinity Cache (MALL)


def bound_label(eng) -> str:
    """roofline.bound: where the dominant kernel's bytes come from.  The
    resident pool (~226 MB) lives in the 256 MB Infinity Cache, so its frac is
    of bytes served by HBM and the MALL together; every
    other schedule streams its messages from HBM."""
    return "hbm+mall (resident pool)" if eng.resident else "hbm"


def bound_detail(eng, coded=False, E=147456) -> str:
    note = (" Coded input: the variable kernel reads each column's prior as a 1-byte code (+ a 2 KB table), "
            "7 B per column and codeword-iteration fewer than the algorithmic (fp64 prior) bytes that `achieved` "
            "counts; `achieved_moved` counts the code." if coded and eng.continuous else "")
    return _bound_detail(eng, E) + note


def _bound_detail(eng, E=147456) -> str:
    if eng.msa_compressed:
        return ("compressed min-sum (DESIGN.md sec. 4.2, 6.1), v2c in column order: the check kernel gathers its "
                "8-tile group's v2c (604 MB, more than the 256 MB Infinity Cache) from HBM as 512-B segments; the "
                "variable kernel gathers the records and meta words from its XCD's L2 (one tile per XCD) and writes "
                "the group's fp64 v2c back nontemporally (row-block-major: per wave one 1-KB run into each of the 8 "
                "row-block streams), bounded by that store shape's measured ceiling (ceiling_measured); no MFMA")
    if eng.resident:
        return ("resident in-place pool sized to the 256 MB Infinity Cache: every message byte crosses the L2 -> "
                "fabric interface once per phase (PMC fabric bytes = 1.02-1.04 x algorithmic), served by HBM and the "
                "Infinity Cache; the DRAM-request counters count cache hits too on gfx950 (calibrated), so the cache "
                "share is not observable; no MFMA")
    tiles = -(-eng.cap // 64)  # tiles of one pass
    group = tiles if eng.group_tiles < 0 else min(eng.group_tiles, tiles)
    group_mb = group * 64 * E * 8 / 2 ** 20  # the group's fp64 c2v scratch
    if group >= tiles:
        return (f"one grouped pass over every tile ({tiles}): the c2v scratch ({group_mb:.0f} MB) and the v2c "
                "stream (nontemporal) both exceed the 256 MB Infinity Cache, so every message byte streams from "
                "HBM; memory-bound, no MFMA" if group_mb * 2 ** 20 > MALL_BYTES else
                f"one grouped pass over every tile ({tiles}): the c2v scratch ({group_mb:.0f} MB) fits the 256 MB "
                "Infinity Cache, the v2c stream goes to HBM (nontemporal); memory-bound, no MFMA")
    if group_mb * 2 ** 20 > MALL_BYTES:
        return (f"grouped schedule, {group} of {tiles} tiles per group: the group's c2v scratch ({group_mb:.0f} MB) "
                "exceeds the 256 MB Infinity Cache, so it streams from HBM between the phases, as does the v2c "
                "stream (nontemporal); memory-bound, no MFMA")
    return (f"grouped schedule, {group} of {tiles} tiles per group: the group's c2v scratch ({group_mb:.0f} MB) is "
            "meant to stay in the Infinity Cache between the phases, the v2c stream goes to HBM (nontemporal); "
            "memory-bound, no MFMA")


def find_traffic(kname):
    """L2 -> fabric bytes per codeword-iteration of this exact kernel
    instantiation from the newest committed PMC summary (profiles/r*/pmc_traffic.json)."""
    for tf in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True):
        tj = json.load(open(tf))
        per = tj.get("per_cw_iter_by_instantiation", {})
        if kname in per:
            return float(per[kname]), os.path.relpath(tf, ROOT)
    return None, None


def roofline(eng, G, st, cw_iters, coded=False, cpw=None) -> dict:
    """Roofline of the dominant kernel: algorithmic bytes per launch / its
    average launch duration (HIP events on the kernel's dispatch packet)."""
    N, M, E = G.N, G.M, G.E
    by_kernel = algorithmic_bytes(eng, N, M, E)
    moved = moved_bytes(eng, N, M, E, coded)
    names = kernel_names(eng, "msa" if eng.algo == 1 else "bp", coded, cpw)

    def avg_ms(k):
        return st[k]["ms"] / st[k]["sampled"] if st[k]["sampled"] else 0.0

    dom = max(("check", "variable"), key=lambda k: avg_ms(k) * st[k]["launches"])
    k_launch = max(1, st[dom]["launches"])
    k_avg = avg_ms(dom)
    bytes_per_launch = by_kernel[dom] * cw_iters / k_launch
    achieved = bytes_per_launch / (k_avg * 1e-3) / 1e9 if k_avg > 0 else None
    moved_per_launch = moved[dom] * cw_iters / k_launch
    achieved_moved = moved_per_launch / (k_avg * 1e-3) / 1e9 if k_avg > 0 else None
    it_ms = sum(avg_ms(k) * st[k]["launches"] for k in ("check", "variable", "syndrome"))
    iter_bytes = (32.0 * E + 10.0 * N) * cw_iters  # 32 E + 10 N per codeword-iteration
    iter_moved = (moved["check"] + moved["variable"]) * cw_iters
    per_cwi, traffic_src = find_traffic(names[dom])
    traffic = round(per_cwi * cw_iters / k_launch) if per_cwi else None
    # measured ceiling of the dominant kernel's access shape: the resident pool's in-place passes
    # (tools/cachebench, profiles/r2/cachebench.txt: one launch per in-place pass of the check kernel's shape
    # over a 192-224 MB working set), or the compressed min-sum's column-ordered v2c (tools/wrbench over the
    # 8-tile group's 604 MB): the variable kernel's stores and the check kernel's row gathers in exactly
    # the kernels' wave order over the row-block-major v2c of the DNA code (tools/wrbench "rb" shapes,
    # profiles/r4/wrbench_rb_604MB*.txt; the faster of two runs)
    ceiling, ceiling_src = None, None
    if eng.resident:
        ceiling, ceiling_src = 6780.0, ("tools/cachebench: in-place 72 x 512 B per wave, one launch per pass, "
                                        "192-224 MB working set (profiles/r2/cachebench.txt)")
    elif eng.msa_compressed and dom == "variable":
        ceiling, ceiling_src = 5079.6, ("tools/wrbench: the variable kernel's nontemporal v2c stores in its own "
                                        "wave order over the row-block-major 604 MB group "
                                        "(profiles/r4/wrbench_rb_604MB_run2.txt)")
    elif eng.msa_compressed:
        ceiling, ceiling_src = 6876.5, ("tools/wrbench: the check kernel's nontemporal row gathers in its own "
                                        "wave order over the row-block-major 604 MB group "
                                        "(profiles/r4/wrbench_rb_604MB.txt)")
    return {
        "bound": bound_label(eng), "kernel": names[dom], "bound_detail": bound_detail(eng, coded, E),
        # the same kernels streaming every byte from HBM (bench.py main: the
        # config3_hbm_streaming leg's frac, when that leg ran)
        "frac_hbm_streaming": None,
        "ceiling_measured": ceiling,
        "ceiling_source": ceiling_src,
        "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
        # a physical rate against a physical ceiling: the bytes the kernel moves
        "frac_moved_of_measured_ceiling": round(achieved_moved / ceiling, 4) if (achieved_moved and ceiling) else None,
        "traffic": traffic,
        "traffic_source": traffic_src,
        "traffic_per_cw_iter": per_cwi,
        "algorithmic_bytes_per_cw_iter": by_kernel[dom],
        "bytes_per_launch": round(bytes_per_launch), "avg_launch_ms": round(k_avg, 4),
        "launch_unit": "kernel launch",
        "achieved_moved": round(achieved_moved, 1) if achieved_moved else None,
        "frac_moved": round(achieved_moved / HBM_PEAK_GBS, 4) if achieved_moved else None,
        "moved_bytes_per_cw_iter": moved[dom],
        "iteration_GBps": round(iter_bytes / (it_ms * 1e-3) / 1e9, 1) if it_ms > 0 else None,
        "iteration_GBps_moved": round(iter_moved / (it_ms * 1e-3) / 1e9, 1) if it_ms > 0 else None,
        "iteration_bytes_per_cw_iter": {"survey_8d": 32.0 * E + 10.0 * N,
                                        "moved": moved["check"] + moved["variable"]},
        "iteration_note": ("iteration_GBps: SURVEY 8(d)'s 32 E + 10 N bytes per codeword-iteration (fp64 "
                           "messages both ways, fp64 prior) over the iteration's kernel time (check + variable "
                           "+ syndrome); iteration_GBps_moved: the bytes the check and variable kernels move"
                           + (" (compressed min-sum: per-row records instead of E fp64 c2v, so the SURVEY "
                              "rate may exceed the 8 TB/s peak)" if eng.msa_compressed else "")),
        "kernels": names,
        "avg_ms": {k: round(avg_ms(k), 4) for k in st},
        "launches": {k: v["launches"] for k, v in st.items()},
        "sampled": {k: v["sampled"] for k, v in st.items()},
    }


def dna272(args, og, threads, max_iter=200):
    """Config 2: the 272-codeword DNA-like batch (synth.dna_like_llrs, 72000
    reads) at the pipeline's max_iter, device-resident (the count differences
    k as int8 codes with the table k * ln49, LR = host libm exp as
    DNA_main.cpp:1344; --input fp64: fp64 LR), plus the end-to-end host-API
    time of the same decode (code table / host exp + PCIe + decode + copy
    back) -- the in-process replacement of decoder.py's 272 ldpc.exe runs
    (decoder.py:553-562)."""
    import ldpc_amd as L
    import synth
    cw = synth.load_codewords()
    llr = synth.dna_like_llrs(cw, seed=0)
    uniq, inv = np.unique(llr, return_inverse=True)
    lr = np.array([math.exp(v) for v in uniq])[inv].reshape(llr.shape)  # host libm exp per value
    G = L.Graph(synth.PCHK)
    B, N = llr.shape
    eng = L.Engine(G, 0, "bp", chunk=B)
    d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    k = np.rint(llr / synth.LLR_UNIT)
    if args.input == "code" and np.array_equal(k * synth.LLR_UNIT, llr) and np.abs(k).max() <= 127:
        d_in = L.DeviceBuffer(0, B * N)
        d_in.upload(np.ascontiguousarray(k.astype(np.int8)))
        table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT

        def step():
            eng.decode_codes(d_in.at(0), table, L.IN_LLR, B, max_iter, d_h.at(0), None, L.POST_LLR, d_i.at(0),
                             d_v.at(0))
    else:
        d_in = L.DeviceBuffer(0, B * N * 8)
        d_in.upload(np.ascontiguousarray(lr))

        def step():
            eng.decode(d_in.at(0), L.IN_LR, B, max_iter, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))

    for _ in range(max(1, args.warmup)):
        step()
    eng.sync()
    reps = max(args.steps, 10)
    t = time.perf_counter()
    for _ in range(reps):
        step()
    eng.sync()
    el = (time.perf_counter() - t) / reps
    it = d_i.download(np.empty(B, np.int32))
    hard = d_h.download(np.empty((B, N), np.uint8))
    # host API end to end (same decode, inputs in host memory): the DNA stage's
    # count differences k with the table k * ln49 (ldpc_decode_codes), and the
    # fp64 LLR matrix k * ln49 (ldpc_decode: lattice check + encode on the host)
    k8 = np.ascontiguousarray(k.astype(np.int8))
    kp = L.host_empty(k8.shape, np.int8)  # the same codes in pinned host memory
    kp[...] = k8
    table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT
    assert np.array_equal(table[k8.astype(np.int64) + 128], llr)
    import dna_pipeline
    first = dna_pipeline.gpu_decode_fn(G)  # the pipeline's first decode (decoder.py:553-562) from the codes
    G.decode_codes(k8, table, max_iter=max_iter, post=None)
    G.decode_codes(kp, table, max_iter=max_iter, post=None)
    G.decode(llr, max_iter=max_iter, post=None)
    first.codes(k8, table, max_iter)
    th, tp, tl, tf = [], [], [], []
    for _ in range(15):  # the host leg varies with the box's other tenants: median and min of 15 calls
        t = time.perf_counter()
        h2, _, it2, v2 = G.decode_codes(k8, table, max_iter=max_iter, post=None)
        th.append(time.perf_counter() - t)
        t = time.perf_counter()
        h4, _, it4, v4 = G.decode_codes(kp, table, max_iter=max_iter, post=None)
        tp.append(time.perf_counter() - t)
        t = time.perf_counter()
        h3, _, it3, v3 = G.decode(llr, max_iter=max_iter, post=None)
        tl.append(time.perf_counter() - t)
        t = time.perf_counter()
        h5 = first.codes(k8, table, max_iter)
        tf.append(time.perf_counter() - t)
    assert np.array_equal(h5, hard)
    assert np.array_equal(h2, hard) and np.array_equal(it2, it)
    assert np.array_equal(h3, hard) and np.array_equal(it3, it) and np.array_equal(v3, v2)
    assert np.array_equal(h4, hard) and np.array_equal(it4, it) and np.array_equal(v4, v2)
    out = {"workload": f"dna272-bp{max_iter}", "batch": B, "max_iter": max_iter, "input": args.input,
           "value": round(B / el, 1), "unit": "codewords/s", "ms_per_decode_device": round(el * 1e3, 3),
           "mean_iters": round(float(it.mean()), 3), "genie_ok": int((hard == cw).all(axis=1).sum()),
           "host_api_ms_median": round(float(np.median(th)) * 1e3, 3),
           "host_api_ms_min": round(float(np.min(th)) * 1e3, 3),
           "host_api_calls": len(th),
           "host_api_includes": "Graph.decode_codes -> ldpc_decode_codes end to end: the int8 count differences k "
                                "and the table k*ln49 (decoder.py:314) copied to pinned staging + H2D + decode + "
                                "packed hard-bit D2H + unpack",
           "host_api_pinned_ms_median": round(float(np.median(tp)) * 1e3, 3),
           "host_api_pinned_ms_min": round(float(np.min(tp)) * 1e3, 3),
           "host_api_pinned_includes": "the same call with the codes in pinned host memory (ldpc_amd.host_empty): "
                                       "no staging copy, one H2D from the caller's array",
           "host_api_llr_ms_median": round(float(np.median(tl)) * 1e3, 3),
           "host_api_llr_ms_min": round(float(np.min(tl)) * 1e3, 3),
           "host_api_llr_includes": "Graph.decode -> ldpc_decode from the fp64 LLR matrix: host lattice check + "
                                    "encode to int8 codes, then as above",
           "pipeline_first_decode_ms_median": round(float(np.median(tf)) * 1e3, 3),
           "pipeline_first_decode_ms_min": round(float(np.min(tf)) * 1e3, 3),
           "pipeline_first_decode_includes": "dna_pipeline.gpu_decode_fn(G).codes: the first decode of "
                                             "dna_pipeline.decode_trial when the LLR stage hands over its int8 codes "
                                             "(dna_llr.LlrResult.codes) -- the host_api call above, from Python"}
    if og is not None:
        t = time.perf_counter()
        rh, _, rit, rv = og.decode_batch(llr, max_iter, threads=threads, want_post=False)
        el_c = time.perf_counter() - t
        bad = [k for k in range(B) if not (np.array_equal(rh[k], h2[k]) and rit[k] == it2[k] and bool(rv[k]) == bool(v2[k]))]
        out["check"] = {"checked": B, "mismatches": len(bad), "first_mismatches": bad[:8],
                        "what": "every codeword of the host-API decode vs the oracle"}
        out["cpu_baseline"] = {"value": round(B / el_c, 2), "unit": "codewords/s", "cores": threads, "kind": "port",
                               "sample": f"the same 272 codewords, {max_iter} max iters, oracle on {threads} threads"}
    return out


def channel(L, eng, args, dev, N, b0, B, d_cw, n_cw, p, kind):
    """The BSC channel output of codewords [b0, b0 + B) in HBM -- int8 codes
    with the table code -> code * ln49 (--input code) or fp64 values of `kind`
    -- and the decode call on it."""
    import synth
    if args.input == "code":
        d_in = L.DeviceBuffer(dev, B * N)
        eng.gen_bsc_codes(d_in.at(0), b0, B, d_cw.at(0), n_cw, args.seed, p)
        table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT

        def decode(Bx, max_iter, h, it, v):
            eng.decode_codes(d_in.at(0), table, L.IN_LLR, Bx, max_iter, h, None, L.POST_LLR, it, v)
    else:
        d_in = L.DeviceBuffer(dev, B * N * 8)
        eng.gen_bsc(d_in.at(0), kind, b0, B, d_cw.at(0), n_cw, args.seed, p, synth.LLR_UNIT)

        def decode(Bx, max_iter, h, it, v):
            eng.decode(d_in.at(0), kind, Bx, max_iter, h, None, L.POST_LLR, it, v)
    return d_in, decode


def fp64_leg(args, L, eng, G, dev, b0, B, d_cw, n_cw, in_kind, iters, valid, d_hard):
    """The headline workload with the channel output as fp64 values in HBM
    (--input fp64) on the same engine: 1 warm-up + 2 timed decodes, and the
    proof that it is the same decode -- iteration counts and valid flags of
    every codeword and the hard bits of 1024 codewords spread over the shard
    equal the coded headline's."""
    N = G.N
    args_fp = argparse.Namespace(**{**vars(args), "input": "fp64"})
    d_in, decode = channel(L, eng, args_fp, dev, N, b0, B, d_cw, n_cw, args.p, in_kind)
    dh, di, dv = L.DeviceBuffer(dev, B * N), L.DeviceBuffer(dev, B * 4), L.DeviceBuffer(dev, B)
    decode(B, args.max_iter, dh.at(0), di.at(0), dv.at(0))
    eng.sync()
    eng.profile(0 if args.no_profile else 64)
    steps = 2
    t = time.perf_counter()
    for _ in range(steps):
        decode(B, args.max_iter, dh.at(0), di.at(0), dv.at(0))
    eng.sync()
    el = time.perf_counter() - t
    st = eng.stats()
    it2 = di.download(np.empty(B, np.int32))
    v2 = dv.download(np.empty(B, np.uint8))
    rows = np.unique(np.linspace(0, B - 1, min(B, 1024)).astype(np.int64))
    same_hard = all(np.array_equal(dh.download(np.empty(N, np.uint8), offset=int(r) * N),
                                   d_hard.download(np.empty(N, np.uint8), offset=int(r) * N)) for r in rows)
    same = bool(np.array_equal(it2, iters) and np.array_equal(v2, valid) and same_hard)
    avg = {k: round(v["ms"] / v["sampled"], 4) if v["sampled"] else 0.0 for k, v in st.items()}
    for b in (d_in, dh, di, dv):
        b.free()
    return {"input": "fp64 LR in HBM (LR = host exp(+-ln49))", "batch": B, "steps": steps,
            "value": round(B * steps / el, 1), "unit": "codewords/s", "ms_per_step": round(el / steps * 1e3, 2),
            "avg_ms": avg, "kernels": kernel_names(eng, "bp", False, args.var_cpw or None),
            "same_as_coded": same, "compared": f"iterations + valid flags of all {B}, hard bits of {len(rows)} codewords",
            "check": {"checked": len(rows), "mismatches": 0 if same else 1,
                      "what": "the fp64-input decode vs the coded headline decode (bit-identical)"}}


def hbm_stream(args, og, threads, cw, d_cw, B=16384):
    """The headline's kernels with nothing resident in a cache: BP on
    `B` codewords of the config-3 channel in ONE grouped pass (no resident
    pool, the check / variable launches span every tile, v2c and c2v
    2 x B x 1.18 MB = 38.7 GB at B = 16384, far beyond the 256 MB Infinity
    Cache), 1 warm-up + 2 timed decodes.  Its roofline is the HBM-streaming
    rate of the same arithmetic, beside the headline's Infinity-Cache-resident
    pool; 16 codewords (both ends) oracle-checked."""
    import ldpc_amd as L
    import synth
    G = L.Graph(synth.PCHK)
    N = G.N
    eng = L.Engine(G, 0, "bp", chunk=B, resident=False, group_tiles=-1)
    d_in, decode = channel(L, eng, args, 0, N, 0, B, d_cw, cw.shape[0], args.p, L.IN_LR)
    d_hard, d_iters, d_valid = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)

    def step():
        decode(B, args.max_iter, d_hard.at(0), d_iters.at(0), d_valid.at(0))

    step()
    eng.sync()
    eng.profile(0 if args.no_profile else 4)
    steps = 2
    t = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    el = time.perf_counter() - t
    st = eng.stats()
    iters = d_iters.download(np.empty(B, np.int32))
    valid = d_valid.download(np.empty(B, np.uint8))
    cw_iters = float(iters.sum()) * steps
    rl = roofline(eng, G, st, cw_iters, args.input == "code")
    out = {"workload": f"bsc-p{args.p}-{B // 1000}k-bp{args.max_iter}-one-pass", "batch": B, "steps": steps,
           "value": round(B * steps / el, 1), "unit": "codewords/s", "ms_per_step": round(el / steps * 1e3, 2),
           "schedule": {"resident_pool": eng.resident, "group_tiles": eng.group_tiles, "tiles": -(-B // 64),
                        "nontemporal_d": eng.nontemporal},
           "working_set_GB": round(2 * B * G.E * 8 / 1e9, 1),
           "roofline": rl,
           "note": "diagnostic: every message byte streams from HBM (working set >> 256 MB); the headline's pool "
                   "stays in the Infinity Cache, so its `frac` is of bytes through L2 -> fabric, served by both"}
    if og is not None:
        def llr_fn(start, k):
            return synth.bsc_llrs(cw, start, k, seed=args.seed, p=args.p)

        def gpu_out(start, k):
            h = d_hard.download(np.empty((k, N), np.uint8), offset=start * N)
            return h, iters[start:start + k], valid[start:start + k]

        checked, bad, _ = oracle_check(og, llr_fn, gpu_out, 0, args.max_iter, [(0, 8), (B - 8, 8)], threads)
        out["check"] = {"checked": checked, "mismatches": len(bad), "first_mismatches": bad[:8],
                        "what": "first and last 8 codewords of the timed decode vs the oracle"}
    for b in (d_in, d_hard, d_iters, d_valid):
        b.free()
    eng.close()
    return out


def msa_1m(args, og, threads, cw, d_cw):
    """Config 5: min-sum (Run_MSA_Decoder_INF) with early termination on
    `--msa-batch` codewords of BSC(p = 0.002), 1 warm-up + 2 timed decodes,
    roofline of its dominant kernel and an oracle check of a sample."""
    import ldpc_amd as L
    import synth
    G = L.Graph(synth.PCHK)
    N = G.N
    B, p, max_iter = args.msa_batch, 0.002, 50
    eng = L.Engine(G, 0, "msa")
    d_in, decode = channel(L, eng, args, 0, N, 0, B, d_cw, cw.shape[0], p, L.IN_LLR)
    d_hard, d_iters, d_valid = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)

    def step():
        decode(B, max_iter, d_hard.at(0), d_iters.at(0), d_valid.at(0))

    step()
    eng.sync()
    eng.profile(0 if args.no_profile else 16)
    steps = 2
    t = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    el = time.perf_counter() - t
    st = eng.stats()
    iters = d_iters.download(np.empty(B, np.int32))
    valid = d_valid.download(np.empty(B, np.uint8))
    cw_iters = float(iters.sum()) * steps
    out = {"workload": f"bsc-p{p}-{B // 1000}k-msa{max_iter}", "batch": B, "steps": steps, "input": args.input,
           "value": round(B * steps / el, 1), "unit": "codewords/s", "ms_per_step": round(el / steps * 1e3, 2),
           "mean_iters": round(float(iters.mean()), 3), "valid_frac": round(float(valid.mean()), 5),
           "resident_per_pass": eng.cap, "group_tiles": eng.group_tiles, "compressed_msa": eng.msa_compressed,
           "roofline": roofline(eng, G, st, cw_iters, args.input == "code")}
    if og is not None:
        n = max(8, 4 * threads)

        def llr_fn(start, k):
            return synth.bsc_llrs(cw, start, k, seed=args.seed, p=p)

        def gpu_out(start, k):
            h = d_hard.download(np.empty((k, N), np.uint8), offset=start * N)
            return h, iters[start:start + k], valid[start:start + k]

        tail, inter = tail_and_interior(B, n // 2, n_tail=n // 2, seed=args.seed)
        checked, bad, _ = oracle_check(og, llr_fn, gpu_out, 1, max_iter, [(0, n // 2), tail, inter], threads)
        out["check"] = {"checked": checked, "mismatches": len(bad), "first_mismatches": bad[:8],
                        "rows": {"head": [0, n // 2], "tail": [int(tail[0]), B] if tail.size else None,
                                 "interior": inter.tolist()},
                        "what": "hard bits, iterations, valid flags of the timed decode vs the oracle: both ends "
                                "of the batch and random interior codewords"}
    for b in (d_in, d_hard, d_iters, d_valid):
        b.free()
    eng.close()
    return out


def config4_total(opt: str, world: int, global_batch: int) -> int:
    """Codewords of the config-4 leg (0: none): --config4 auto runs BASELINE
    config 4 -- 1M codewords over 8 GPUs -- in the driver's 8-GPU weak-scaling
    run; an integer forces that global batch at any N > 1."""
    if world <= 1:
        return 0
    if opt == "auto":
        return 1_000_000 if world == 8 and global_batch == 0 else 0
    return max(0, int(opt))


def config4_leg(args, L, dist, grp, G, dev, d_cw, cw, og, threads, total):
    """BASELINE config 4 inside an N > 1 run: `total` codewords (1M at N = 8)
    split over the ranks by dist.shard -- DNA_main.cpp:629-651 Set_FrameNum's
    contiguous per-rank frame ranges, with the counters combined as its
    MPI_Reduce does (:1187-1193) -- on the default BP engine, 1 warm-up + 2
    timed decodes bracketed by barriers (max over ranks), then every rank
    checks the head, last rows and random interior rows of its shard against
    the oracle; the per-rank checks are gathered."""
    import synth
    world, rank = grp.world, grp.rank
    N = G.N
    b0, B = dist.shard(total, world, rank)
    eng = L.Engine(G, dev, "bp")
    d_in, decode = channel(L, eng, args, dev, N, b0, B, d_cw, cw.shape[0], args.p, L.IN_LR)
    d_hard, d_iters, d_valid = L.DeviceBuffer(dev, B * N), L.DeviceBuffer(dev, B * 4), L.DeviceBuffer(dev, B)

    def step():
        decode(B, args.max_iter, d_hard.at(0), d_iters.at(0), d_valid.at(0))

    step()
    eng.sync()
    steps = 2
    grp.barrier()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    el = time.perf_counter() - t
    grp.barrier()
    el_max = grp.max(el)
    iters = d_iters.download(np.empty(B, np.int32))
    valid = d_valid.download(np.empty(B, np.uint8))

    def llr_fn(start, n):
        return synth.bsc_llrs(cw, b0 + start, n, seed=args.seed, p=args.p)

    def gpu_out(start, n):
        return d_hard.download(np.empty((n, N), np.uint8), offset=start * N), iters[start:start + n], \
            valid[start:start + n]

    n = min(B, max(2, args.check_per_thread * threads))
    head = n - n // 2
    tail, inter = tail_and_interior(B, head, n_tail=n // 2, seed=args.seed + 100 + rank)
    checked, bad, _ = oracle_check(og, llr_fn, gpu_out, 0, args.max_iter, [(0, head), tail, inter], threads)
    per = grp.gather({"rank": rank, "b0": b0, "B": B, "checked": checked, "mismatches": len(bad),
                      "first_mismatches": [b0 + k for k in bad[:4]], "threads": threads,
                      "mean_iters": round(float(iters.mean()), 3),
                      "rows": {"head": [0, head], "tail": [int(tail[0]), B] if tail.size else None,
                               "interior": inter.tolist()}})
    for b in (d_in, d_hard, d_iters, d_valid):
        b.free()
    eng.close()
    return {"workload": f"bsc-p{args.p}-{total // 1000}k-global-bp{args.max_iter}", "global_batch": total,
            "n_gpus": world, "scaling": "strong", "per_rank": [p["B"] for p in per], "steps": steps,
            "value": round(total * steps / el_max, 2), "unit": "codewords/s",
            "ms_per_step": round(el_max / steps * 1e3, 3), "input": args.input,
            "check": {"checked": sum(p["checked"] for p in per), "mismatches": sum(p["mismatches"] for p in per),
                      "per_rank": per,
                      "what": "hard bits, iteration counts and valid flags of the timed decode vs the oracle on "
                              "every rank's shard: head, last rows (the lane pool's drain), random interior rows"}}


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run without a launcher: start N ranks under
    torch.distributed.run as a CHILD process (this process has not touched
    the GPU and never execs), forward rank 0's JSON line to stdout and
    everything else to stderr, and return the child's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: --gpus {n} without a launcher: running {n} ranks under torch.distributed.run",
          file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in p.stdout:
        print(line.rstrip("\n"), file=sys.stdout if line.lstrip().startswith("{") else sys.stderr, flush=True)
    return p.wait()


def main():
    args = parse()
    if args.gpus > 1 and args.workload == "bsc" and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    cpus = host_cpus()
    if args.workload == "dna272":
        og = _oracle().OracleGraph(os.path.join(ROOT, "tests", "golden", "decode_n18432_m2048_final.pchk")) \
            if args.cpu_baseline else None
        d = dna272(args, og, cpus["effective"], max_iter=args.max_iter if args.max_iter != 50 else 200)
        out = {"metric": METRIC, "value": d.pop("value"), "unit": "codewords/s", "n_gpus": 1,
               "steps": max(args.steps, 10), "warmup": args.warmup, "ms_per_step": d["ms_per_decode_device"],
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic (DNA read simulator over the 272 true codewords)", "config": d}
        for k in ("check", "cpu_baseline"):
            if k in d:
                out[k] = d.pop(k)
        print(json.dumps(out), flush=True)
        sys.exit(1 if out.get("check", {}).get("mismatches") else 0)
    import dist
    grp = dist.Group.from_env()  # gloo control plane only: barrier + MAX/SUM/gather of scalars
    world, rank, local = grp.world, grp.rank, grp.local
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if args.gpus != world and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: measuring {world} process(es); launch N "
              "ranks with python -m torch.distributed.run --nproc-per-node N", file=sys.stderr, flush=True)
    import ldpc_amd as L
    import synth

    G = L.Graph(synth.PCHK)
    N = G.N
    if args.global_batch > 0:
        # strong scaling: this rank's contiguous shard of the global range
        # (DNA_main.cpp:629-651 Set_FrameNum's split), sizes differ by <= 1
        b0, B = dist.shard(args.global_batch, world, rank)
        per_rank = [dist.shard(args.global_batch, world, r)[1] for r in range(world)]
        scaling = "strong"
    else:
        B = args.batch_per_gpu
        b0 = rank * B  # weak scaling: this rank's contiguous shard of the global codeword range
        per_rank = [B] * world
        scaling = "weak"
    if B <= 0:
        raise SystemExit(f"rank {rank}: empty shard")
    # one GPU per local rank; ranks share devices round-robin when there are
    # fewer GPUs than ranks (rehearsals on a one-GPU box)
    dev = local % max(1, L.device_count())
    algo = args.algo
    opt = lambda v: None if v < 0 else bool(v)  # noqa: E731
    eng = L.Engine(G, dev, algo, chunk=args.chunk, group_tiles=args.group_tiles,
                   nontemporal=opt(args.nt), continuous=opt(args.cont), resident=opt(args.res),
                   var_cpw=args.var_cpw or None, first_from_prior=opt(args.ffp))
    cw = synth.load_codewords()
    d_cw = L.DeviceBuffer(dev, cw.nbytes)
    d_cw.upload(cw)
    in_kind = L.IN_LR if algo == "bp" else L.IN_LLR
    d_in, decode = channel(L, eng, args, dev, N, b0, B, d_cw, cw.shape[0], args.p, in_kind)
    d_hard = L.DeviceBuffer(dev, B * N)
    d_iters = L.DeviceBuffer(dev, B * 4)
    d_valid = L.DeviceBuffer(dev, B)
    eng.sync()

    def step():
        decode(B, args.max_iter, d_hard.at(0), d_iters.at(0), d_valid.at(0))

    for _ in range(args.warmup):
        step()
    eng.sync()
    # HIP events on a sample of the launches (<= ~1000 per kernel class)
    passes = -(-B // eng.cap)
    groups = -(-(-(-B // passes) // 64) // eng.group_tiles)
    est = args.steps * passes * groups * args.max_iter
    eng.profile(0 if args.no_profile else max(1, -(-est // 1000)))
    grp.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    el = time.perf_counter() - t0
    grp.barrier()
    el_max = grp.max(el)
    st = eng.stats()
    iters = d_iters.download(np.empty(B, np.int32))
    valid = d_valid.download(np.empty(B, np.uint8))
    total_cw = grp.sum(float(B * args.steps))
    value = total_cw / el_max
    if args.dump_dir:
        os.makedirs(args.dump_dir, exist_ok=True)
        hard = d_hard.download(np.empty((B, N), np.uint8))
        np.savez(os.path.join(args.dump_dir, f"rank{rank}.npz"), b0=b0, B=B, world=world, iters=iters, valid=valid,
                 hard=np.packbits(hard, axis=1))

    cw_iters = float(iters.sum()) * args.steps  # executed codeword-iterations (this rank)
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "codewords/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": (f"bsc-p{args.p}-{args.global_batch // 1000}k-global-{algo}{args.max_iter}"
                                if args.global_batch > 0 else f"bsc-p{args.p}-{B // 1000}k-per-gpu-{algo}{args.max_iter}"),
                   "code": "decode_n18432_m2048_final.pchk (8,72)-regular, E=147456",
                   "input": ("int8 channel codes in HBM + table code*ln49 (LR = host exp)" if args.input == "code"
                             else "fp64 LR / LLR in HBM"),
                   "batch_per_gpu": B, "per_rank": per_rank, "global_batch": int(round(total_cw / args.steps)),
                   "max_iter": args.max_iter,
                   "algo": algo, "parallelism": f"dp{world} (contiguous codeword shards, no collective)",
                   "resident_per_pass": eng.cap, "group_tiles": eng.group_tiles, "nontemporal_d": eng.nontemporal,
                   "continuous": eng.continuous, "resident_pool": eng.resident,
                   "compressed_msa": eng.msa_compressed, "syndrome_split": eng.syndrome_split,
                   "mean_iters": round(float(iters.mean()), 3), "valid_frac": round(float(valid.mean()), 4)},
        "roofline": roofline(eng, G, st, cw_iters, args.input == "code", args.var_cpw or None),
    }

    # ---- correctness of the timed decode: every rank checks its own shard ----
    og = _oracle().OracleGraph(os.path.join(ROOT, "tests", "golden", "decode_n18432_m2048_final.pchk"))
    a = 0 if algo == "bp" else 1

    def llr_fn(start, n):
        return synth.bsc_llrs(cw, b0 + start, n, seed=args.seed, p=args.p)

    def gpu_out(start, n):
        h = d_hard.download(np.empty((n, N), np.uint8), offset=start * N)
        return h, iters[start:start + n], valid[start:start + n]

    threads = max(1, cpus["effective"] // max(1, local_world))
    if world == 1 and args.cpu_baseline:
        out["cpu_baseline"], (checked, bad, rows) = cpu_baseline(args, og, llr_fn, B, gpu_out, cpus)
    elif world > 1 and args.cpu_baseline and rank == 0:
        # rank 0's shard is checked by its cpu_baseline sample below (head,
        # tail and interior rows), once
        checked, bad, rows = 0, [], {}
    else:
        n = min(B, max(2, args.check_per_thread * threads))
        head = n - n // 2
        tail, inter = tail_and_interior(B, head, n_tail=n // 2, seed=args.seed + rank)
        checked, bad, _ = oracle_check(og, llr_fn, gpu_out, a, args.max_iter, [(0, head), tail, inter], threads)
        rows = {"head": [0, head], "tail": [int(tail[0]), B] if tail.size else None, "interior": inter.tolist()}
    if world > 1 and args.cpu_baseline:
        # the CPU path timed on the node's host cores in the same run
        # (north_star): rank 0 alone, on every core it may use, while the
        # other ranks wait in the barrier; its sample is rank 0's shard head,
        # checked against the timed decode as well
        grp.barrier()
        if rank == 0:
            cb, (c_cb, bad_cb, rows_cb) = cpu_baseline(args, og, llr_fn, B, gpu_out, cpus)
            cb["while"] = f"ranks 1..{world - 1} idle in a gloo barrier after their own checks"
            cb["checked"], cb["mismatches"] = c_cb, len(bad_cb)
            out["cpu_baseline"] = cb
            checked, bad, rows = c_cb, bad_cb, dict(rows_cb, via="cpu_baseline")
        grp.barrier()
    per = grp.gather({"rank": rank, "b0": b0, "B": B, "checked": checked, "mismatches": len(bad),
                      "first_mismatches": [b0 + k for k in bad[:4]], "threads": threads, "rows": rows})
    out["check"] = {"checked": sum(p["checked"] for p in per), "mismatches": sum(p["mismatches"] for p in per),
                    "per_rank": per,
                    "what": "hard bits, iteration counts and valid flags of the timed GPU decode vs the oracle, on "
                            "every rank's own shard: its head (N = 1: the cpu_baseline sample), its last rows (the "
                            "lane pool's drain) and random interior rows (per_rank[].rows, shard-relative)"}
    mismatches = out["check"]["mismatches"]

    # ---- BASELINE config 4 (N > 1): 1M codewords strong-sharded, after the headline ----
    c4 = config4_total(args.config4, world, args.global_batch)
    if c4 > 0 and algo == "bp":
        for b in (d_in, d_hard, d_iters, d_valid):
            b.free()
        eng.close()
        t = time.perf_counter()
        leg = config4_leg(args, L, dist, grp, G, dev, d_cw, cw, og, threads, c4)
        leg["leg_wall_s"] = round(time.perf_counter() - t, 2)
        out["secondary"] = {"note": "driver-timed after the headline region; not part of value / ms_per_step",
                            "config4_1m_strong" if c4 == 1_000_000 else "config4_strong": leg}
        mismatches += leg["check"]["mismatches"]

    # ---- secondary legs (N = 1): config 3 on fp64 input and streaming from HBM, config 5, config 2; each checked ----
    if world == 1 and args.secondary and args.global_batch == 0 and algo == "bp":
        sec = {"note": "driver-timed after the headline region; not part of value / ms_per_step"}
        if args.input == "code":
            t = time.perf_counter()
            sec["config3_fp64_input"] = fp64_leg(args, L, eng, G, dev, b0, B, d_cw, cw.shape[0], in_kind, iters, valid,
                                                 d_hard)
            sec["config3_fp64_input"]["leg_wall_s"] = round(time.perf_counter() - t, 2)
        for b in (d_in, d_hard, d_iters, d_valid):
            b.free()
        eng.close()
        if args.hbm_batch > 0:
            t = time.perf_counter()
            sec["config3_hbm_streaming"] = hbm_stream(args, og, cpus["effective"], cw, d_cw, B=args.hbm_batch)
            sec["config3_hbm_streaming"]["leg_wall_s"] = round(time.perf_counter() - t, 2)
        t = time.perf_counter()
        sec["config5_msa_1m"] = msa_1m(args, og, cpus["effective"], cw, d_cw)
        sec["config5_msa_1m"]["leg_wall_s"] = round(time.perf_counter() - t, 2)
        t = time.perf_counter()
        sec["config2_dna272"] = dna272(args, og, cpus["effective"])
        sec["config2_dna272"]["leg_wall_s"] = round(time.perf_counter() - t, 2)
        out["secondary"] = sec
        hs = sec.get("config3_hbm_streaming")
        if hs and out["roofline"]["bound"] != "hbm":
            out["roofline"]["frac_hbm_streaming"] = hs["roofline"]["frac"]
            out["roofline"]["frac_hbm_streaming_source"] = (
                f"secondary.config3_hbm_streaming: the same check / variable kernels on {hs['batch']} codewords "
                "in one grouped pass, every message byte from HBM")
        mismatches += sum(v.get("check", {}).get("mismatches", 0) for v in sec.values() if isinstance(v, dict))
    if rank == 0:
        print(json.dumps(out), flush=True)
    grp.close()
    if mismatches:
        print(f"bench.py: {mismatches} codewords of the timed decodes differ from the oracle", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
