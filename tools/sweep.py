#!/usr/bin/env python3
"""A/B the engine's schedule knobs in ONE process with interleaved rounds
(cdna_hip_programming.md rule 24): group tiles x nontemporal d-stream.
All variants must produce identical hard bits / iteration counts.

    python tools/sweep.py --batch 8192 --rounds 3 --configs 0:0,0:1,1:0,1:1,2:0,4:0
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))
import ldpc_amd as L  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--max-iter", type=int, default=50)
    ap.add_argument("--algo", default="bp")
    ap.add_argument("--p", type=float, default=0.02)
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--configs", default="0:0:0,1:1:1,2:1:0")  # group:nt:pipe:csc:cont
    args = ap.parse_args()
    G = L.Graph(synth.PCHK)
    N, E = G.N, G.E
    B = args.batch
    cfgs = [tuple(int(x) for x in (c + ":0:0:0:0").split(":")[:5]) for c in args.configs.split(",")]
    engines = [L.Engine(G, 0, args.algo, chunk=args.chunk or B, group_tiles=g, nontemporal=bool(nt),
                        pipeline=bool(pp), csc_scratch=bool(cs), continuous=bool(ct)) for g, nt, pp, cs, ct in cfgs]
    cw = synth.load_codewords()
    d_cw = L.DeviceBuffer(0, cw.nbytes)
    d_cw.upload(cw)
    kind = L.IN_LR if args.algo == "bp" else L.IN_LLR
    d_in = L.DeviceBuffer(0, B * N * 8)
    engines[0].gen_bsc(d_in.at(0), kind, 0, B, d_cw.at(0), 272, args.seed, args.p, synth.LLR_UNIT)
    engines[0].sync()
    outs = [(L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4)) for _ in cfgs]
    dv = L.DeviceBuffer(0, B)
    times = {c: [] for c in cfgs}
    kstats = {}
    for r in range(args.rounds + 1):
        for c, e, (dh, di) in zip(cfgs, engines, outs):
            e.profile(8 if r == args.rounds else 0)
            e.sync()
            t = time.perf_counter()
            e.decode(d_in.at(0), kind, B, args.max_iter, dh.at(0), None, L.POST_LLR, di.at(0), dv.at(0))
            e.sync()
            el = time.perf_counter() - t
            if r > 0:
                times[c].append(el)
            if r == args.rounds:
                kstats[c] = e.stats()
    ref_h = outs[0][0].download(np.empty((B, N), np.uint8))
    ref_i = outs[0][1].download(np.empty(B, np.int32))
    cwi = float(ref_i.sum())
    for c, (dh, di) in zip(cfgs, outs):
        same = np.array_equal(dh.download(np.empty((B, N), np.uint8)), ref_h) and \
            np.array_equal(di.download(np.empty(B, np.int32)), ref_i)
        best = min(times[c])
        st = kstats[c]
        ck = st["check"]["ms"] / max(1, st["check"]["sampled"])
        vk = st["variable"]["ms"] / max(1, st["variable"]["sampled"])
        per_launch_cw = B / max(1, st["check"]["launches"] / args.max_iter)
        res = {
            "group": c[0], "nt": c[1], "pipe": c[2], "csc": c[3], "cont": c[4], "identical": same, "best_s": round(best, 4),
            "median_s": round(float(np.median(times[c])), 4), "cw_per_s": round(B / best, 1),
            "iter_TBps": round((32 * E + 10 * N) * cwi / best / 1e12, 3), "mean_iters": round(cwi / B, 3),
            "check_ms": round(ck, 4), "var_ms": round(vk, 4),
            "check_TBps": round(16 * E * per_launch_cw / (ck * 1e-3) / 1e12, 3) if ck else None,
            "var_TBps": round((16 * E + 8 * N) * per_launch_cw / (vk * 1e-3) / 1e12, 3) if vk else None,
            "launches": st["check"]["launches"],
        }
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
