"""In-process A/B timing of engine variants on the same device-resident
workload (the bench's BSC config 3 input), alternating variants so clock,
thermal and allocation effects hit both alike.

    python tools/ab_engines.py --var A:var_cpw=1 --var B:var_cpw=8 --reps 6

Each variant is NAME:KEY=VAL[,KEY=VAL...], KEY a ldpc_schedule keyword
(ldpc_amd.Schedule.make: resident, group_tiles, var_cpw, ...) or `chunk`.
Prints one JSON line per variant with the median/min seconds per decode and
cw/s.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", action="append", required=True)
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--max-iter", type=int, default=50)
    ap.add_argument("--algo", default="bp")
    ap.add_argument("--p", type=float, default=0.02)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--chunk", type=int, default=16384)
    ap.add_argument("--profile", type=int, default=0, help="HIP-event sample stride per kernel class (0: off)")
    ap.add_argument("--input", default="fp64", choices=["fp64", "code"],
                    help="channel output as fp64 LLRs or int8 codes + table (ldpc_engine_decode_codes)")
    ap.add_argument("--fresh", type=int, default=0,
                    help="rounds of create/time/free per variant (averages allocation placement); 0 = one "
                         "engine per variant, timed --reps times")
    args = ap.parse_args()
    import ldpc_amd as L
    import synth
    G = L.Graph(synth.PCHK)
    cw = synth.load_codewords()
    B, N = args.batch, G.N
    d_cw = L.DeviceBuffer(0, cw.size)
    d_cw.upload(np.ascontiguousarray(cw))
    coded = args.input == "code"
    d_in = L.DeviceBuffer(0, B * N * (1 if coded else 8))
    table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT

    def gen(e):
        if coded:
            e.gen_bsc_codes(d_in.at(0), 0, B, d_cw.at(0), cw.shape[0], 2026, args.p)
        else:
            e.gen_bsc(d_in.at(0), L.IN_LLR, 0, B, d_cw.at(0), cw.shape[0], 2026, args.p, synth.LLR_UNIT)

    def run(e):
        if coded:
            e.decode_codes(d_in.at(0), table, L.IN_LLR, B, args.max_iter, d_h.at(0), None, L.POST_LLR, d_i.at(0),
                           d_v.at(0))
        else:
            e.decode(d_in.at(0), L.IN_LLR, B, args.max_iter, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
    d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    def make(spec):
        name, _, kvs = spec.partition(":")
        kw = {}
        for kv in filter(None, kvs.split(",")):
            k, v = kv.split("=", 1)
            kw[k] = int(v)
        chunk = kw.pop("chunk", args.chunk)
        return name, L.Engine(G, 0, args.algo, chunk=chunk, schedule=kw)

    if args.fresh:
        gen = None
        res = {}
        ref = None
        for rnd in range(args.fresh):
            # rotate the creation order: the allocator hands out the same
            # memory to the same creation slot, so every variant visits every slot
            k0 = rnd % len(args.var)
            for spec in args.var[k0:] + args.var[:k0]:
                name, e = make(spec)
                if gen is None:
                    gen(e)
                    gen = True
                ts = []
                for k in range(2):  # warm-up + timed
                    t = time.perf_counter()
                    run(e)
                    e.sync()
                    ts.append(time.perf_counter() - t)
                it = d_i.download(np.empty(B, np.int32))
                if ref is None:
                    ref = it.copy()
                elif not np.array_equal(ref, it):
                    raise SystemExit(f"variant {name} changed the iteration counts")
                res.setdefault(name, []).append(B / ts[1])
                del e
            print(json.dumps({"round": rnd, **{n: round(v[-1], 1) for n, v in res.items()}}), flush=True)
        for name, v in res.items():
            print(json.dumps({"variant": name, "cw_per_s_mean": round(float(np.mean(v)), 1),
                              "cw_per_s_std": round(float(np.std(v)), 1), "cw_per_s_min": round(min(v), 1),
                              "cw_per_s_max": round(max(v), 1), "rounds": len(v)}), flush=True)
        return

    engines = []
    for spec in args.var:
        name, e = make(spec)
        if args.profile:
            e.profile(args.profile)
        engines.append((name, e))
    gen(engines[0][1])
    engines[0][1].sync()
    times = {n: [] for n, _ in engines}
    ref = None
    for rep in range(args.reps + 1):
        for name, e in engines:
            t = time.perf_counter()
            run(e)
            e.sync()
            el = time.perf_counter() - t
            if rep > 0:
                times[name].append(el)
            it = d_i.download(np.empty(B, np.int32))
            if ref is None:
                ref = it.copy()
            elif not np.array_equal(ref, it):
                raise SystemExit(f"variant {name} changed the iteration counts")
        print(json.dumps({"rep": rep, **{n: round(B / v[-1], 1) for n, v in times.items() if v}}), flush=True)
    for name, e in engines:
        if args.profile:
            st = e.stats()
            print(json.dumps({"variant": name, "kernels": {k: {"launches": v["launches"], "avg_ms": round(
                v["ms"] / max(v["sampled"], 1), 4)} for k, v in st.items() if v["launches"]}}), flush=True)
    for name, v in times.items():
        print(json.dumps({"variant": name, "median_s": round(float(np.median(v)), 5), "min_s": round(min(v), 5),
                          "cw_per_s_median": round(B / float(np.median(v)), 1), "cw_per_s_best": round(B / min(v), 1),
                          "reps": len(v)}), flush=True)


if __name__ == "__main__":
    main()
