"""Throughput of the decoder on codes other than the DNA code (not part of
the product): RS-LDPC codes from the native constructor (RS_LDPC.c
parameters), random regular and irregular codes.  BP (and min-sum) on BSC
words of the all-zero codeword (--p; the default 0.05 makes most words run
all iterations), device-resident engine, 1 warm-up + 2 timed decodes.
Prints codewords/s, the kernel path (specialised 72/8 or generic; resident,
grouped continuous or fixed passes), the iteration's algorithmic bytes
(32 E + 10 N per codeword-iteration) over the kernel time
against 8 TB/s, and the sampled per-launch kernel times.

    python tools/code_bench.py [--batch 8192] [--iters 30] [--algo bp|msa] [--p 0.05]
                               [--chunk LANES | --pool] [--fixed] [--only SUBSTRING]

--chunk sets the lane pool / pass size (default: the whole batch), --pool
takes the engine's own default pool (resident where it applies), --fixed
runs fixed passes.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def codes(L, tmp):
    import synth
    from test_random_graphs_gpu import _regular_graph
    out = [("DNA RS(8,72,8) colperm", L.Graph(synth.PCHK))]
    for s, rho, gamma in ((8, 64, 4), (7, 64, 6), (8, 32, 4), (6, 32, 6), (9, 72, 8)):
        out.append((f"RS({s},{rho},{gamma})", L.Graph.rs_ldpc(s, rho, gamma)))
    rng = np.random.default_rng(5)
    M, N, rows, cols = _regular_graph(rng, 256, dv=3, dc=6)
    out.append(("random (3,6)-regular N=1536", L.Graph.from_edges(M, N, rows, cols)))
    M, N, rows, cols = _regular_graph(rng, 1024, dv=4, dc=32)
    out.append(("random (4,32)-regular N=32768", L.Graph.from_edges(M, N, rows, cols)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--algo", default="bp")
    ap.add_argument("--p", type=float, default=0.05)
    ap.add_argument("--chunk", type=int, default=0, help="lane pool / pass size (default: the batch)")
    ap.add_argument("--fixed", action="store_true", help="fixed passes instead of the continuous lane pool")
    ap.add_argument("--pool", action="store_true", help="the engine's default pool (resident where it applies)")
    ap.add_argument("--only", default="", help="substring of the code names to run")
    a = ap.parse_args()
    import ldpc_amd as L
    print(f"{'code':32s} {'N':>6} {'M':>5} {'E':>7} {'dv':>3} {'dc':>3} {'path':>14} {'cw/s':>10} "
          f"{'it/cw':>6} {'GB/s':>7} {'frac':>6} {'chk us':>7} {'var us':>7} {'syn us':>7}", flush=True)
    for name, G in codes(L, None):
        if a.only and a.only not in name:
            continue
        N, E = G.N, G.E
        # a few GB of state at most (with --chunk the state is the pool's; the batch as given)
        B = a.batch if a.chunk > 0 else max(64, min(a.batch, int(4e9 // (E * 16 + N * 10))))
        kw = {"continuous": False} if a.fixed else {}
        eng = L.Engine(G, 0, a.algo, chunk=0 if a.pool else min(B, a.chunk) if a.chunk > 0 else B, **kw)
        cw = np.zeros((1, N), np.uint8)
        d_cw = L.DeviceBuffer(0, N)
        d_cw.upload(cw)
        d_in = L.DeviceBuffer(0, B * N * 8)
        kind = L.IN_LR if a.algo == "bp" else L.IN_LLR
        eng.gen_bsc(d_in.at(0), kind, 0, B, d_cw.at(0), 1, 11, a.p, float(np.log((1 - 0.02) / 0.02)))
        d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)

        def run():
            eng.decode(d_in.at(0), kind, B, a.iters, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))

        run()
        eng.sync()
        eng.profile(8)
        t = time.perf_counter()
        for _ in range(2):
            run()
        eng.sync()
        el = (time.perf_counter() - t) / 2
        st = eng.stats()
        iters = d_i.download(np.empty(B, np.int32))
        ms = sum(st[k]["ms"] / st[k]["sampled"] * st[k]["launches"] for k in ("check", "variable", "syndrome")
                 if st[k]["sampled"]) / 2
        cwi = float(iters.sum())

        def per(k):  # average launch, us
            return st[k]["ms"] / st[k]["sampled"] * 1e3 if st[k]["sampled"] else 0.0
        gbs = (32.0 * E + 10.0 * N) * cwi / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        path = "72/8" if (G.dc == 72 and G.dv == 8 and G.regular_dc and G.regular_dv) else "generic"
        path += "/res" if eng.resident else "/grp" if eng.continuous else "/fix"
        print(f"{name:32s} {N:>6} {G.M:>5} {E:>7} {G.dv:>3} {G.dc:>3} {path:>14} {B / el:>10.1f} "
              f"{cwi / B:>6.1f} {gbs:>7.1f} {gbs / 8000:>6.3f} {per('check'):>7.1f} {per('variable'):>7.1f} "
              f"{per('syndrome'):>7.1f}", flush=True)
        for b in (d_cw, d_in, d_h, d_i, d_v):
            b.free()
        eng.close()


if __name__ == "__main__":
    main()
