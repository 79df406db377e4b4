"""Schedule sweep of bench.py's config3_hbm_streaming leg (not part of the
product): BP on 16 384 codewords of the config-3 channel in one grouped pass
(nothing resident), for each columns-per-wave of the variable kernel and
with / without the nontemporal v2c stream.  Prints the per-launch kernel
times (HIP events) and the dominant kernel's fraction of 8 TB/s, the way
bench.roofline computes it.

    python tools/hbm_sweep.py [--batch 16384] [--iters 50]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cpw", default="1,2,4,8")
    ap.add_argument("--nt", default="1,0")
    a = ap.parse_args()
    import bench
    import ldpc_amd as L
    import synth
    G = L.Graph(synth.PCHK)
    N, B = G.N, a.batch
    cw = synth.load_codewords()
    d_cw = L.DeviceBuffer(0, cw.nbytes)
    d_cw.upload(cw)
    args = argparse.Namespace(input="code", seed=2026, var_cpw=0)
    print(f"{'cpw':>4} {'nt':>3} {'cw/s':>9} {'check ms':>9} {'var ms':>8} {'frac':>7} {'kernel'}", flush=True)
    for cpw in (int(x) for x in a.cpw.split(",")):
        for nt in (bool(int(x)) for x in a.nt.split(",")):
            eng = L.Engine(G, 0, "bp", chunk=B, resident=False, group_tiles=-1, var_cpw=cpw, nontemporal=nt)
            d_in, decode = bench.channel(L, eng, args, 0, N, 0, B, d_cw, cw.shape[0], 0.02, L.IN_LR)
            d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
            decode(B, a.iters, d_h.at(0), d_i.at(0), d_v.at(0))
            eng.sync()
            eng.profile(4)
            t = time.perf_counter()
            for _ in range(2):
                decode(B, a.iters, d_h.at(0), d_i.at(0), d_v.at(0))
            eng.sync()
            el = (time.perf_counter() - t) / 2
            st = eng.stats()
            iters = d_i.download(np.empty(B, np.int32))
            rl = bench.roofline(eng, G, st, float(iters.sum()) * 2, True, cpw)
            print(f"{cpw:>4} {int(nt):>3} {B / el:>9.1f} {rl['avg_ms']['check']:>9.3f} {rl['avg_ms']['variable']:>8.3f} "
                  f"{rl['frac']:>7.4f} {rl['kernel']}", flush=True)
            for b in (d_in, d_h, d_i, d_v):
                b.free()
            eng.close()


if __name__ == "__main__":
    main()
