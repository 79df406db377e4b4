"""Placement diagnostic (not part of the product): several resident-pool BP
engines created one after another in one process (all kept alive, so each
lands on different memory), each timed on the same config 3 input with
sampled per-kernel HIP events.  Spread between engines = allocation
placement, which the engine's c2v probe is meant to remove.
    python tools/placement_diag.py [engines] [batch]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))
import ldpc_amd as L  # noqa: E402
import synth  # noqa: E402

ne = int(sys.argv[1]) if len(sys.argv) > 1 else 6
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
G = L.Graph(synth.PCHK)
cw = synth.load_codewords()
N = G.N
d_cw = L.DeviceBuffer(0, cw.size)
d_cw.upload(np.ascontiguousarray(cw))
d_in = L.DeviceBuffer(0, B * N * 8)
d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
keep = []
for e in range(ne):
    eng = L.Engine(G, 0, "bp", chunk=0)
    keep.append(eng)
    if e == 0:
        eng.gen_bsc(d_in.at(0), L.IN_LR, 0, B, d_cw.at(0), cw.shape[0], 2026, 0.02, synth.LLR_UNIT)
    eng.decode(d_in.at(0), L.IN_LR, B, 50, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
    eng.sync()
    eng.profile(10)
    t = time.perf_counter()
    eng.decode(d_in.at(0), L.IN_LR, B, 50, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
    eng.sync()
    el = time.perf_counter() - t
    st = eng.stats()
    avg = {k: 1e3 * st[k]["ms"] / max(1, st[k]["sampled"]) for k in ("check", "variable")}
    print(f"engine {e}: {B / el / 1000:.2f}k cw/s  check {avg['check']:.1f} us  variable {avg['variable']:.1f} us",
          flush=True)
