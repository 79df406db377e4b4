"""Tile-group size for single-fill decodes (not part of the product): device
time of one decode of B DNA-like codewords through an engine whose pool
holds all of them, per LDPC_GROUP_TILES value, medians of 10.
    python tools/group_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))
import ldpc_amd as L  # noqa: E402
import synth  # noqa: E402

G = L.Graph(synth.PCHK)
cw = synth.load_codewords()
base = synth.dna_like_llrs(cw, seed=0)
for B in (192, 272, 448, 768, 1024):
    llr = np.concatenate([base] * (B // len(base) + 1))[:B]
    lr = np.exp(llr)
    N = G.N
    d_in = L.DeviceBuffer(0, B * N * 8)
    d_in.upload(np.ascontiguousarray(lr))
    d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    res = []
    for g in (1, 2, 3, 4):
        os.environ["LDPC_GROUP_TILES"] = str(g)
        eng = L.Engine(G, 0, "bp", chunk=B)
        os.environ.pop("LDPC_GROUP_TILES")
        ts = []
        for r in range(12):
            t = time.perf_counter()
            eng.decode(d_in.at(0), L.IN_LR, B, 200, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
            eng.sync()
            ts.append(time.perf_counter() - t)
        res.append(f"g{g} {np.median(ts[2:]) * 1e3:.3f}")
        eng.close()
    print(f"B {B} ({(B + 63) // 64} tiles): " + "  ".join(res), flush=True)
    d_in.free()
