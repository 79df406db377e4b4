"""Tile-stream bimodality diagnostic (not part of the product): per-decode
throughput of several freshly created resident-pool engines with one stream
per pool tile (LDPC_RES_STREAMS=1) against the single-stream default, on the
config 3 input.  A per-engine split points at allocation placement, a
per-decode one at the chains' phase dynamics.
    python tools/tstream_diag.py [engines] [decodes] [batch]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))
import ldpc_amd as L  # noqa: E402
import synth  # noqa: E402

ne = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nd = int(sys.argv[2]) if len(sys.argv) > 2 else 6
B = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
G = L.Graph(synth.PCHK)
cw = synth.load_codewords()
N = G.N
d_cw = L.DeviceBuffer(0, cw.size)
d_cw.upload(np.ascontiguousarray(cw))
d_in = L.DeviceBuffer(0, B * N * 8)
d_h, d_i, d_v = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
for e in range(ne):
    for mode in ("1", "0"):
        os.environ["LDPC_RES_STREAMS"] = mode
        eng = L.Engine(G, 0, "bp", chunk=0)
        os.environ.pop("LDPC_RES_STREAMS")
        eng.gen_bsc(d_in.at(0), L.IN_LR, 0, B, d_cw.at(0), cw.shape[0], 2026, 0.02, float(np.log(49.0)))
        eng.decode(d_in.at(0), L.IN_LR, B, 50, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
        eng.sync()
        rates = []
        for _ in range(nd):
            t = time.perf_counter()
            eng.decode(d_in.at(0), L.IN_LR, B, 50, d_h.at(0), None, L.POST_LLR, d_i.at(0), d_v.at(0))
            eng.sync()
            rates.append(B / (time.perf_counter() - t))
        print(f"engine {e} streams={mode} tile_streams={int(eng.tile_streams)}: " +
              " ".join(f"{r / 1000:.2f}k" for r in rates), flush=True)
        eng.close()
