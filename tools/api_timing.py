"""Host-API time of one ldpc_decode call on the DNA batch (debug, not part of
the product), for variants given as NAME:KEY=VAL[,...] arguments (KEY an
ldpc_amd.Schedule keyword, or host_threads / chunk).  With
LDPC_API_TIMING=1 in the environment the library prints the host-leg split
of every call to stderr.

    LDPC_API_TIMING=1 python tools/api_timing.py default: t8:host_threads=8
"""
import hashlib
import os
import sys
import time

import numpy as np

if os.environ.get("API_TIMING_TORCH"):  # the bench.py process has torch and its HIP context up
    import torch
    torch.zeros(1, device="cuda")

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-ldpc-codes_amd"))
import ldpc_amd as L  # noqa: E402
import synth  # noqa: E402

cw = synth.load_codewords()
llr = synth.dna_like_llrs(cw, seed=0)
ref = None
G = L.Graph(synth.PCHK)
for spec in sys.argv[1:] or ["default:"]:
    name, _, kvs = spec.partition(":")
    kw = {}
    for kv in filter(None, kvs.split(",")):
        k, v = kv.split("=", 1)
        kw[k] = int(v)
    call = {k: kw.pop(k) for k in ("host_threads", "chunk") if k in kw}
    ts = []
    for r in range(14):
        t = time.perf_counter()
        h, _, it, v = G.decode(llr, max_iter=200, post=None, schedule=kw or None, **call)
        ts.append(time.perf_counter() - t)
    if ref is None:
        ref = (h, it)
    assert np.array_equal(h, ref[0]) and np.array_equal(it, ref[1])
    dig = hashlib.sha256(h.tobytes() + it.tobytes() + v.tobytes()).hexdigest()[:16]
    print(f"{name}: median {np.median(ts[2:]) * 1e3:.3f} ms, min {min(ts[2:]) * 1e3:.3f} ms, outputs sha {dig}",
          flush=True)
