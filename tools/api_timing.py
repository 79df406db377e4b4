"""Host-API time of one ldpc_decode call on the DNA batch (debug, not part of
the product), for settings given as NAME=ENV=VAL[,...] arguments
(LDPC_API_TIMING=1 prints the host-leg split per chunk)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dna-ldpc-codes_amd"))
import ldpc_amd as L, synth
cw = synth.load_codewords()
llr = synth.dna_like_llrs(cw, seed=0)
ref = None
for spec in sys.argv[1:] or ["default:"]:
    name, _, envs = spec.partition(":")
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    G = L.Graph(synth.PCHK)
    ts = []
    for r in range(12):
        t = time.perf_counter()
        h, _, it, v = G.decode(llr, max_iter=200, post=None)
        ts.append(time.perf_counter() - t)
    if ref is None:
        ref = (h, it)
    assert np.array_equal(h, ref[0]) and np.array_equal(it, ref[1])
    print(f"{name}: median {np.median(ts[2:]) * 1e3:.3f} ms, min {min(ts[2:]) * 1e3:.3f} ms", flush=True)
    for kv in filter(None, envs.split(",")):
        os.environ.pop(kv.split("=", 1)[0])
