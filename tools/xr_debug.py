"""XR decoder debug (not part of the product): iteration mismatches against
the oracle on the DNA batch across slot / variable-task / L1-invalidate
settings, and the time per decode."""
import os, sys, time, numpy as np
sys.path[:0] = ['dna-ldpc-codes_amd', 'oracle', 'tests']
import ldpc_amd as L, synth, oracle
og = oracle.OracleGraph(synth.PCHK)
cw = synth.load_codewords()
llr = synth.dna_like_llrs(cw, seed=0)
ref_h, ref_p, ref_it, ref_v = og.decode_batch(llr, 50, algo=0, post_mode=1, threads=8)
for spec in sys.argv[1:]:
    env = dict(kv.split("=") for kv in spec.split(","))
    os.environ.update(LDPC_XR="1", **env)
    G = L.Graph(synth.PCHK)
    G.decode(llr, max_iter=50, post="ratio")
    bads = []
    t = time.perf_counter()
    for r in range(5):
        h, p, it, v = G.decode(llr, max_iter=50, post="ratio")
        bads.append(int((it != ref_it).sum()))
    el = (time.perf_counter() - t) / 5
    print(spec, "bad per rep", bads, "hard_ok", np.array_equal(h, ref_h), f"{el*1e3:.2f} ms", flush=True)
    for k in env: os.environ.pop(k)
