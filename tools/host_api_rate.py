"""PCIe-inclusive rate of the host-buffer boundary (ldpc_decode through the
ctypes shim) on config 3's BSC p = 0.02 input: host LLRs in, hard bits /
iterations / valid flags out.  DESIGN.md sec. 6 quotes it next to the
device-resident bench value.
    python tools/host_api_rate.py [B]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dna-ldpc-codes_amd"))
import ldpc_amd as L  # noqa: E402
import synth  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    cw = synth.load_codewords()
    G = L.Graph(synth.PCHK)
    llr = synth.bsc_llrs(cw, 0, B, seed=2026, p=0.02)
    G.decode(llr[:64], max_iter=50, post=None)  # device context, pinned pools
    for chunk, host_exp in ((0, True), (8192, True), (0, False)):
        ts = []
        for _ in range(2):
            t = time.perf_counter()
            _, _, it, _ = G.decode(llr, max_iter=50, post=None, chunk=chunk, exp_on_host=host_exp)
            ts.append(time.perf_counter() - t)
        assert (it == 50).all()
        print(json.dumps({"B": B, "pool": chunk or "engine default (resident 192 lanes), 4096-codeword PCIe chunks", "exp_on_host": host_exp,
                          "cw_per_s": round(B / min(ts), 1), "s": [round(x, 3) for x in ts]}), flush=True)


if __name__ == "__main__":
    main()
