import sys, numpy as np
sys.path.insert(0, 'dna-ldpc-codes_amd')
import ldpc_amd as L, synth
G = L.Graph(synth.PCHK); cw = synth.load_codewords()
for B in (65536, 262144):
    eng = L.Engine(G, 0, "msa")
    d_cw = L.DeviceBuffer(0, cw.nbytes); d_cw.upload(cw)
    din = L.DeviceBuffer(0, B * G.N * 8)
    eng.gen_bsc(din.at(0), L.IN_LLR, 0, B, d_cw.at(0), 272, 2026, 0.002, synth.LLR_UNIT)
    dh, di, dv = L.DeviceBuffer(0, B * G.N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    eng.profile(1000000)
    eng.decode(din.at(0), L.IN_LLR, B, 50, dh.at(0), None, L.POST_LLR, di.at(0), dv.at(0)); eng.sync()
    st = eng.stats()
    it = di.download(np.empty(B, np.int32))
    print(B, "cap", eng.cap, "syndrome launches", st["syndrome"]["launches"], "check", st["check"]["launches"],
          "cw-iters", int(it.sum()), "ideal steps", it.sum() / eng.cap, "mean", it.mean())
