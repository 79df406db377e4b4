"""BASELINE config 4 (1M codewords sharded evenly across 8 GPUs), one shard at
a time on the box's one GPU: exactly what rank r of

    torch.distributed.run --nproc-per-node 8 bench.py --gpus 8 --global-batch 1000000

decodes -- its dist.shard of the global range (DNA_main.cpp:629-651
Set_FrameNum's split), 125 000 codewords of BSC(p = 0.02) from the device
generator with seed 2026, BP, 50 iterations, the engine's default schedule.
Nothing converges at p = 0.02, so every codeword must run all 50 iterations
and end invalid; a sample of 64 codewords at their global indices (both ends
of the shard and random interior ones) equals the oracle bit for bit.  Rank 7
runs as bench.py does by default (the channel output as int8 codes,
ldpc_engine_decode_codes), rank 3 on fp64 LR input.
"""
import numpy as np
import pytest

import dist
import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.mark.timeout(240)
@pytest.mark.parametrize("rank,coded", [(7, True), (3, False)])
def test_config4_shard(gpu, G, og, codewords, rank, coded):
    L = gpu
    b0, B = dist.shard(1_000_000, 8, rank)
    assert B == 125_000 and b0 == 125_000 * rank
    N, max_iter, seed, p = G.N, 50, 2026, 0.02
    eng = L.Engine(G, 0, "bp")
    cwbuf = L.DeviceBuffer(0, codewords.nbytes)
    cwbuf.upload(codewords)
    table = np.arange(-128, 128, dtype=np.float64) * synth.LLR_UNIT
    din = L.DeviceBuffer(0, B * N * (1 if coded else 8))
    dh, dit, dv = L.DeviceBuffer(0, B * N), L.DeviceBuffer(0, B * 4), L.DeviceBuffer(0, B)
    if coded:
        eng.gen_bsc_codes(din.at(0), b0, B, cwbuf.at(0), 272, seed, p)
        eng.decode_codes(din.at(0), table, L.IN_LLR, B, max_iter, dh.at(0), None, L.POST_LLR, dit.at(0), dv.at(0))
    else:
        eng.gen_bsc(din.at(0), L.IN_LR, b0, B, cwbuf.at(0), 272, seed, p, synth.LLR_UNIT)
        eng.decode(din.at(0), L.IN_LR, B, max_iter, dh.at(0), None, L.POST_LLR, dit.at(0), dv.at(0))
    eng.sync()
    it = dit.download(np.empty(B, np.int32))
    v = dv.download(np.empty(B, np.uint8))
    assert (it == max_iter).all() and not v.any()
    # device input = the host replica at the global indices (spot rows)
    for k in (0, B // 2, B - 1):
        if coded:
            row = table[din.download(np.empty((1, N), np.int8), offset=k * N).astype(np.int64) + 128]
        else:
            row = din.download(np.empty((1, N), np.float64), offset=k * N * 8)
        assert np.array_equal(row, synth.bsc_llrs(codewords, b0 + k, 1, seed=seed, p=p, as_lr=not coded))
    rng = np.random.default_rng(rank)
    idx = np.unique(np.concatenate([[0, 1, B - 2, B - 1], rng.choice(B, 60, replace=False)]))
    llr = np.concatenate([synth.bsc_llrs(codewords, b0 + int(k), 1, seed=seed, p=p) for k in idx])
    rh, _, rit, rv = og.decode_batch(llr, max_iter, algo=0, threads=8, want_post=False)
    assert (rit == max_iter).all() and not rv.any()
    for q, k in enumerate(idx):
        h = np.empty((1, N), np.uint8)
        dh.download(h, offset=int(k) * N)
        assert np.array_equal(h[0], rh[q]), b0 + int(k)
    for b in (din, dh, dit, dv, cwbuf):
        b.free()
