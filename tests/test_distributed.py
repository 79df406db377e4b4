"""Multi-process (gloo, world_size 2) tests of the sharded path on CPU.

The decode has no collective; what must hold is that (a) the shards tile the
global codeword range exactly, (b) every rank's synthetic input depends only on
the global codeword index (so results do not depend on the GPU count), and
(c) the timing/counter reductions are MAX/SUM over ranks.  The per-rank work
here is the CPU oracle on the rank's shard (the GPU decode is covered by the
`-m gpu` tests); the gathered results must equal a single-process run.
"""
import os
import tempfile

import numpy as np
import pytest

import dist
import synth


def test_shard_tiles_range():
    for total in (0, 1, 7, 100, 100_000, 1_000_000):
        for world in (1, 2, 3, 4, 8):
            spans = [dist.shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_inputs_independent_of_world_size():
    cw = synth.load_codewords()
    whole = synth.bsc_llrs(cw, 1000, 64, seed=2026, p=0.02)
    parts = []
    for r in range(4):
        s, c = dist.shard(64, 4, r)
        parts.append(synth.bsc_llrs(cw, 1000 + s, c, seed=2026, p=0.02))
    assert np.array_equal(np.concatenate(parts), whole)


def _rank_work(g, outdir, total):
    import oracle
    og = oracle.OracleGraph(synth.PCHK)
    cw = synth.load_codewords()
    s, c = dist.shard(total, g.world, g.rank)
    llr = synth.bsc_llrs(cw, s, c, seed=2026, p=0.006)
    h, _, it, v = og.decode_batch(llr, 20, threads=2, want_post=False)
    np.savez(os.path.join(outdir, f"rank{g.rank}.npz"), start=s, hard=np.packbits(h, axis=1), iters=it, valid=v)
    g.barrier()
    t_max = g.max(float(g.rank + 1))
    n_sum = g.sum(float(c))
    if g.rank == 0:
        np.savez(os.path.join(outdir, "reduce.npz"), t_max=t_max, n_sum=n_sum)


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_single_process(og, codewords):
    total = 10
    with tempfile.TemporaryDirectory() as d:
        dist.launch_local(_rank_work, 2, args=(d, total))
        red = np.load(os.path.join(d, "reduce.npz"))
        assert float(red["t_max"]) == 2.0 and float(red["n_sum"]) == total
        parts = [np.load(os.path.join(d, f"rank{r}.npz")) for r in range(2)]
        parts.sort(key=lambda z: int(z["start"]))
        hard = np.concatenate([np.unpackbits(z["hard"], axis=1, count=og.N) for z in parts])
        iters = np.concatenate([z["iters"] for z in parts])
    llr = synth.bsc_llrs(codewords, 0, total, seed=2026, p=0.006)
    h, _, it, v = og.decode_batch(llr, 20, threads=4, want_post=False)
    assert np.array_equal(hard, h) and np.array_equal(iters, it)


@pytest.mark.timeout(180)
def test_plain_bench_gpus_n_starts_n_ranks():
    """`python bench.py --gpus 2` without a launcher starts two ranks under
    torch.distributed.run as a child process and forwards its exit code.  On
    this GPU-less host both ranks join the gloo group and then fail at engine
    creation (no device), which must surface as a non-zero exit, not as a
    one-process measurement."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--global-batch", "128",
                        "--steps", "1", "--warmup", "0", "--cpu-baseline", "0"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=170)
    assert "running 2 ranks under torch.distributed.run" in r.stderr
    assert r.returncode != 0 and not r.stdout.strip(), (r.returncode, r.stdout)
    assert r.stderr.count("ldpc_amd error") >= 2, r.stderr[-3000:]
