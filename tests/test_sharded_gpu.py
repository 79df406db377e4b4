"""Sharded decodes on the GPU (BASELINE config 4's path).

* bench.py under torch.distributed.run with 2 ranks (both on the box's one
  GPU) and --global-batch: each rank decodes its dist.shard of the global
  range (DNA_main.cpp:629-651 Set_FrameNum's split), and the outputs it
  dumps equal one single-process decode of the same global range, row for
  row;
* ldpc_decode's in-process multi-device path (opts.n_devices, one host
  thread + stream per device): every visible device, and ragged shards over
  repeated device ids, bit-exact against the oracle.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import synth
from test_gpu_parity import _cmp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def _load(d, world, N):
    parts = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
    parts.sort(key=lambda z: int(z["b0"]))
    return parts


SHARD_ARGS = ["--global-batch", "1000", "--max-iter", "20", "--p", "0.0065", "--steps", "1", "--warmup", "0",
              "--no-profile", "--cpu-baseline", "0"]
LAUNCH_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_PORT",
              "TORCHELASTIC_RUN_ID")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_ENV}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    return env


@pytest.fixture(scope="module")
def single_process_dump(tmp_path_factory):
    """One single-process bench.py decode of the whole global range [0, 1000)."""
    d1 = str(tmp_path_factory.mktemp("one"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dump-dir", d1, *SHARD_ARGS], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out1 = _line(r.stdout)
    assert out1["n_gpus"] == 1 and out1["config"]["per_rank"] == [1000]
    one = _load(d1, 1, None)[0]
    assert len(np.unique(one["iters"])) > 2 and one["valid"].any()
    return one


def _check_two_rank_run(stdout, d2, one):
    out2 = _line(stdout)
    assert out2["n_gpus"] == 2 and out2["scaling"] == "strong"
    assert out2["config"]["per_rank"] == [500, 500] and out2["config"]["global_batch"] == 1000
    # every rank checked its own shard against the oracle: head, tail, interior
    ck = out2["check"]
    assert ck["mismatches"] == 0 and [p["rank"] for p in ck["per_rank"]] == [0, 1]
    assert [p["b0"] for p in ck["per_rank"]] == [0, 500] and all(p["checked"] >= 16 for p in ck["per_rank"])
    for p in ck["per_rank"]:
        assert p["rows"]["tail"][1] == 500 and len(p["rows"]["interior"]) > 0
    two = _load(d2, 2, None)
    assert [int(z["b0"]) for z in two] == [0, 500] and [int(z["B"]) for z in two] == [500, 500]
    for z in two:
        b0, B = int(z["b0"]), int(z["B"])
        assert np.array_equal(z["iters"], one["iters"][b0:b0 + B])
        assert np.array_equal(z["valid"], one["valid"][b0:b0 + B])
        assert np.array_equal(z["hard"], one["hard"][b0:b0 + B])


@pytest.mark.timeout(240)
def test_two_rank_bench_shards_match_single_process(gpu, single_process_dump, tmp_path):
    """bench.py under an explicit torch.distributed.run (the driver's N > 1 form)."""
    d2 = str(tmp_path / "two")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dump-dir", d2, *SHARD_ARGS],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    _check_two_rank_run(r.stdout, d2, single_process_dump)


@pytest.mark.timeout(240)
def test_plain_bench_gpus2_runs_two_ranks(gpu, single_process_dump, tmp_path):
    """A plain `python bench.py --gpus 2` (no launcher in the environment)
    starts the two ranks itself (DNA_main.cpp:629-651's per-rank split, one
    process per GPU) and reports n_gpus 2 with both ranks' oracle checks."""
    d2 = str(tmp_path / "two")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dump-dir", d2,
                        *SHARD_ARGS], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "running 2 ranks under torch.distributed.run" in r.stderr
    _check_two_rank_run(r.stdout, d2, single_process_dump)


@pytest.mark.timeout(300)
def test_plain_bench_gpus2_cpu_baseline_and_config4_leg(gpu):
    """The N > 1 line carries what the driver's 8-GPU run needs by itself:
    rank 0's cpu_baseline (the oracle timed on the host cores while rank 1
    waits) and the config-4 leg -- here forced at a 1000-codeword global
    batch -- with both ranks' oracle checks of their dist.shard ranges."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch-per-gpu", "256",
                        "--max-iter", "20", "--p", "0.0065", "--steps", "1", "--warmup", "0", "--no-profile",
                        "--cpu-seconds", "1", "--config4", "1000"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["check"]["mismatches"] == 0
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1 and cb["checked"] > 0
    assert cb["mismatches"] == 0 and "barrier" in cb["while"]
    leg = out["secondary"]["config4_strong"]
    assert leg["global_batch"] == 1000 and leg["per_rank"] == [500, 500] and leg["scaling"] == "strong"
    assert leg["value"] > 0 and leg["check"]["mismatches"] == 0
    per = leg["check"]["per_rank"]
    assert [p["rank"] for p in per] == [0, 1] and [p["b0"] for p in per] == [0, 500]
    for p in per:
        assert p["checked"] >= 16 and p["rows"]["tail"][1] == 500 and len(p["rows"]["interior"]) > 0


def test_bench_global_batch_odd_split(gpu, tmp_path):
    """A global batch that does not divide: dist.shard sizes differ by one;
    single process -> the whole range."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--global-batch", "129", "--max-iter", "5",
                        "--steps", "1", "--warmup", "0", "--cpu-seconds", "0.5", "--dump-dir", str(tmp_path)],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = _line(r.stdout)
    assert out["config"]["per_rank"] == [129] and out["scaling"] == "strong"
    assert out["check"]["mismatches"] == 0 and out["check"]["checked"] >= 16
    z = np.load(os.path.join(tmp_path, "rank0.npz"))
    assert int(z["B"]) == 129 and z["iters"].shape == (129,)


def test_ldpc_decode_every_visible_device(gpu, G, og, codewords):
    """opts.n_devices = device_count(): the in-process multi-GPU path on
    every device of the box (one on a one-GPU box, eight on a node)."""
    n = gpu.device_count()
    llr = synth.bsc_llrs(codewords, 0, 64 * n + 37, seed=12, p=0.005)
    _cmp(G, og, llr, 25, devices=list(range(n)))


@pytest.mark.parametrize("devs,B", [([0, 0, 0], 200), ([0, 0, 0, 0, 0], 7), ([0, 0], 1)])
def test_ldpc_decode_ragged_shards(G, og, codewords, devs, B):
    """Ragged shards: B not divisible by the device count, shards smaller than
    a tile, more devices than codewords (empty shards)."""
    llr = synth.bsc_llrs(codewords, 3, B, seed=13, p=0.005)
    _cmp(G, og, llr, 25, devices=devs)
