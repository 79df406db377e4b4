"""bench.py end to end on a small batch: the one-JSON-line contract the
driver reads (metric / value / roofline / cpu_baseline), for the default BP
workload, min-sum, and the DNA batch."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METRIC = "decoded codewords/sec (n=18432, m=2048, 50 BP iters) at 1/2/4/8 GPUs; % HBM roofline"


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["metric"] == METRIC and out["unit"] == "codewords/s" and out["n_gpus"] == 1
    assert out["value"] > 0 and out["higher_is_better"] is True and out["scaling"] == "weak"
    return out


@pytest.mark.parametrize("algo,p", [("bp", 0.02), ("msa", 0.002)])
def test_bench_bsc_line(gpu, algo, p):
    out = _bench("--algo", algo, "--p", str(p), "--batch-per-gpu", "2048", "--steps", "1", "--warmup", "1",
                 "--cpu-seconds", "1", "--secondary", "0")
    assert out["steps"] == 1 and out["dtype"] == "f64"
    rl = out["roofline"]
    # BP's default schedule is the resident pool, sized to the Infinity Cache (MALL)
    assert rl["bound"] == ("hbm+mall (resident pool)" if algo == "bp" else "hbm")
    assert rl["unit"] == "GB/s" and rl["peak"] == 8000.0 and "frac_hbm_streaming" in rl
    assert rl["achieved"] > 0 and 0 < rl["frac"] < 1.2
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1 and cb["per_core"] > 0
    if algo == "bp":
        assert out["config"]["mean_iters"] == 50.0
    ck = out["check"]
    assert ck["mismatches"] == 0 and ck["checked"] >= 16 and len(ck["per_rank"]) == 1
    assert rl["kernel"] in rl["kernels"].values()


def test_bench_secondary_legs(gpu):
    """The driver-run line's secondary legs (config 5 min-sum, config 2 DNA
    batch through the host API), shrunk: each has its own oracle check."""
    out = _bench("--batch-per-gpu", "1024", "--steps", "1", "--warmup", "0", "--cpu-seconds", "0.5",
                 "--msa-batch", "8192", "--hbm-batch", "2048")
    sec = out["secondary"]
    m = sec["config5_msa_1m"]
    assert m["batch"] == 8192 and m["compressed_msa"] and m["check"]["mismatches"] == 0 and m["check"]["checked"] >= 8
    assert m["roofline"]["kernel"].startswith("k_var_msa_c") and m["roofline"]["achieved"] > 0
    d = sec["config2_dna272"]
    assert d["genie_ok"] == 272 and d["check"]["mismatches"] == 0 and d["check"]["checked"] == 272
    assert d["host_api_ms_median"] > 0
    # the headline on fp64 input decodes exactly what the coded headline does
    f = sec["config3_fp64_input"]
    assert f["same_as_coded"] and f["value"] > 0 and f["batch"] == 1024
    assert out["config"]["input"].startswith("int8") and "true>" in out["roofline"]["kernels"]["variable"]
    assert "false>" in f["kernels"]["variable"]
    # the headline's kernels streaming from HBM: one pass over every tile, nothing resident
    h = sec["config3_hbm_streaming"]
    assert h["batch"] == 2048 and not h["schedule"]["resident_pool"] and h["schedule"]["group_tiles"] == 32
    assert h["check"]["mismatches"] == 0 and h["check"]["checked"] == 16 and h["roofline"]["achieved"] > 0
    assert h["roofline"]["kernel"].startswith("k_check_bp<72,true,false>") or \
        h["roofline"]["kernel"].startswith("k_var_m<false,8,true,true")
    # the headline states both fractions: its resident pool's and the HBM-streaming leg's
    assert h["roofline"]["bound"] == "hbm" and out["roofline"]["bound"] == "hbm+mall (resident pool)"
    assert out["roofline"]["frac_hbm_streaming"] == h["roofline"]["frac"]
    # the pipeline's first decode from the LLR stage's int8 codes
    assert d["pipeline_first_decode_ms_median"] > 0


def test_bench_dna272_line(gpu):
    out = _bench("--workload", "dna272", "--steps", "2", "--warmup", "1")
    assert out["config"]["genie_ok"] == 272
