"""bench.py's host-side helpers on CPU (no GPU): the oracle-check row
selection and the roofline block's algorithmic / moved byte accounting."""
import importlib.util
import os
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_tail_and_interior_rows():
    b = _bench()
    for B, lo in ((100_000, 200), (1_000_000, 32), (129, 16), (40, 30), (10, 10)):
        tail, inter = b.tail_and_interior(B, lo, seed=7)
        rows = np.concatenate([np.arange(lo), tail, inter])
        assert len(np.unique(rows)) == len(rows)  # disjoint
        assert rows.max() < B and (tail.size == 0 or tail[-1] == B - 1)
        assert np.all(np.diff(inter) > 0) and (inter.size == 0 or (inter.min() >= lo and inter.max() < B - 32))
        assert inter.size == min(32, max(0, B - 32 - lo))


def _eng(**kw):
    d = dict(msa_compressed=False, resident=True, continuous=True, nontemporal=False, algo=0)
    d.update(kw)
    return types.SimpleNamespace(**d)


def test_roofline_moved_bytes():
    b = _bench()
    G = types.SimpleNamespace(N=18432, M=2048, E=147456)
    st = {"check": {"ms": 0.07, "sampled": 1, "launches": 100}, "variable": {"ms": 0.068, "sampled": 1, "launches": 100},
          "syndrome": {"ms": 0.0, "sampled": 0, "launches": 0}}
    cw_iters = 100 * 192.0
    r = b.roofline(_eng(), G, st, cw_iters, coded=True)
    assert r["kernel"].startswith("k_check_bp")  # dominant
    assert r["achieved_moved"] == r["achieved"]  # the check kernel reads no prior
    assert r["iteration_bytes_per_cw_iter"]["survey_8d"] == 32 * G.E + 10 * G.N
    assert r["iteration_bytes_per_cw_iter"]["moved"] == 16 * G.E + 16 * G.E + 8 * G.N + G.N / 8 - 7 * G.N
    assert r["iteration_GBps_moved"] < r["iteration_GBps"]
    # compressed min-sum: the variable kernel dominates; moved = algorithmic - 7 N with coded priors
    st["variable"]["ms"] = 0.0713
    st["check"]["ms"] = 0.049
    rm = b.roofline(_eng(msa_compressed=True, resident=False, nontemporal=True, algo=1), G, st, cw_iters, coded=True)
    assert rm["kernel"].startswith("k_var_msa_c")
    assert rm["moved_bytes_per_cw_iter"] == rm["algorithmic_bytes_per_cw_iter"] - 7 * G.N
    assert abs(rm["achieved_moved"] / rm["achieved"] - rm["moved_bytes_per_cw_iter"] /
               rm["algorithmic_bytes_per_cw_iter"]) < 1e-3
    assert rm["frac_moved_of_measured_ceiling"] == round(rm["achieved_moved"] / rm["ceiling_measured"], 4)
    rf = b.roofline(_eng(msa_compressed=True, resident=False, nontemporal=True, algo=1), G, st, cw_iters, coded=False)
    assert rf["achieved_moved"] == rf["achieved"]


def test_kernel_names_match_the_committed_trace_and_traffic_table():
    """bench.kernel_names gives the template instantiations the engine
    launches in the default line (config 3: resident BP with coded priors;
    config 5: continuous compressed min-sum with coded priors): each must be a
    kernel of the committed rocprofv3 trace of that command and have an entry
    in the PMC traffic table bench.py reads for roofline.traffic, so a
    renamed template cannot silently drop the line's `traffic`."""
    import csv
    import glob
    import json
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_summary import short
    b = _bench()
    final = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "final", "default_bench_rocprofv3_kernel_stats.csv")))[-1]
    traced = {short(r["Name"]) for r in csv.DictReader(open(final))}
    table = json.load(open(sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))[-1]))
    known = set(table["per_cw_iter_by_instantiation"])
    bp = b.kernel_names(_eng(), "bp", coded=True)
    msa = b.kernel_names(_eng(msa_compressed=True, resident=False, nontemporal=True, algo=1), "msa", coded=True)
    for names in (bp, msa):
        for kind, name in names.items():
            assert name in traced, (kind, name)
            assert name in known, (kind, name)


def test_config4_leg_selection():
    """BASELINE config 4 (1M codewords over 8 GPUs) runs inside the driver's
    8-GPU weak-scaling bench by default; --config4 G forces it at N > 1."""
    b = _bench()
    assert b.config4_total("auto", 8, 0) == 1_000_000
    assert b.config4_total("auto", 8, 1_000_000) == 0  # the headline already is config 4
    assert [b.config4_total("auto", n, 0) for n in (1, 2, 4)] == [0, 0, 0]
    assert b.config4_total("4096", 2, 0) == 4096 and b.config4_total("4096", 1, 0) == 0
    assert b.config4_total("0", 8, 0) == 0


def test_roofline_bound_names_residency():
    """The headline's resident pool lives in the 256 MB Infinity Cache: its
    roofline says so in `bound`, and carries the HBM-streaming fraction of the
    same kernels beside `frac` (filled by main() from the
    config3_hbm_streaming leg)."""
    b = _bench()
    G = types.SimpleNamespace(N=18432, M=2048, E=147456)
    st = {"check": {"ms": 0.07, "sampled": 1, "launches": 100}, "variable": {"ms": 0.068, "sampled": 1, "launches": 100},
          "syndrome": {"ms": 0.0, "sampled": 0, "launches": 0}}
    r = b.roofline(_eng(), G, st, 100 * 192.0, coded=True)
    assert r["bound"] == "hbm+mall (resident pool)"
    assert "frac_hbm_streaming" in r and r["frac"] > 0
    g = b.roofline(_eng(resident=False, cap=16384, group_tiles=-1), G, st, 100 * 192.0)
    assert g["bound"] == "hbm" and "frac_hbm_streaming" in g
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'out["roofline"]["frac_hbm_streaming"] = hs["roofline"]["frac"]' in src


def test_bound_detail_grouped_schedules():
    """_bound_detail tells a one-pass grouped run (every tile in one group)
    from a multi-pass one, with the working set from the graph's E
    (ADVICE r5)."""
    b = _bench()
    E = 147456
    one = b._bound_detail(_eng(resident=False, cap=16384, group_tiles=-1), E)
    assert one.startswith("one grouped pass over every tile (256)") and "streams from HBM" in one
    assert b._bound_detail(_eng(resident=False, cap=16384, group_tiles=256), E).startswith("one grouped pass")
    multi = b._bound_detail(_eng(resident=False, cap=16384, group_tiles=4), E)
    assert multi.startswith("grouped schedule, 4 of 256 tiles per group") and "exceeds" in multi  # 288 MB
    small = b._bound_detail(_eng(resident=False, cap=16384, group_tiles=2), E)
    assert "meant to stay in the Infinity Cache" in small  # 144 MB
    tiny = b._bound_detail(_eng(resident=False, cap=16384, group_tiles=2), 1000)
    assert "(1 MB)" in tiny
