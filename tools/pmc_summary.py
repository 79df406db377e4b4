#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 --pmc passes (one pass per counter
group, each a run of the same bench.py command), keyed by the kernel's full
template instantiation.

    python tools/pmc_summary.py <dir with pmc_*/run_counter_collection.csv> <bench .out> [out.json]

To feed bench.py's roofline.traffic, merge the "per_cw_iter_by_instantiation"
maps of the BP and min-sum summaries into profiles/r<N>/pmc_traffic.json
(tools/pmc_summary.py --merge out.json a.json b.json ...).

<bench .out> is the stdout of one of the passes (the bench JSON line): its
config gives the executed codeword-iterations (batch x mean_iters x steps).
Bytes: TCC_EA0_RDREQ x 128 + TCC_EA0_WRREQ x 64, the calibration of
profiles/r2/pmc_calib_and_decode.json (8-byte-per-lane message accesses);
FETCH_SIZE x 2 + WRITE_SIZE is reported beside it (MI355X_MICROARCH.md:
FETCH_SIZE reads half the bytes of a wide streaming read).
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("ldpc::dev::", "").strip()
    return n.replace(", ", ",")


def load(d):
    """kernel -> counter -> [sum over dispatches, dispatches]."""
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0]))
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            a = agg[k][r["Counter_Name"]]
            a[0] += float(r["Counter_Value"])
            a[1] += 1
    return agg


def merge(out, parts):
    m = {"what": "L2 -> fabric (EA) bytes per executed codeword-iteration of each decode kernel instantiation "
                 "(TCC_EA0_RDREQ x 128 + TCC_EA0_WRREQ x 64; calibration profiles/r2/pmc_calib_and_decode.json)",
         "sources": parts, "per_cw_iter_by_instantiation": {}}
    for p in parts:
        j = json.load(open(p))
        m["per_cw_iter_by_instantiation"].update(j["per_cw_iter_by_instantiation"])
    open(out, "w").write(json.dumps(m, indent=1) + "\n")
    print(json.dumps(m, indent=1))


def main():
    if sys.argv[1] == "--merge":
        return merge(sys.argv[2], sys.argv[3:])
    d, bench_out = sys.argv[1], sys.argv[2]
    line = [ln for ln in open(bench_out) if ln.startswith("{")][-1]
    bj = json.loads(line)
    c = bj["config"]
    cw_iters = float(c["batch_per_gpu"]) * float(c["mean_iters"]) * float(bj["steps"])
    agg = load(d)
    out = {"source": d, "bench": {k: c[k] for k in ("workload", "batch_per_gpu", "mean_iters", "algo")},
           "cw_iters": cw_iters,
           "bytes_formula": "TCC_EA0_RDREQ_sum x 128 + TCC_EA0_WRREQ_sum x 64 (profiles/r2/pmc_calib_and_decode.json)",
           "kernels": {}}
    for k, cs in sorted(agg.items()):
        if not k.startswith("k_"):
            continue
        e = {"dispatches": max(v[1] for v in cs.values())}
        for cn, (tot, n) in sorted(cs.items()):
            e[cn + "_per_cw_iter"] = round(tot / cw_iters, 2)
            e[cn + "_per_dispatch"] = round(tot / max(n, 1), 1)
        if "TCC_EA0_RDREQ_sum" in cs and "TCC_EA0_WRREQ_sum" in cs:
            e["ea_bytes_per_cw_iter"] = round((cs["TCC_EA0_RDREQ_sum"][0] * 128 + cs["TCC_EA0_WRREQ_sum"][0] * 64)
                                              / cw_iters)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["fetch2_write_bytes_per_cw_iter"] = round((cs["FETCH_SIZE"][0] * 2 + cs["WRITE_SIZE"][0]) * 1024
                                                        / cw_iters)
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            h, m = cs["TCC_HIT_sum"][0], cs["TCC_MISS_sum"][0]
            e["l2_hit_rate"] = round(h / max(h + m, 1), 4)
        if "SQ_WAVES" in cs and "SQ_INSTS_VALU" in cs:
            w = cs["SQ_WAVES"][0]
            for q in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if q in cs:
                    e[q + "_per_wave"] = round(cs[q][0] / max(w, 1), 1)
        out["kernels"][k] = e
    # bench.py's roofline.traffic lookup: EA bytes per executed codeword-iteration by instantiation
    out["per_cw_iter_by_instantiation"] = {k: e["ea_bytes_per_cw_iter"] for k, e in out["kernels"].items()
                                           if "ea_bytes_per_cw_iter" in e}
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
