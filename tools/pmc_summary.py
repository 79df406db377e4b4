#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (counter_collection.csv) per kernel.

FETCH_SIZE / WRITE_SIZE are in KB; FETCH_SIZE is doubled for gfx950
(MI355X_MICROARCH.md sec. HBM: it reports half of a wide coalesced read).
TCC_EA0_{RD,WR}REQ_DRAM_sum count 64-B requests that reach DRAM (the rest of
the L2 misses are served by the Infinity Cache).
    python tools/pmc_summary.py gpurun_out/<tag> [out.csv]
"""
import collections
import csv
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not sub.startswith("pmc") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace(", ", ";")
            a = agg[k][r["Counter_Name"]]
            a[0] += 1
            a[1] += float(r["Counter_Value"])
    return agg


def main():
    d = sys.argv[1]
    agg = load(d)
    rows = []
    for k, cs in sorted(agg.items()):
        g = {c: v[1] / v[0] for c, v in cs.items()}
        n = max(v[0] for v in cs.values())
        fetch = g.get("FETCH_SIZE", 0) * 1024 * 2
        write = g.get("WRITE_SIZE", 0) * 1024
        drd = g.get("TCC_EA0_RDREQ_DRAM_sum", 0) * 64
        dwr = g.get("TCC_EA0_WRREQ_DRAM_sum", 0) * 64
        rows.append((k, n, fetch, write, drd, dwr))
    hdr = "kernel,dispatches,fetch_bytes_x2,write_bytes,dram_read_bytes,dram_write_bytes"
    out = [hdr] + [f"{k},{n},{f:.0f},{w:.0f},{r:.0f},{x:.0f}" for k, n, f, w, r, x in rows]
    print("\n".join(out))
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
