#!/usr/bin/env python3
"""Round-2 PMC analysis (tools/gpu_pmc_r2.sh output): per-dispatch counters of
the known-bytes calibration (tools/cachebench calib) and of the bench's decode
kernels, turned into bytes.

    python tools/pmc_r2.py gpurun_out/<tag> profiles/r2

Calibration: rows_rmw<72> reads and rewrites exactly `bytes` per dispatch
(2048 MB from HBM, 64 MB Infinity-Cache resident after its first pass).  From
it: bytes per TCC_EA0_RDREQ / WRREQ (fabric requests), whether FETCH_SIZE /
WRITE_SIZE need a correction for this access width, and what a DRAM request
counts.  Then the decode kernels' fabric bytes and DRAM bytes per executed
codeword-iteration (the bench run: 8192 codewords x 50 iterations through the
3-tile resident pool; the resident pool's placement-probe dispatches -- the
in-place kernels without the fused syndrome -- are excluded).
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    """kernel -> counter -> list of per-dispatch values (dispatch order)."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace(", ", ";")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    d, out = sys.argv[1], sys.argv[2]
    cal = load(os.path.join(d, "calib"))
    rows = [k for k in cal if k.startswith("rows_rmw")]
    assert rows, "no calibration dispatches"
    c = cal[rows[0]]
    # dispatches: 3 x 2048 MB, then 3 x 64 MB; bytes read = bytes written
    mbs = [2048] * 3 + [64] * 3
    nbytes = [(m * (1 << 20)) // 512 // 72 * 72 * 512 for m in mbs]
    calib = []
    for i, b in enumerate(nbytes):
        e = {"bytes_read": b, "bytes_written": b}
        for cn, v in c.items():
            if i < len(v):
                e[cn] = v[i]
        calib.append(e)
    # use the last dispatch of each size (steady state)
    hbm, mall = calib[2], calib[5]
    per = {
        "rdreq_bytes": hbm["bytes_read"] / hbm["TCC_EA0_RDREQ_sum"],
        "wrreq_bytes": hbm["bytes_written"] / hbm["TCC_EA0_WRREQ_sum"],
        "fetch_kb_per_byte": hbm["FETCH_SIZE"] * 1024 / hbm["bytes_read"],
        "write_kb_per_byte": hbm["WRITE_SIZE"] * 1024 / hbm["bytes_written"],
        "dram_rd_bytes_per_req": hbm["bytes_read"] / hbm["TCC_EA0_RDREQ_DRAM_sum"],
        "dram_wr_bytes_per_req": hbm["bytes_written"] / hbm["TCC_EA0_WRREQ_DRAM_sum"],
        "mall_resident_dram_rd_share": mall["TCC_EA0_RDREQ_DRAM_sum"] / mall["TCC_EA0_RDREQ_sum"],
        "mall_resident_dram_wr_share": mall["TCC_EA0_WRREQ_DRAM_sum"] / mall["TCC_EA0_WRREQ_sum"],
    }
    rq = per["rdreq_bytes"]
    wq = per["wrreq_bytes"]
    drq = per["dram_rd_bytes_per_req"]
    dwq = per["dram_wr_bytes_per_req"]
    ben = load(os.path.join(d, "bench"))
    cw_iters = 8192 * 50.0
    kern = {}
    for k, cs in sorted(ben.items()):
        if not k.startswith("ldpc::dev::k_") or "RDREQ" not in str(list(cs)):
            continue
        # probe launches: the in-place kernels without the fused syndrome
        if k.startswith("ldpc::dev::k_check_bp<72;false;false;false;true>") or \
                k.startswith("ldpc::dev::k_var_m<false;8;false;true;4;true>") and False:
            continue
        rd = sum(cs.get("TCC_EA0_RDREQ_sum", [])) * rq
        wr = sum(cs.get("TCC_EA0_WRREQ_sum", [])) * wq
        drd = sum(cs.get("TCC_EA0_RDREQ_DRAM_sum", [])) * drq
        dwr = sum(cs.get("TCC_EA0_WRREQ_DRAM_sum", [])) * dwq
        n = len(cs.get("TCC_EA0_RDREQ_sum", []))
        kern[k] = {"dispatches": n, "fabric_read_bytes": rd, "fabric_write_bytes": wr, "dram_read_bytes": drd,
                   "dram_write_bytes": dwr,
                   "fetch_size_x1_bytes": sum(cs.get("FETCH_SIZE", [])) * 1024,
                   "write_size_bytes": sum(cs.get("WRITE_SIZE", [])) * 1024}
    res = {"source": d, "calibration": calib, "per_request": per, "cw_iters": cw_iters, "kernels": kern}
    os.makedirs(out, exist_ok=True)
    json.dump(res, open(os.path.join(out, "pmc_calib_and_decode.json"), "w"), indent=1)
    print(json.dumps(per, indent=1))
    for k, v in kern.items():
        print(k[:70], v["dispatches"], {kk: round(vv / cw_iters) for kk, vv in v.items() if kk != "dispatches"})


if __name__ == "__main__":
    main()
