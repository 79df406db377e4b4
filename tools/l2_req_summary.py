#!/usr/bin/env python3
"""L2 request counters per codeword-iteration of each decode kernel class,
from the rocprofv3 --pmc passes of tools/gpu_l2_req.sh (1024 codewords x 50
iterations, non-converging inputs).

    python tools/l2_req_summary.py gpurun_out/<tag> [out.csv]

TCC_HIT/TCC_MISS count L2 requests by outcome; TCP_TCC_READ/WRITE_REQ count
the requests the vector L1s send to L2.  The placement-probe launches of the
resident pool (plain in-place instantiations) run outside the decode and are
left out.
"""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import CLASSES  # noqa: E402

PROBE = {"ldpc::dev::k_check_bp<72;false;false;false>", "ldpc::dev::k_var_m<false;8;false;false;4>"}
CW_ITERS = 1024 * 50


def main():
    d = sys.argv[1]
    tot = collections.defaultdict(float)  # (class, counter) -> summed value
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace(", ", ";")
            if k in PROBE:
                continue
            for cls, prefixes in CLASSES.items():
                if k.startswith(prefixes):
                    tot[(cls, r["Counter_Name"])] += float(r["Counter_Value"])
    counters = sorted({c for _, c in tot})
    classes = sorted({k for k, _ in tot})
    out = ["class," + ",".join(f"{c}_per_cw_iter" for c in counters)]
    for cls in classes:
        out.append(cls + "," + ",".join(f"{tot.get((cls, c), 0.0) / CW_ITERS:.0f}" for c in counters))
    print("\n".join(out))
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
