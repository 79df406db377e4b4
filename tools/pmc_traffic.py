#!/usr/bin/env python3
"""Per-codeword-iteration memory-side bytes of each decode kernel class from
the rocprofv3 PMC passes of tools/gpu_profile.sh, written as the
pmc_traffic.json bench.py reads for the roofline `traffic` field.

    python tools/pmc_traffic.py gpurun_out/<tag> <cw_iters> profiles/<round>/pmc_traffic.json [exclude ...]

exclude: kernel names to leave out (e.g. the engine's placement-probe
launches, which run outside the decode: the plain in-place instantiations
k_check_bp<72;false;false;false> / k_var_m<false;8;false;false;4> of the
resident pool).

cw_iters = executed codeword-iterations of the profiled run (the PMC passes
run bench.py --batch-per-gpu 1024 on BSC p=0.02, which never converges: 1024
x 50).  Bytes = FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md sec.
HBM) + WRITE_SIZE, summed over the kernel's dispatches.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402

CLASSES = {  # logical class -> kernel-name prefixes (template instantiations)
    "k_check_bp": ("ldpc::dev::k_check_bp<",),
    "k_var_bp": ("ldpc::dev::k_var_m<false", "ldpc::dev::k_var_bp<"),
    "k_check_msa": ("ldpc::dev::k_check_msa<",),
    "k_var_msa": ("ldpc::dev::k_var_m<true", "ldpc::dev::k_var_msa<"),
    "k_check_msa_c": ("ldpc::dev::k_check_msa_c<",),
    "k_var_msa_c": ("ldpc::dev::k_var_msa_c<",),
}


def main():
    d, cw_iters, out = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    exclude = set(sys.argv[4:])
    agg = pmc_summary.load(d)
    per, kernels = {}, {}
    for cls, prefixes in CLASSES.items():
        tot, names = 0.0, []
        for k, cs in agg.items():
            if not k.startswith(prefixes) or k in exclude:
                continue
            names.append(k)
            for c, mult in (("FETCH_SIZE", 2048.0), ("WRITE_SIZE", 1024.0)):
                if c in cs:
                    tot += cs[c][1] * mult  # summed over dispatches (KB -> bytes, fetch x2)
        if names:
            per[cls] = round(tot / cw_iters)
            kernels[cls] = names
    json.dump({"source": f"{d} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)",
               "correction": "FETCH_SIZE x2 (gfx950) + WRITE_SIZE, summed over dispatches / executed cw-iterations",
               "cw_iters": cw_iters, "per_cw_iter": per, "kernels": kernels}, open(out, "w"), indent=1)
    print(json.dumps(per))


if __name__ == "__main__":
    main()
