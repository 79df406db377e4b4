"""Random-code parity soak (not part of the product or the test suite):
many random parity-check matrices, batch sizes, iteration limits, input
distributions and schedules, each decode checked bit for bit against the
oracle (tests/test_random_graphs_gpu.py's rules).  Prints one line per case
and every mismatch; a mismatch becomes a regression case in the tests.

    python tools/random_soak.py [--cases 150] [--seed 1] [--seconds 240]
"""
import argparse
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("dna-ldpc-codes_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

SCHEDULES = [{}, {"resident": False}, {"continuous": False}, {"resident": False, "nontemporal": True},
             {"msa_compressed": False}, {"resident": False, "group_tiles": 1, "var_cpw": 2}]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=150)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=240.0)
    a = ap.parse_args()
    import ldpc_amd as L
    import oracle
    from test_gpu_parity import _write_pchk
    from test_random_graphs_gpu import _random_graph, _regular_graph
    rng = np.random.default_rng(a.seed)
    tmp = tempfile.mkdtemp()
    t_end = time.time() + a.seconds
    bad = 0
    for c in range(a.cases):
        if time.time() > t_end:
            print(f"time limit after {c} cases", flush=True)
            break
        if rng.random() < 0.3:
            M, N, rows, cols = _regular_graph(rng, int(rng.choice([1, 2, 3, 4, 8, 16])))
            shape = "reg8x72"
        else:
            M = int(rng.integers(1, 160))
            N = int(rng.integers(2, 700))
            lo = int(rng.integers(0, 6))
            hi = lo + int(rng.integers(0, 90))
            rows, cols = _random_graph(rng, M, N, lo, hi, dup=bool(rng.random() < 0.5))
            shape = f"rand{lo}-{hi}"
        path = os.path.join(tmp, f"c{c}.pchk")
        _write_pchk(path, M, N, rows, cols)
        og = oracle.OracleGraph(path)
        G = L.Graph(path)
        B = int(rng.choice([1, 2, 63, 64, 65, 127, 200, 333]))
        max_iter = int(rng.choice([0, 1, 2, 5, 13, 40]))
        kind = rng.integers(0, 3)
        if kind == 0:
            x = rng.normal(float(rng.uniform(-1, 4)), float(rng.uniform(0.5, 5)), size=(B, N))
        else:
            p = float(rng.choice([0.001, 0.01, 0.05, 0.2]))
            x = np.where(rng.random((B, N)) < p, -3.8918202981106265, 3.8918202981106265)
            x[rng.random((B, N)) < 0.01] = 0.0
            if kind == 2:
                for v in (np.inf, -np.inf, np.nan, -0.0):
                    x[rng.random((B, N)) < 0.003] = v
        x = np.ascontiguousarray(x)
        r = rng.random()
        algo = "bp" if r < 0.4 else "msa" if r < 0.8 else str(rng.choice(["qmsa", "gallager_a", "gallager_b1",
                                                                          "gallager_b2"]))
        sch = SCHEDULES[int(rng.integers(0, len(SCHEDULES)))]
        ai = {"bp": 0, "msa": 1, "qmsa": 2, "gallager_a": 3, "gallager_b1": 4, "gallager_b2": 5}[algo]
        try:
            if ai >= 2:  # integer decoders: random quantizer / offset / tie seed (Set_MSA dec.cpp:1683)
                prec, step = int(rng.integers(2, 17)), float(rng.choice([0.25, 0.5, 1.0, 1.7]))
                beta, seed = int(rng.integers(0, 3)), int(rng.integers(0, 1 << 30))
                sch = {"prec": prec, "step": step, "beta": beta}
                rh, rp, rit, rv = og.decode_int_batch(x, max_iter, ai, precision=prec, step=step, beta=beta, seed=seed,
                                                      threads=8)
                h, ph, it, v = G.decode(x, max_iter=max_iter, algo=algo, post="llr", msa_precision=prec,
                                        msa_step=step, msa_offset=beta, tie_seed=seed)
            else:
                rh, rp, rit, rv = og.decode_batch(x, max_iter, algo=ai, post_mode=1 if ai == 0 else 0, threads=8)
                h, ph, it, v = G.decode(x, max_iter=max_iter, algo=algo, post="ratio" if ai == 0 else "llr",
                                        schedule=sch)
            nan = np.isnan(rp)
            ok = (np.array_equal(h, rh) and np.array_equal(it, rit) and np.array_equal(v, rv.astype(bool))
                  and np.array_equal(np.isnan(ph), nan) and np.array_equal(ph[~nan].view(np.uint64),
                                                                            rp[~nan].view(np.uint64)))
        except Exception as e:  # noqa: BLE001 -- a soak reports, it does not stop
            ok = False
            print(f"case {c}: exception {e}", flush=True)
        if not ok:
            bad += 1
        print(f"case {c:3d} {'ok ' if ok else 'BAD'} {shape:>12} M={M:4d} N={N:4d} E={G.E:6d} B={B:3d} "
              f"it={max_iter:2d} in={kind} {algo:11s} {sch}", flush=True)
    print(f"soak: {bad} mismatching case(s)", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
