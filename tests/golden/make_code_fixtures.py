"""Regenerate tests/golden/code_fixtures.npz from the REFERENCE tools built
in place by `make -C oracle ref` (oracle/_ref/RS_LDPC from RS_LDPC.c,
oracle/_ref/alist-to-pchk from alist-to-pchk.cpp + the mod2sparse sources).

Stored per case: inputs and the reference's outputs (bytes, exit codes),
plus sha256 digests of the large (8, 72, 8) outputs and the column
permutation that maps tests/golden/decode_n18432_m2048_final.pchk onto the
(8, 72, 8) RS-LDPC code.  Only data -- no reference source -- is stored.

    python tests/golden/make_code_fixtures.py
"""
import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.path.join(ROOT, "oracle", "_ref")
OUT = os.path.join(ROOT, "tests", "golden", "code_fixtures.npz")

# (s, rho, gamma): small codes stored whole, incl. rho = q and gamma = q edges
RS_SMALL = [(2, 3, 1), (2, 4, 4), (3, 5, 3), (3, 8, 8), (4, 8, 3), (4, 16, 4), (5, 16, 4), (6, 32, 6)]
RS_BIG = (8, 72, 8)  # the DNA code (up to a column permutation)


def alist_cases():
    """(name, alist text, transpose) -- valid, irregular and malformed inputs."""
    rs = run([os.path.join(REF, "RS_LDPC"), "4", "8", "3", "x.alist", "2"], keep="x.alist")[2]
    cases = [("rs_4_8_3", rs, 0), ("rs_4_8_3_t", rs, 1)]
    # irregular: row 3 empty, column 4 empty, zero padding (1-based lists)
    M, N, rows = 4, 6, [[1, 2], [1, 3, 6], [], [2, 5]]
    irr, head, rsec, csec = mk_alist(M, N, rows)
    cases += [("irregular", irr, 0), ("irregular_t", irr, 1),
              ("no_newline", irr.rstrip(), 0), ("trailing_ws", irr + "  \n\n\t", 0)]
    r = rsec.split("\n")
    c = csec.split("\n")
    bad = {
        "dup_in_row": head + rsec.replace("1 3 6", "1 1 6") + csec,
        "col_mismatch": head + rsec + csec.replace("4 0 ", "3 0 "),
        "extra_number": irr + "7\n",
        "trailing_garbage": irr + "x\n",
        "nonzero_pad": head + "\n".join([r[0].replace("1 2 0", "1 2 5")] + r[1:]) + csec,
        "zero_in_list": head + rsec.replace("1 3 6", "1 0 6") + csec,
        "mxrw_too_big": irr.replace("3 2\n", "7 2\n", 1),
        "neg_M": "-" + irr,
        "truncated": irr[: len(irr) // 2],
        "col_out_of_range": head + rsec.replace("1 3 6", "1 3 7") + csec,
        "empty": "",
        # reference quirk: a column list naming a row twice and omitting
        # another still balances the entry count and is accepted
        # (alist-to-pchk.cpp:126-145)
        "col_dup_balanced": head + rsec + "\n".join([c[0].replace("1 2", "1 1")] + c[1:]),
    }
    cases += [(k, v, 0) for k, v in bad.items()]
    return cases


def mk_alist(M, N, rows):
    """alist text for 1-based row lists; returns (text, header, rows, cols)."""
    cols = [[i + 1 for i in range(M) if j + 1 in rows[i]] for j in range(N)]
    mxrw, mxcw = max(map(len, rows)), max(map(len, cols))
    head = f"{M} {N}\n{mxrw} {mxcw}\n" + " ".join(str(len(x)) for x in rows) + " \n" + \
        " ".join(str(len(x)) for x in cols) + " \n"
    pad = lambda xs, n: "".join(f"{v} " for v in xs + [0] * (n - len(xs))) + "\n"  # noqa: E731
    rsec = "".join(pad(x, mxrw) for x in rows)
    csec = "".join(pad(x, mxcw) for x in cols)
    return head + rsec + csec, head, rsec, csec


def run(cmd, keep=None, cwd=None, inputs=None):
    with tempfile.TemporaryDirectory() as td:
        for name, data in (inputs or {}).items():
            with open(os.path.join(td, name), "w") as f:
                f.write(data)
        p = subprocess.run(cmd, cwd=td, capture_output=True)
        data = b""
        if keep and os.path.exists(os.path.join(td, keep)):
            data = open(os.path.join(td, keep), "rb").read()
        return p.returncode, p.stdout, data.decode() if keep and keep.endswith(".alist") else data, p.stderr


def colperm(pchk_a, pchk_b):
    """perm[j] = column of pchk_a whose row set equals column j of pchk_b."""
    def cols(path):
        w = np.fromfile(path, dtype="<i4")
        N = int(w[2])
        lists = [[] for _ in range(N)]
        r = -1
        for v in w[3:]:
            if v == 0:
                break
            if v < 0:
                r = -v - 1
            else:
                lists[v - 1].append(r)
        return [tuple(sorted(x)) for x in lists]
    a, b = cols(pchk_a), cols(pchk_b)
    where = {c: j for j, c in enumerate(a)}
    return np.array([where[c] for c in b], np.int32)


def main():
    for tool in ("RS_LDPC", "alist-to-pchk"):
        if not os.path.exists(os.path.join(REF, tool)):
            sys.exit(f"oracle/_ref/{tool} missing: run `make -C oracle ref` (needs /root/reference)")
    out = {}
    for s, rho, gamma in RS_SMALL:
        for hp in (0, 2):
            rc, stdout, alist, _ = run([os.path.join(REF, "RS_LDPC"), str(s), str(rho), str(gamma), "o.alist", str(hp)],
                                       keep="o.alist")
            assert rc == 0
            out[f"rs_{s}_{rho}_{gamma}_stdout{hp}"] = np.frombuffer(stdout, np.uint8)
        out[f"rs_{s}_{rho}_{gamma}_alist"] = np.frombuffer(alist.encode(), np.uint8)
    s, rho, gamma = RS_BIG
    with tempfile.TemporaryDirectory() as td:
        a = os.path.join(td, "big.alist")
        p = os.path.join(td, "big.pchk")
        st = subprocess.run([os.path.join(REF, "RS_LDPC"), str(s), str(rho), str(gamma), a, "0"],
                            capture_output=True, check=True).stdout
        subprocess.run([os.path.join(REF, "alist-to-pchk"), a, p], check=True)
        out["rs_big_params"] = np.array(RS_BIG, np.int32)
        out["rs_big_alist_sha256"] = np.frombuffer(hashlib.sha256(open(a, "rb").read()).hexdigest().encode(), np.uint8)
        out["rs_big_pchk_sha256"] = np.frombuffer(hashlib.sha256(open(p, "rb").read()).hexdigest().encode(), np.uint8)
        out["rs_big_stdout0_sha256"] = np.frombuffer(hashlib.sha256(st).hexdigest().encode(), np.uint8)
        out["rs_big_colperm"] = colperm(p, os.path.join(ROOT, "tests", "golden", "decode_n18432_m2048_final.pchk"))
    names = []
    for name, text, t in alist_cases():
        cmd = [os.path.join(REF, "alist-to-pchk")] + (["-t"] if t else []) + ["in.alist", "out.pchk"]
        rc, _, pchk, err = run(cmd, keep="out.pchk", inputs={"in.alist": text})
        names.append(name)
        out[f"a2p_{name}_in"] = np.frombuffer(text.encode(), np.uint8)
        out[f"a2p_{name}_t"] = np.array(t, np.int32)
        out[f"a2p_{name}_rc"] = np.array(rc, np.int32)
        out[f"a2p_{name}_pchk"] = np.frombuffer(pchk if rc == 0 else b"", np.uint8)
        out[f"a2p_{name}_stderr"] = np.frombuffer(err, np.uint8)
    out["a2p_names"] = np.array(names)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(RS_SMALL)} RS codes, {len(names)} alist cases")


if __name__ == "__main__":
    main()
