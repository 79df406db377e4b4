"""CPU tests of the C ABI: the library loads, exports exactly what
include/ldpc_amd.h declares, and the host-side graph functions match the
oracle.  No compute calls that need a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PCHK, ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "ldpc_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc_[a-z_]+)\s*\(", src)))


def test_exports_match_header(L):
    declared = _declared()
    assert len(declared) >= 20
    out = subprocess.check_output(["nm", "-D", "--defined-only", L.LIB_PATH], text=True)
    exported = sorted(set(m for m in re.findall(r" T (ldpc_\w+)", out)))
    assert exported == declared
    assert sorted(L.EXPORTS) == declared
    lib = L.lib()
    for name in declared:
        assert hasattr(lib, name)
    assert lib.ldpc_abi_version() == 3 == L.ABI_VERSION


def test_stale_library_is_a_clear_import_error(L, monkeypatch):
    """A library that lacks a symbol the shim binds (a stale build) fails
    lib() with the ABI ImportError, not an AttributeError while binding."""
    L.lib()
    monkeypatch.setattr(L, "EXPORTS", L.EXPORTS + ["ldpc_not_in_this_build"])
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(ImportError, match="missing symbols .*ldpc_not_in_this_build"):
        L.lib()
    monkeypatch.undo()
    assert L.lib() is not None


def test_graph_load_matches_oracle(L, og):
    G = L.Graph(PCHK)
    assert (G.M, G.N, G.E) == (og.M, og.N, og.E)
    assert (G.dv, G.regular_dv, G.dc, G.regular_dc) == (8, True, 72, True)
    rp, ci, cp, ce = G.edges()
    assert np.array_equal(rp, og.row_ptr) and np.array_equal(ci, og.col_idx)
    assert np.array_equal(cp, og.col_ptr) and np.array_equal(ce, og.col_edge)


def test_host_syndrome_matches_oracle(L, og, codewords):
    G = L.Graph(PCHK)
    rng = np.random.default_rng(1)
    for x in [codewords[0], codewords[271], (rng.random(G.N) < 0.3).astype(np.uint8)]:
        c, p = G.syndrome(x)
        c2, p2 = og.check(x)
        assert c == c2 and np.array_equal(p, p2)


def test_bad_files(L, tmp_path):
    with pytest.raises(L.LdpcError) as e:
        L.Graph(str(tmp_path / "missing.pchk"))
    assert e.value.code == L.LDPC_ERR_IO
    bad = tmp_path / "bad.pchk"
    bad.write_bytes(b"\x00\x00\x00\x00" * 4)
    with pytest.raises(L.LdpcError) as e:
        L.Graph(str(bad))
    assert e.value.code == L.LDPC_ERR_FORMAT
    # truncated: no terminator (mod2sparse.cpp:421-426)
    ints = np.array([(ord("P") << 8) + 0x80, 2, 3, -1, 1, 2], dtype="<i4")
    trunc = tmp_path / "trunc.pchk"
    ints.tofile(str(trunc))
    with pytest.raises(L.LdpcError) as e:
        L.Graph(str(trunc))
    assert e.value.code == L.LDPC_ERR_FORMAT
    # column before any row selector
    ints = np.array([(ord("P") << 8) + 0x80, 2, 3, 1, 0], dtype="<i4")
    p = tmp_path / "norow.pchk"
    ints.tofile(str(p))
    with pytest.raises(L.LdpcError):
        L.Graph(str(p))
    # column out of range
    ints = np.array([(ord("P") << 8) + 0x80, 2, 3, -1, 4, 0], dtype="<i4")
    ints.tofile(str(p))
    with pytest.raises(L.LdpcError):
        L.Graph(str(p))


def test_ordering_and_dedup(L, oracle_mod, tmp_path):
    # rows/cols given out of order with a duplicate -> sorted, deduplicated
    ints = np.array([(ord("P") << 8) + 0x80, 3, 4, -2, 4, 1, 4, -1, 3, 2, -3, 1, 0], dtype="<i4")
    p = tmp_path / "o.pchk"
    ints.tofile(str(p))
    G = L.Graph(str(p))
    og = oracle_mod.OracleGraph(str(p))
    rp, ci, cp, ce = G.edges()
    assert G.E == 5
    assert rp.tolist() == [0, 2, 4, 5] and ci.tolist() == [1, 2, 0, 3, 0]
    assert np.array_equal(rp, og.row_ptr) and np.array_equal(ci, og.col_idx)
    assert np.array_equal(cp, og.col_ptr) and np.array_equal(ce, og.col_edge)
    G2 = L.Graph.from_edges(3, 4, [1, 1, 0, 0, 2, 1], [3, 0, 2, 1, 0, 3])
    assert np.array_equal(G2.edges()[1], ci)


def test_argument_validation_needs_no_gpu(L):
    G = L.Graph(PCHK)
    with pytest.raises(ValueError):
        G.decode(np.zeros((2, 5)))
    with pytest.raises(ValueError):
        G.decode(np.zeros((1, G.N)), algo="gallager")
    # B = 0 is a no-op that never touches a device
    h, p, it, v = G.decode(np.zeros((0, G.N)))
    assert h.shape == (0, G.N) and it.shape == (0,)


def test_algo_ints_are_reference_decoder_types(L):
    """An int algo is the reference's decoder_type (DNA_main.cpp:41-53, as
    LDPC_Decode :1565-1594 and bin/ldpc dispatch it); the ABI codes are
    reachable only by name."""
    assert L._algo(0) == L.ALGO_BP and L._algo("bp") == L.ALGO_BP
    assert L._algo(1) == L.ALGO_GALLAGER_A == L._algo("gallager_a")
    assert L._algo(2) == L.ALGO_GALLAGER_B1 and L._algo(3) == L.ALGO_GALLAGER_B2
    assert L._algo(20) == L._algo(21) == L._algo(22) == L.ALGO_MSA == L._algo("msa")
    assert L._algo(np.int32(20)) == L.ALGO_MSA
    for bad in (4, 5, 10, 50, True, "gallager", 1.0):
        with pytest.raises(ValueError):
            L._algo(bad)
    # the module's own ABI constants are Algo members: they select their decoder,
    # never the decoder_type with the same number (ALGO_MSA == 1 is not Gallager A)
    for a in L.Algo:
        assert L._algo(a) == int(a)
    assert L._algo(L.ALGO_MSA) == 1 and L._algo(L.ALGO_QMSA) == 2 and L._algo(L.ALGO_GALLAGER_B2) == 5
    # result file names carry the decoder_type the call ran as
    assert [L._decoder_type(a) for a in ("bp", "msa", "gallager_a", 1, 21, "qmsa")] == [0, 20, 1, 1, 21, 21]
    assert [L._decoder_type(a) for a in (L.ALGO_BP, L.ALGO_MSA, L.ALGO_GALLAGER_A)] == [0, 20, 1]


def test_schedule_struct_matches_header(L):
    """ldpc_schedule / ldpc_opts layouts of the ctypes shim against the
    header (ABI version 2), and Schedule.make's keyword mapping."""
    import ctypes as C
    hdr = open(os.path.join(ROOT, "include", "ldpc_amd.h")).read()
    for name, bit in L.SCHED_FLAGS.items():
        m = re.search(r"LDPC_SCHED_" + name.upper() + r"\s*=\s*1\s*<<\s*(\d+)", hdr)
        assert m and (1 << int(m.group(1))) == bit, name
    assert C.sizeof(L.Schedule) == 32 and C.sizeof(L.Opts) == 72
    s = L.Schedule.make(resident=False, continuous=True, group_tiles=2, syn_blocks=7)
    assert s.flags_set == L.SCHED_FLAGS["resident"] | L.SCHED_FLAGS["continuous"]
    assert s.flags == L.SCHED_FLAGS["continuous"] and s.group_tiles == 2 and s.syn_blocks == 7
    with pytest.raises(TypeError):
        L.Schedule.make(pingpong=True)
    assert L._schedule_kw(s) == {"resident": False, "continuous": True, "group_tiles": 2, "syn_blocks": 7}


def test_cli_rejects_bad_argc():
    exe = os.path.join(ROOT, "dna-ldpc-codes_amd", "bin", "ldpc")
    r = subprocess.run([exe, "0", "0", "0"], capture_output=True, text=True)
    assert r.returncode == 1 and "argc error!" in r.stderr


def test_cli_punct_short_argv(tmp_path):
    """Puncturing / shortening argv as SetUp consumes it (DNA_main.cpp:333-478):
    counts per type, the SC-code side file of types 2-4, and the exits for
    indices outside the code.  Every case stops before any GPU call."""
    import shutil
    exe = os.path.join(ROOT, "dna-ldpc-codes_amd", "bin", "ldpc")
    d = str(tmp_path)
    shutil.copyfile(PCHK, os.path.join(d, "code.pchk"))
    for f in ("cw", "soft"):
        with open(os.path.join(d, f + ".txt"), "w") as fh:
            fh.write("0 " * 18432)
    head = ["0", "0", "0", "7", "5", "1", "cw", "soft", "code", "0"]

    def run(*tail):
        return subprocess.run([exe, *head, *map(str, tail)], cwd=d, capture_output=True, text=True)

    for tail in [(1, 0, 0), (1, 0, 0, 5), (0, 1, 0, 1), (0, 2, 0, 3), (2, 0, 0, 1, 2, 3), (0, 0, 1, 5)]:
        r = run(*tail)  # one argument short of what SetUp reads
        assert r.returncode == 1 and "argc error!" in r.stderr, tail
    r = run(1, 0, 0, 1, 2, 99)  # one too many
    assert r.returncode == 1 and "argc error!" in r.stderr
    r = run(2, 0, 0, 1, 2, 3, 4)  # type 2 without <pchk>.txt
    assert r.returncode == 1 and "cannot open" in r.stderr and "code.txt" in r.stderr
    with open(os.path.join(d, "code.txt"), "w") as fh:
        fh.write("18431\n")  # D = L + w - 1 = 4 entries; the missing ones read as 0
    r = run(2, 0, 0, 1, 2, 3, 2)  # position 1 starts at bit 18431: 18432.. is outside
    assert r.returncode == 1 and "outside the code" in r.stderr
    for tail in [(1, 0, 0, 0, 3), (1, 0, 0, 18430, 18433), (0, 1, 0, 18432, 18433)]:
        r = run(*tail)
        assert r.returncode == 1 and "outside the code" in r.stderr, tail


def test_graph_blocks_array_structure(L):
    """ldpc_graph_blocks: the DNA code is RS-LDPC(8, 72, 8) with permuted
    columns; its column blocks are found by row-set matching and equal the RS
    blocks of the committed column permutation (tests/golden/code_fixtures.npz).
    Codes built in natural order get contiguous blocks (any Q); graphs without
    the structure (irregular) report none."""
    from conftest import GOLDEN
    G = L.Graph(PCHK)
    Q, rb, cb, cls = G.blocks()
    assert (Q, rb, cb) == (256, 8, 72)
    perm = np.load(os.path.join(GOLDEN, "code_fixtures.npz"))["rs_big_colperm"]
    assert np.array_equal(cls, perm // 256)
    rp, ci, _, _ = G.edges()
    rows = ci.reshape(G.M, G.dc)
    assert (np.sort(cls[rows], axis=1) == np.arange(72)).all()  # one column of every block per row
    R = L.Graph.rs_ldpc(7, 72, 8)
    Q, rb, cb, cls = R.blocks()
    assert (Q, rb, cb) == (128, 8, 72) and np.array_equal(cls, np.arange(R.N) // 128)
    Q, rb, cb, cls = L.Graph.rs_ldpc(5, 16, 4).blocks()
    assert (Q, rb, cb) == (32, 4, 16) and np.array_equal(cls, np.arange(16 * 32) // 32)
    irr = L.Graph.from_edges(4, 6, [0, 0, 1, 1, 2, 3], [0, 1, 2, 3, 4, 5])
    assert irr.blocks() is None


def test_decode_codes_rejects_codes_off_int8(L):
    """Graph.decode_codes checks the caller's codes before any device call:
    wider integer codes outside [-128, 127] and non-integer arrays raise
    instead of wrapping or truncating (in range, any integer dtype is taken)."""
    G = L.Graph(PCHK)
    table = np.arange(-128, 128, dtype=np.float64)
    with pytest.raises(ValueError, match="int8 range"):
        G.decode_codes(np.full((2, G.N), 200, np.int16), table, max_iter=1)
    with pytest.raises(ValueError, match="int8 range"):
        G.decode_codes(np.full((2, G.N), -129, np.int64), table, max_iter=1)
    with pytest.raises(TypeError, match="integers"):
        G.decode_codes(np.zeros((2, G.N), np.float64), table, max_iter=1)
    with pytest.raises(ValueError, match="256 entries"):
        G.decode_codes(np.zeros((2, G.N), np.int32), table[:10], max_iter=1)
