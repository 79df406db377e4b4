"""ctypes wrapper for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline.  The product
(dna-ldpc-codes_amd/) never imports it.

Wraps oracle/liboracle.so (the C restatement of LDPC_dec/ldpc/dec.cpp:583-694,
1216-1678, check.cpp:28-45, rcode.cpp:54-85; see ldpc_oracle.c) and, when
built, oracle/_ref/libref.so (the reference's own unmodified loader +
syndrome sources; see ref_harness.cpp).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ALGO_BP, ALGO_MSA = 0, 1
ALGO_QMSA, ALGO_GALLAGER_A, ALGO_GALLAGER_B1, ALGO_GALLAGER_B2 = 2, 3, 4, 5
POST_LLR, POST_RATIO = 0, 1


class _Graph(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("E", C.c_int64),
                ("row_ptr", C.POINTER(C.c_int)), ("col_idx", C.POINTER(C.c_int)),
                ("col_ptr", C.POINTER(C.c_int)), ("col_edge", C.POINTER(C.c_int))]


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so not built (run `make -C oracle`)")
        L = C.CDLL(path)
        L.oracle_graph_load.argtypes = [C.c_char_p, C.POINTER(_Graph)]
        L.oracle_graph_free.argtypes = [C.POINTER(_Graph)]
        L.oracle_check_regular.argtypes = [C.POINTER(_Graph)] + [C.POINTER(C.c_int)] * 4
        L.oracle_check.argtypes = [C.POINTER(_Graph), C.c_void_p, C.c_void_p]
        L.oracle_bp.argtypes = [C.POINTER(_Graph), C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.oracle_msa.argtypes = [C.POINTER(_Graph), C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.oracle_decode_int_batch.argtypes = [C.POINTER(_Graph), C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int,
                                              C.c_double, C.c_int, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_void_p]
        L.oracle_decode_batch.argtypes = [C.POINTER(_Graph), C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int,
                                          C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class OracleGraph:
    """Parity-check graph as loaded by the oracle (CSR rows by ascending column,
    column lists by ascending row -- mod2sparse.cpp:502-604)."""

    def __init__(self, path: str):
        self._g = _Graph()
        rc = lib().oracle_graph_load(path.encode(), C.byref(self._g))
        if rc != 0:
            raise ValueError(f"oracle_graph_load({path}) failed: {rc}")
        g = self._g
        self.M, self.N, self.E = g.M, g.N, g.E
        self.row_ptr = np.ctypeslib.as_array(g.row_ptr, (g.M + 1,)).copy()
        self.col_idx = np.ctypeslib.as_array(g.col_idx, (max(g.E, 1),))[: g.E].copy()
        self.col_ptr = np.ctypeslib.as_array(g.col_ptr, (g.N + 1,)).copy()
        self.col_edge = np.ctypeslib.as_array(g.col_edge, (max(g.E, 1),))[: g.E].copy()

    def __del__(self):
        try:
            lib().oracle_graph_free(C.byref(self._g))
        except Exception:
            pass

    def regular(self):
        v = [C.c_int() for _ in range(4)]
        lib().oracle_check_regular(C.byref(self._g), *[C.byref(x) for x in v])
        return tuple(x.value for x in v)  # (dv, regular_dv, dc, regular_dc)

    def check(self, dblk: np.ndarray):
        dblk = np.ascontiguousarray(dblk, dtype=np.uint8)
        pchk = np.zeros(self.M, np.uint8)
        c = lib().oracle_check(C.byref(self._g), _p(dblk), _p(pchk))
        return c, pchk

    def bp(self, LR: np.ndarray, max_iter: int):
        """One codeword, LR domain (dec.cpp:583).  Returns (hard, post_ratio, iters, valid)."""
        LR = np.ascontiguousarray(LR, dtype=np.float64)
        hard = np.zeros(self.N, np.uint8)
        post = np.zeros(self.N, np.float64)
        v = C.c_int()
        n = lib().oracle_bp(C.byref(self._g), _p(LR), max_iter, _p(hard), _p(post), C.byref(v))
        return hard, post, n, bool(v.value)

    def msa(self, LLR: np.ndarray, max_iter: int):
        LLR = np.ascontiguousarray(LLR, dtype=np.float64)
        hard = np.zeros(self.N, np.uint8)
        L = np.zeros(self.N, np.float64)
        v = C.c_int()
        n = lib().oracle_msa(C.byref(self._g), _p(LLR), max_iter, _p(hard), _p(L), C.byref(v))
        return hard, L, n, bool(v.value)

    def decode_batch(self, llr: np.ndarray, max_iter: int, algo: int = ALGO_BP,
                     post_mode: int = POST_LLR, threads: int = 1, want_post: bool = True):
        """Batch decode of LLRs [B][N] (BP computes LR = exp(LLR) like
        DNA_main.cpp:1344).  Returns (hard[B][N] u8, post[B][N] f64|None,
        iters[B] i32, valid[B] u8)."""
        llr = np.ascontiguousarray(llr, dtype=np.float64)
        B = llr.shape[0]
        hard = np.zeros((B, self.N), np.uint8)
        post = np.zeros((B, self.N), np.float64) if want_post else None
        iters = np.zeros(B, np.int32)
        valid = np.zeros(B, np.uint8)
        lib().oracle_decode_batch(C.byref(self._g), _p(llr), B, max_iter, algo, post_mode, threads,
                                  _p(hard), _p(post) if post is not None else None, _p(iters), _p(valid))
        return hard, post, iters, valid

    def decode_int_batch(self, llr: np.ndarray, max_iter: int, algo: int, precision: int = 6, step: float = 0.5,
                         beta: int = 0, seed: int = 0, threads: int = 1):
        """Integer decoders (algo 2 = quantized/offset min-sum, 3/4/5 =
        Gallager A/B1/B2).  Returns (hard, post, iters, valid)."""
        llr = np.ascontiguousarray(llr, dtype=np.float64)
        B = llr.shape[0]
        hard = np.zeros((B, self.N), np.uint8)
        post = np.zeros((B, self.N), np.float64)
        iters = np.zeros(B, np.int32)
        valid = np.zeros(B, np.uint8)
        rc = lib().oracle_decode_int_batch(C.byref(self._g), _p(llr), B, max_iter, algo, precision, step, beta, seed,
                                           threads, _p(hard), _p(post), _p(iters), _p(valid))
        if rc != 0:
            raise ValueError("bad integer-decoder parameters")
        return hard, post, iters, valid

# ---------------------------------------------------------------------------
# oracle/_ref: the reference's own loader + syndrome (built only where the
# reference sources exist, i.e. in the build container).
# ---------------------------------------------------------------------------
def ref_available() -> bool:
    return os.path.exists(os.path.join(_HERE, "_ref", "libref.so"))


class RefGraph:
    """The reference's mod2sparse matrix (one per process: the reference keeps
    H in a global, rcode.cpp:33)."""

    _lib = None

    @staticmethod
    def _load_lib():
        if RefGraph._lib is None:
            L = C.CDLL(os.path.join(_HERE, "_ref", "libref.so"))
            L.ref_load.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
            L.ref_try_load.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
            L.ref_rows.argtypes = [C.c_void_p, C.c_void_p]
            L.ref_rows.restype = C.c_int64
            L.ref_cols.argtypes = [C.c_void_p, C.c_void_p]
            L.ref_cols.restype = C.c_int64
            L.ref_check.argtypes = [C.c_void_p, C.c_void_p]
            RefGraph._lib = L
        return RefGraph._lib

    def __init__(self, path: str):
        M, N = C.c_int(), C.c_int()
        RefGraph._load_lib().ref_load(path.encode(), C.byref(M), C.byref(N))
        self.M, self.N = M.value, N.value

    @classmethod
    def try_load(cls, path: str):
        """read_pchk's steps without its exit() (ref_harness.cpp ref_try_load):
        (rc, graph) with rc 0 accepted, -1 open, -2 magic, -3 records.  The
        reference allocates what the header asks for: keep M and N small."""
        M, N = C.c_int(), C.c_int()
        rc = cls._load_lib().ref_try_load(path.encode(), C.byref(M), C.byref(N))
        if rc != 0:
            return rc, None
        g = cls.__new__(cls)
        g.M, g.N = M.value, N.value
        return 0, g

    def rows(self, E_hint: int):
        deg = np.zeros(self.M, np.int32)
        cols = np.zeros(E_hint, np.int32)
        k = RefGraph._lib.ref_rows(_p(deg), _p(cols))
        return deg, cols[:k]

    def cols(self, E_hint: int):
        deg = np.zeros(self.N, np.int32)
        rows = np.zeros(E_hint, np.int32)
        k = RefGraph._lib.ref_cols(_p(deg), _p(rows))
        return deg, rows[:k]

    def check(self, dblk: np.ndarray):
        dblk = np.ascontiguousarray(dblk, dtype=np.uint8)
        pchk = np.zeros(self.M, np.uint8)
        c = RefGraph._lib.ref_check(_p(dblk), _p(pchk))
        return c, pchk
