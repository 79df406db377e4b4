"""Python ctypes shim over lib/libldpc_amd.so (include/ldpc_amd.h).

This is the in-process replacement for the reference pipeline's
``write_bat(...); os.system('soft_decoder.bat'); file_read('dec_...')`` round
trip (ex_decoder/decoder.py:553-562, 630-640; def_func.py:29-57): the .pchk is
parsed once and cached, and a whole batch of LLR vectors is decoded per call on
the GPU(s).

    import ldpc_amd as L
    hard, post, iters, valid = L.decode(llr, max_iter=200)          # llr: [B][N]
    L.decode_files("codeword_n18432_m1860_1", "soft72000_n18432_m1860_1",
                   "decode_n18432_m2048_final")                        # ldpc.exe side effects

There is deliberately no CPU fallback: if the HIP library is missing or no GPU
is visible, every decode raises.
"""
from __future__ import annotations

import ctypes as C
import enum
import math
import os
import threading
import time
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libldpc_amd.so")

ABI_VERSION = 3
LDPC_OK, LDPC_ERR_ARG, LDPC_ERR_IO, LDPC_ERR_FORMAT, LDPC_ERR_DEVICE, LDPC_ERR_UNSUPPORTED = 0, -1, -2, -3, -4, -5


class Algo(enum.IntEnum):
    """The ABI's LDPC_ALGO_* codes.  A plain int passed as `algo` is the
    reference's decoder_type instead (DECODER_TYPES below); these members are
    recognised as ABI codes by their type."""
    BP = 0
    MSA = 1
    QMSA = 2
    GALLAGER_A = 3
    GALLAGER_B1 = 4
    GALLAGER_B2 = 5


ALGO_BP, ALGO_MSA, ALGO_QMSA = Algo.BP, Algo.MSA, Algo.QMSA
ALGO_GALLAGER_A, ALGO_GALLAGER_B1, ALGO_GALLAGER_B2 = Algo.GALLAGER_A, Algo.GALLAGER_B1, Algo.GALLAGER_B2
POST_LLR, POST_RATIO = 0, 1
IN_LLR, IN_LR = 0, 1
H2D, D2H, D2D = 0, 1, 2

# Algorithm selection.  Names and Algo members select the ABI's LDPC_ALGO_*
# decoders; a plain int is the reference's decoder_type (enum DECODER_TYPE,
# DNA_main.cpp:41-53), mapped as LDPC_Decode (DNA_main.cpp:1565-1594)
# dispatches it and as bin/ldpc does: 0 BP, 1/2/3 Gallager A/B1/B2, 20/21/22
# the float min-sum Run_MSA_Decoder_INF (the DNA build never sets g_precision,
# so the quantized Run_MSA_Decoder is unreachable from a decoder_type; use
# 'qmsa' or Algo.QMSA).  A reference caller's decoder_type never silently picks
# another decoder, and neither does this module's own ALGO_* constant.
_NAMES = {"bp": ALGO_BP, "msa": ALGO_MSA, "min-sum": ALGO_MSA, "qmsa": ALGO_QMSA,
          "gallager_a": ALGO_GALLAGER_A, "gallager_b1": ALGO_GALLAGER_B1, "gallager_b2": ALGO_GALLAGER_B2}
DECODER_TYPES = {0: ALGO_BP, 1: ALGO_GALLAGER_A, 2: ALGO_GALLAGER_B1, 3: ALGO_GALLAGER_B2,
                 20: ALGO_MSA, 21: ALGO_MSA, 22: ALGO_MSA}
# decoder_type written into result file names (DNA_main.cpp:1047-1048) for a named algorithm
_RESULT_TYPE = {ALGO_BP: 0, ALGO_GALLAGER_A: 1, ALGO_GALLAGER_B1: 2, ALGO_GALLAGER_B2: 3, ALGO_MSA: 20,
                ALGO_QMSA: 21}


class LdpcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ldpc_amd error {code}: {msg}")
        self.code = code


# ldpc_schedule flag bits (include/ldpc_amd.h LDPC_SCHED_*) by keyword
SCHED_FLAGS = {"nontemporal": 1 << 0, "continuous": 1 << 3, "msa_compressed": 1 << 4, "resident": 1 << 5,
               "split_syndrome": 1 << 6, "first_from_prior": 1 << 12, "lr_table": 1 << 13,
               "debug_no_drain": 1 << 14, "debug_bad_lane": 1 << 15}
SCHED_FIELDS = ("group_tiles", "var_cpw", "pool_tiles", "poll_every", "syn_blocks")


class Schedule(C.Structure):
    """ldpc_schedule: how a decode is laid out over launches (never what it
    computes).  Schedule.make(resident=False, group_tiles=2, ...) -- unset
    keywords keep the library's defaults."""
    _fields_ = [("flags_set", C.c_int32), ("flags", C.c_int32), ("group_tiles", C.c_int32), ("var_cpw", C.c_int32),
                ("pool_tiles", C.c_int32), ("poll_every", C.c_int32), ("syn_blocks", C.c_int32),
                ("reserved", C.c_int32)]

    @classmethod
    def make(cls, **kw) -> "Schedule":
        s = cls()
        for k, v in kw.items():
            if v is None:
                continue
            if k in SCHED_FLAGS:
                s.flags_set |= SCHED_FLAGS[k]
                if v:
                    s.flags |= SCHED_FLAGS[k]
            elif k in SCHED_FIELDS:
                setattr(s, k, int(v))
            else:
                raise TypeError(f"unknown schedule keyword {k!r} (flags: {sorted(SCHED_FLAGS)}, fields: {SCHED_FIELDS})")
        return s


def _schedule(schedule) -> Optional[Schedule]:
    if schedule is None or isinstance(schedule, Schedule):
        return schedule
    return Schedule.make(**dict(schedule))


class Opts(C.Structure):
    _fields_ = [("n_devices", C.c_int32), ("devices", C.POINTER(C.c_int32)), ("chunk", C.c_int64),
                ("exp_on_host", C.c_int32), ("post_kind", C.c_int32), ("host_threads", C.c_int32),
                ("msa_precision", C.c_int32), ("msa_offset", C.c_int32), ("reserved0", C.c_int32),
                ("msa_step", C.c_double), ("tie_seed", C.c_uint64), ("schedule", C.POINTER(Schedule))]


class KernelStats(C.Structure):
    _fields_ = [("launches", C.c_int64 * 6), ("sampled", C.c_int64 * 6), ("ms", C.c_double * 6)]


KCLASS = ("check", "variable", "syndrome", "init", "finalize", "other")

_lib = None
_lib_lock = threading.Lock()

EXPORTS = [
    "ldpc_abi_version", "ldpc_last_error", "ldpc_device_count", "ldpc_graph_load", "ldpc_graph_from_edges",
    "ldpc_graph_load_alist", "ldpc_graph_rs_ldpc", "ldpc_graph_save_pchk", "ldpc_graph_save_alist",
    "ldpc_graph_free", "ldpc_graph_info", "ldpc_graph_blocks", "ldpc_graph_edges", "ldpc_graph_syndrome", "ldpc_decode",
    "ldpc_decode_codes",
    "ldpc_engine_create", "ldpc_engine_create_ex", "ldpc_engine_info", "ldpc_engine_free", "ldpc_engine_decode", "ldpc_engine_sync", "ldpc_engine_stream",
    "ldpc_engine_decode_codes", "ldpc_engine_gen_bsc", "ldpc_engine_gen_bsc_codes", "ldpc_engine_set_params", "ldpc_engine_profile", "ldpc_engine_stats", "ldpc_dev_malloc", "ldpc_dev_free",
    "ldpc_dev_memcpy", "ldpc_host_alloc", "ldpc_host_free", "ldpc_dna_llr", "ldpc_dna_llr_codes", "ldpc_dna_edit_distance", "ldpc_write_soft_files", "ldpc_py_float_repr",
]


def lib():
    """Load the HIP library (fails loudly when it has not been built)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C dna-ldpc-codes_amd` "
                              "(there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        missing = [n for n in EXPORTS if not hasattr(L, n)]
        version = L.ldpc_abi_version() if "ldpc_abi_version" not in missing else None
        if missing or version != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: ABI version {version}, this shim needs {ABI_VERSION}"
                              + (f"; missing symbols {missing}" if missing else "")
                              + " (rebuild with `make -C dna-ldpc-codes_amd`)")
        vp, i32, i64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_double
        pint = C.POINTER(C.c_int)
        L.ldpc_abi_version.restype = C.c_int
        L.ldpc_last_error.restype = C.c_char_p
        L.ldpc_device_count.restype = C.c_int
        L.ldpc_graph_load.argtypes = [C.c_char_p, pint]
        L.ldpc_graph_load.restype = vp
        L.ldpc_graph_from_edges.argtypes = [i32, i32, vp, vp, i64, pint]
        L.ldpc_graph_from_edges.restype = vp
        L.ldpc_graph_load_alist.argtypes = [C.c_char_p, i32, pint]
        L.ldpc_graph_load_alist.restype = vp
        L.ldpc_graph_rs_ldpc.argtypes = [i32, i32, i32, vp, vp, pint]
        L.ldpc_graph_rs_ldpc.restype = vp
        L.ldpc_graph_save_pchk.argtypes = [vp, C.c_char_p]
        L.ldpc_graph_save_alist.argtypes = [vp, C.c_char_p]
        L.ldpc_graph_free.argtypes = [vp]
        L.ldpc_graph_free.restype = None
        L.ldpc_graph_info.argtypes = [vp] + [vp] * 7
        L.ldpc_graph_edges.argtypes = [vp, vp, vp, vp, vp]
        L.ldpc_graph_blocks.argtypes = [vp, vp, vp, vp, vp]
        L.ldpc_graph_syndrome.argtypes = [vp, vp, vp]
        L.ldpc_decode.argtypes = [vp, vp, i64, i32, i32, vp, vp, vp, vp, C.POINTER(Opts)]
        L.ldpc_decode_codes.argtypes = [vp, vp, vp, i32, i64, i32, i32, vp, vp, vp, vp, C.POINTER(Opts)]
        L.ldpc_engine_create.argtypes = [vp, i32, i32, i64, pint]
        L.ldpc_engine_create.restype = vp
        L.ldpc_engine_create_ex.argtypes = [vp, i32, i32, i64, C.POINTER(Schedule), pint]
        L.ldpc_engine_create_ex.restype = vp
        L.ldpc_engine_info.argtypes = [vp, vp, vp, vp]
        L.ldpc_engine_free.argtypes = [vp]
        L.ldpc_engine_free.restype = None
        L.ldpc_engine_decode.argtypes = [vp, vp, i32, i64, i32, vp, vp, i32, vp, vp]
        L.ldpc_engine_decode_codes.argtypes = [vp, vp, vp, i32, i64, i32, vp, vp, i32, vp, vp]
        L.ldpc_engine_sync.argtypes = [vp]
        L.ldpc_engine_stream.argtypes = [vp]
        L.ldpc_engine_stream.restype = vp
        L.ldpc_engine_gen_bsc.argtypes = [vp, vp, i32, i64, i64, vp, i32, C.c_uint64, dbl, dbl]
        L.ldpc_engine_gen_bsc_codes.argtypes = [vp, vp, i64, i64, vp, i32, C.c_uint64, dbl]
        L.ldpc_engine_profile.argtypes = [vp, i32]
        L.ldpc_engine_set_params.argtypes = [vp, i32, dbl, i32, C.c_uint64]
        L.ldpc_engine_stats.argtypes = [vp, C.POINTER(KernelStats)]
        L.ldpc_host_alloc.argtypes = [C.c_size_t]
        L.ldpc_host_alloc.restype = vp
        L.ldpc_host_free.argtypes = [vp]
        L.ldpc_dev_malloc.argtypes = [i32, C.c_size_t]
        L.ldpc_dev_malloc.restype = vp
        L.ldpc_dev_free.argtypes = [i32, vp]
        L.ldpc_dev_memcpy.argtypes = [i32, vp, vp, C.c_size_t, i32]
        _lib = L
        return L


def _check(rc: int):
    if rc != LDPC_OK:
        raise LdpcError(rc, (lib().ldpc_last_error() or b"").decode(errors="replace"))
    return rc


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def device_count() -> int:
    return int(lib().ldpc_device_count())


def _algo(a) -> int:
    """ABI algorithm code of a name, an Algo member, or a reference decoder_type int."""
    if isinstance(a, Algo):
        return int(a)
    if isinstance(a, str):
        if a.lower() in _NAMES:
            return _NAMES[a.lower()]
    elif isinstance(a, (int, np.integer)) and not isinstance(a, bool) and int(a) in DECODER_TYPES:
        return DECODER_TYPES[int(a)]
    raise ValueError(f"unknown algorithm {a!r} (names: 'bp', 'msa', 'qmsa', 'gallager_a', 'gallager_b1', "
                     "'gallager_b2'; Algo members; ints: the reference's decoder_type 0, 1, 2, 3, 20, 21, 22)")


def _decoder_type(a) -> int:
    """The reference decoder_type a call runs as (result file names)."""
    if isinstance(a, (int, np.integer)) and not isinstance(a, (bool, Algo)):
        _algo(a)
        return int(a)
    return _RESULT_TYPE[_algo(a)]


class Graph:
    """A parity-check graph loaded from a .pchk file (read_pchk, rcode.cpp:54-85)."""

    def __init__(self, path: Optional[str] = None, *, handle=None):
        if handle is None:
            err = C.c_int(0)
            handle = lib().ldpc_graph_load(os.fsencode(path), C.byref(err))
            if not handle:
                raise LdpcError(err.value, (lib().ldpc_last_error() or b"").decode(errors="replace"))
        self._h = handle
        self.path = path
        M, N, dv, rdv, dc, rdc = (C.c_int32() for _ in range(6))
        E = C.c_int64()
        _check(lib().ldpc_graph_info(self._h, *[C.byref(x) for x in (M, N, E, dv, rdv, dc, rdc)]))
        self.M, self.N, self.E = M.value, N.value, E.value
        self.dv, self.regular_dv, self.dc, self.regular_dc = dv.value, bool(rdv.value), dc.value, bool(rdc.value)

    @classmethod
    def from_edges(cls, M: int, N: int, rows: Sequence[int], cols: Sequence[int]) -> "Graph":
        r = np.ascontiguousarray(rows, dtype=np.int32)
        c = np.ascontiguousarray(cols, dtype=np.int32)
        err = C.c_int(0)
        h = lib().ldpc_graph_from_edges(M, N, _ptr(r), _ptr(c), len(r), C.byref(err))
        if not h:
            raise LdpcError(err.value, (lib().ldpc_last_error() or b"").decode(errors="replace"))
        return cls(handle=h)

    @classmethod
    def from_alist(cls, path: str, transpose: bool = False) -> "Graph":
        """alist file -> graph with alist-to-pchk's checks (alist-to-pchk.cpp:36-160)."""
        err = C.c_int(0)
        h = lib().ldpc_graph_load_alist(os.fsencode(path), int(bool(transpose)), C.byref(err))
        if not h:
            raise LdpcError(err.value, (lib().ldpc_last_error() or b"").decode(errors="replace"))
        g = cls(handle=h)
        g.path = path
        return g

    @classmethod
    def rs_ldpc(cls, s: int, rho: int, gamma: int, tables: bool = False):
        """RS-based LDPC code of RS_LDPC.c:221-431 (q = 2^s, M = gamma*q,
        N = rho*q).  With tables=True also returns (gen_poly, coset)."""
        q = 1 << s if 2 <= s <= 10 else 0
        gp = np.zeros(max(rho - 1, 1), np.int32)
        cs = np.zeros(max(q * q, 1), np.int32)
        err = C.c_int(0)
        h = lib().ldpc_graph_rs_ldpc(s, rho, gamma, _ptr(gp), _ptr(cs), C.byref(err))
        if not h:
            raise LdpcError(err.value, (lib().ldpc_last_error() or b"").decode(errors="replace"))
        g = cls(handle=h)
        return (g, gp[: rho - 1], cs[: q * q]) if tables else g

    def save_pchk(self, path: str):
        """Write a .pchk (intio magic + mod2sparse_write, mod2sparse.cpp:338-376)."""
        _check(lib().ldpc_graph_save_pchk(self._h, os.fsencode(path)))

    def save_alist(self, path: str):
        """Write an alist file in RS_LDPC.c's layout (RS_LDPC.c:434-474)."""
        _check(lib().ldpc_graph_save_alist(self._h, os.fsencode(path)))

    def close(self):
        if getattr(self, "_h", None):
            lib().ldpc_graph_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def edges(self):
        """(row_ptr[M+1], col_idx[E], col_ptr[N+1], col_edge[E]) int32 arrays."""
        rp = np.zeros(self.M + 1, np.int32)
        ci = np.zeros(max(self.E, 1), np.int32)
        cp = np.zeros(self.N + 1, np.int32)
        ce = np.zeros(max(self.E, 1), np.int32)
        _check(lib().ldpc_graph_edges(self._h, _ptr(rp), _ptr(ci), _ptr(cp), _ptr(ce)))
        return rp, ci[: self.E], cp, ce[: self.E]

    def blocks(self):
        """Array-code block structure (ldpc_graph_blocks): (Q, row_blocks,
        col_blocks, col_block[N]) or None when H has none."""
        Q, rb, cb = C.c_int32(), C.c_int32(), C.c_int32()
        cls = np.full(self.N, -1, np.int32)
        _check(lib().ldpc_graph_blocks(self._h, C.byref(Q), C.byref(rb), C.byref(cb), _ptr(cls)))
        return None if Q.value == 0 else (Q.value, rb.value, cb.value, cls)

    def syndrome(self, dblk: np.ndarray):
        """Number of unsatisfied checks and the parity vector (check.cpp:28-45)."""
        d = np.ascontiguousarray(dblk, dtype=np.uint8)
        if d.shape != (self.N,):
            raise ValueError(f"dblk must have shape ({self.N},)")
        pchk = np.zeros(self.M, np.uint8)
        c = lib().ldpc_graph_syndrome(self._h, _ptr(d), _ptr(pchk))
        if c < 0:
            _check(c)
        return int(c), pchk

    def decode(self, llr: np.ndarray, max_iter: int = 200, algo="bp", post: Optional[str] = "llr",
               devices: Optional[Sequence[int]] = None, chunk: int = 0, exp_on_host: bool = True,
               host_threads: int = 0, msa_precision: int = 0, msa_step: float = 0.0, msa_offset: int = 0,
               tie_seed: int = 0, schedule=None):
        """Decode a batch of LLR vectors ([B][N] or [N]) on the GPU(s).

        Returns (hard u8[B][N], post f64[B][N] or None, iters i32[B], valid bool[B]);
        a 1-D input returns 1-D / scalar outputs.  post: 'llr' (log of the BP
        posterior ratio / the min-sum L), 'ratio' (BP raw posterior ratio) or
        None.  msa_* / tie_seed: parameters of algo='qmsa' (0 = defaults q 6,
        step 0.5).  schedule: a Schedule or a dict of its keywords (None: the
        library's default schedule)."""
        x = np.ascontiguousarray(llr, dtype=np.float64)
        return self._decode(x, "llr", None, IN_LLR, max_iter, algo, post, devices, chunk, exp_on_host, host_threads,
                            msa_precision, msa_step, msa_offset, tie_seed, schedule)

    def decode_codes(self, codes: np.ndarray, table: np.ndarray, table_kind: int = IN_LLR, max_iter: int = 200,
                     algo="bp", post: Optional[str] = "llr", devices: Optional[Sequence[int]] = None, chunk: int = 0,
                     host_threads: int = 0, msa_precision: int = 0, msa_step: float = 0.0, msa_offset: int = 0,
                     tie_seed: int = 0, schedule=None):
        """Decode a batch given as int8 codes ([B][N] or [N]) and a 256-entry
        table (table[k + 128] = the channel LLR of code k, or with
        table_kind=IN_LR and BP its LR) -- the DNA stage's count differences
        with table k * ln((1-eps)/eps) (decoder.py:314), ldpc_decode_codes.
        Same outputs as decode(table[codes + 128])."""
        c = np.asarray(codes)
        if c.dtype != np.int8:
            # no silent wrap-around or truncation of the caller's codes
            if not np.issubdtype(c.dtype, np.integer):
                raise TypeError(f"codes must be integers (got {c.dtype})")
            if c.size and (int(c.min()) < -128 or int(c.max()) > 127):
                raise ValueError("codes outside the int8 range [-128, 127]")
        x = np.ascontiguousarray(c, dtype=np.int8)
        t = np.ascontiguousarray(table, dtype=np.float64)
        if t.shape != (256,):
            raise ValueError("the code table has 256 entries (code + 128)")
        return self._decode(x, "codes", t, int(table_kind), max_iter, algo, post, devices, chunk, True, host_threads,
                            msa_precision, msa_step, msa_offset, tie_seed, schedule)

    def _decode(self, x, form, table, table_kind, max_iter, algo, post, devices, chunk, exp_on_host, host_threads,
                msa_precision, msa_step, msa_offset, tie_seed, schedule):
        a = _algo(algo)
        single = x.ndim == 1
        if single:
            x = x[None, :]
        if x.ndim != 2 or x.shape[1] != self.N:
            raise ValueError(f"{form} must have shape [B][{self.N}]")
        B = x.shape[0]
        hard = np.empty((B, self.N), np.uint8)
        postv = np.empty((B, self.N), np.float64) if post else None
        iters = np.zeros(B, np.int32)
        valid = np.zeros(B, np.uint8)
        o = Opts()
        devs = None
        if devices:
            devs = (C.c_int32 * len(devices))(*devices)
            o.n_devices = len(devices)
            o.devices = C.cast(devs, C.POINTER(C.c_int32))
        o.chunk = chunk
        o.exp_on_host = 1 if exp_on_host else 0
        o.post_kind = {None: POST_LLR, "llr": POST_LLR, "ratio": POST_RATIO}[post]
        o.host_threads = host_threads
        o.msa_precision, o.msa_step, o.msa_offset, o.tie_seed = int(msa_precision), float(msa_step), int(msa_offset), \
            int(tie_seed)
        sch = _schedule(schedule)
        if sch is not None:
            o.schedule = C.pointer(sch)
        if form == "codes":
            _check(lib().ldpc_decode_codes(self._h, _ptr(x), _ptr(table), table_kind, B, int(max_iter), a, _ptr(hard),
                                           _ptr(postv), _ptr(iters), _ptr(valid), C.byref(o)))
        else:
            _check(lib().ldpc_decode(self._h, _ptr(x), B, int(max_iter), a, _ptr(hard), _ptr(postv), _ptr(iters),
                                     _ptr(valid), C.byref(o)))
        valid = valid.astype(bool)
        if single:
            return hard[0], (postv[0] if postv is not None else None), int(iters[0]), bool(valid[0])
        return hard, postv, iters, valid


# ---------------------------------------------------------------------------
# module-level API: cached graphs (the .pchk is parsed once per process)
# ---------------------------------------------------------------------------
_graphs: dict = {}


def graph(pchk_path: str) -> Graph:
    key = os.path.abspath(pchk_path)
    g = _graphs.get(key)
    if g is None:
        g = Graph(pchk_path)
        _graphs[key] = g
    return g


def decode(llr: np.ndarray, max_iter: int = 200, algo="bp", pchk: Optional[str] = None, **kw):
    """Batch decode with a cached graph (default: the DNA code shipped in tests/golden)."""
    if pchk is None:
        pchk = default_pchk()
    return graph(pchk).decode(llr, max_iter=max_iter, algo=algo, **kw)


def default_pchk() -> str:
    return os.path.join(os.path.dirname(_HERE), "tests", "golden", "decode_n18432_m2048_final.pchk")


# ---------------------------------------------------------------------------
# ldpc.exe file contract, in-process (DNA_main.cpp:300-505, 916-927, 965-1123)
# ---------------------------------------------------------------------------
def _read_tokens(path: str, n: int, conv):
    with open(path, "r") as f:
        toks = f.read().split()
    if len(toks) < n:
        raise ValueError(f"{path}: expected {n} values, found {len(toks)}")
    return [conv(t) for t in toks[:n]]


def decode_files(codeword_base: str, soft_base: str, pchk_base: str, max_iter: int = 200, algo="bp",
                 seed: int = 7, EbNo: float = 0.0, directory: str = ".") -> dict:
    """Reproduce `ldpc 0 <algo> 0 <seed> <max_iter> 1 <codeword> <soft> <pchk> <EbNo> 0 0 0`
    (def_func.write_bat) in-process: reads <codeword>.txt, <soft>.txt,
    <pchk>.pchk from `directory`, writes dec_<codeword>.txt and the result file,
    and returns the statistics.  decoder.py can replace its os.system call
    (decoder.py:557-558, 635-636) with this."""
    decoder_type = _decoder_type(algo)
    j = lambda p: os.path.join(directory, p)  # noqa: E731
    g = graph(j(pchk_base + ".pchk"))
    N, M = g.N, g.M
    K = N - M
    t_start = time.time()
    cw = np.array(_read_tokens(j(codeword_base + ".txt"), N, int), dtype=np.int64)
    llr = np.array(_read_tokens(j(soft_base + ".txt"), N, float), dtype=np.float64)
    raw = int(np.sum(cw != (llr < 0)))  # LDPC_Raw_Error_Check, AWGN soft decision (DNA_main.cpp:1727-1732)
    hard, _, iters, valid = g.decode(llr, max_iter=max_iter, algo=algo, post=None)
    bit_err = int(np.sum(cw != hard))
    with open(j("dec_" + codeword_base + ".txt"), "w") as f:
        f.write("".join(f"{int(b)} " for b in hard))
    t_end = time.time()
    rate = 1.0 - M / N
    std_dev = 1 / math.sqrt(2 * rate * math.pow(10.0, EbNo * 0.1))
    name = "result_(%s.txt)_%s.pchk_%d_%.3fdB_%d_%d_%d.txt" % (soft_base, pchk_base, decoder_type, EbNo, 0,
                                                             max_iter, seed)
    d = int(t_end - t_start)
    lines = [
        f"code N        : {N}", f"code K        : {K}", f"code M        : {M}", "code rate     : %.3f" % rate,
        "Eb/No         : %.2f dB" % EbNo, "g_std_dev     : %.2f" % std_dev, f"max iteration : {max_iter}",
        f"dv            : {g.dv}", f"bRegular_dv   : {int(g.regular_dv)}", f"dc            : {g.dc}",
        f"bRegular_dc   : {int(g.regular_dc)}", "=============================================",
        "                 result", "=============================================",
        "start time      : " + time.ctime(t_start), "end time        : " + time.ctime(t_end),
        "simulation time : %d hours %d mins %d secs\n" % (d // 3600, (d % 3600) // 60, d % 60),
        "# of processes         : 1", f"initial seed value     : {seed}\n",
        "# of Frame[ 0]          :1", "# of Frame[ 1]          :1", "",
        f"# of Bit Errors[ 0]     : {raw}", f"# of Bit Errors[ 1]     : {bit_err}", "",
        "BER[ 0]                 : %.5e" % (raw / N), "BER[ 1]                 : %.5e" % (bit_err / N), "", "",
    ]
    with open(j(name), "w") as f:
        f.write("\n".join(lines))
    return {"iters": iters, "valid": valid, "bit_errors": bit_err, "raw_errors": raw, "hard": hard,
            "dec_file": "dec_" + codeword_base + ".txt", "result_file": name}


def _schedule_kw(schedule) -> dict:
    """Schedule / dict / None -> Schedule.make keywords."""
    if schedule is None:
        return {}
    if isinstance(schedule, Schedule):
        kw = {k: bool(schedule.flags & b) for k, b in SCHED_FLAGS.items() if schedule.flags_set & b}
        kw.update({k: getattr(schedule, k) for k in SCHED_FIELDS if getattr(schedule, k)})
        return kw
    return dict(schedule)


def host_empty(shape, dtype=np.int8) -> np.ndarray:
    """A numpy array in pinned host memory (ldpc_host_alloc), freed with the
    array.  Graph.decode_codes sends such an input across PCIe without a
    staging copy."""
    import weakref
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    p = lib().ldpc_host_alloc(max(n, 1))
    if not p:
        raise LdpcError(LDPC_ERR_DEVICE, (lib().ldpc_last_error() or b"").decode())
    buf = (C.c_char * max(n, 1)).from_address(p)
    weakref.finalize(buf, lib().ldpc_host_free, p)
    return np.frombuffer(buf, dt, count=int(np.prod(shape))).reshape(shape)


# ---------------------------------------------------------------------------
# device-resident engine (bench / pipelines keeping data in HBM)
# ---------------------------------------------------------------------------
class DeviceBuffer:
    def __init__(self, device: int, nbytes: int):
        self.device, self.nbytes = device, nbytes
        self.ptr = lib().ldpc_dev_malloc(device, nbytes)
        if not self.ptr:
            raise LdpcError(LDPC_ERR_DEVICE, (lib().ldpc_last_error() or b"").decode())

    def upload(self, a: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        _check(lib().ldpc_dev_memcpy(self.device, C.c_void_p(self.ptr + offset), _ptr(a), a.nbytes, H2D))

    def download(self, a: np.ndarray, offset: int = 0):
        assert a.flags.c_contiguous and offset + a.nbytes <= self.nbytes
        _check(lib().ldpc_dev_memcpy(self.device, _ptr(a), C.c_void_p(self.ptr + offset), a.nbytes, D2H))
        return a

    def at(self, offset: int):
        return C.c_void_p(self.ptr + offset)

    def free(self):
        if self.ptr:
            lib().ldpc_dev_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Engine:
    """Device-resident decoder (ldpc_engine_*): one device, one HIP stream.
    The schedule comes from `schedule` (a Schedule or dict) and/or the
    keyword shortcuts (group_tiles, nontemporal, continuous, resident, ...,
    any Schedule.make keyword); unset ones keep the library defaults.  Values
    pass through as the ABI defines them (group_tiles 0 = default, < 0 = the
    whole pass)."""

    def __init__(self, g: Graph, device: int = 0, algo="bp", chunk: int = 0, schedule=None, **sched_kw):
        self.g, self.device, self.algo = g, device, _algo(algo)
        kw = dict(_schedule_kw(schedule))
        kw.update({k: v for k, v in sched_kw.items() if v is not None})
        sch = Schedule.make(**kw)
        err = C.c_int(0)
        self._h = lib().ldpc_engine_create_ex(g.handle, device, self.algo, chunk, C.byref(sch), C.byref(err))
        if not self._h:
            raise LdpcError(err.value, (lib().ldpc_last_error() or b"").decode())
        cap, grp, fl = C.c_int64(), C.c_int64(), C.c_int32()
        _check(lib().ldpc_engine_info(self._h, C.byref(cap), C.byref(grp), C.byref(fl)))
        self.cap, self.group_tiles, self.flags = cap.value, grp.value, fl.value
        f = fl.value
        self.nontemporal = bool(f & SCHED_FLAGS["nontemporal"])
        self.continuous = bool(f & SCHED_FLAGS["continuous"])
        self.msa_compressed = bool(f & SCHED_FLAGS["msa_compressed"])  # min-sum c2v as per-row records + meta words
        self.resident = bool(f & SCHED_FLAGS["resident"])  # in-place pool of a few tiles
        self.syndrome_split = bool(f & SCHED_FLAGS["split_syndrome"])  # multi-block continuous-mode syndrome
        self.first_from_prior = bool(f & SCHED_FLAGS["first_from_prior"])

    def decode(self, d_in, in_kind: int, B: int, max_iter: int, d_hard=None, d_post=None, post_kind=POST_LLR,
               d_iters=None, d_valid=None):
        _check(lib().ldpc_engine_decode(self._h, d_in, in_kind, B, max_iter, d_hard, d_post, post_kind, d_iters,
                                        d_valid))

    def decode_codes(self, d_codes, table: np.ndarray, table_kind: int, B: int, max_iter: int, d_hard=None,
                     d_post=None, post_kind=POST_LLR, d_iters=None, d_valid=None):
        """Decode int8 channel codes [B][N] (device) with table[code + 128] the
        channel value of a code (ldpc_engine_decode_codes)."""
        t = np.ascontiguousarray(table, dtype=np.float64)
        if t.shape != (256,):
            raise ValueError("the code table has 256 entries (code + 128)")
        _check(lib().ldpc_engine_decode_codes(self._h, d_codes, _ptr(t), table_kind, B, max_iter, d_hard, d_post,
                                              post_kind, d_iters, d_valid))

    def set_params(self, msa_precision: int = 6, msa_step: float = 0.5, msa_offset: int = 0, tie_seed: int = 0):
        """Quantized min-sum parameters (Set_MSA dec.cpp:1683)."""
        _check(lib().ldpc_engine_set_params(self._h, msa_precision, msa_step, msa_offset, tie_seed))

    def gen_bsc(self, d_out, out_kind: int, b0: int, B: int, d_cw, n_cw: int, seed: int, p: float, llr_mag: float):
        _check(lib().ldpc_engine_gen_bsc(self._h, d_out, out_kind, b0, B, d_cw, n_cw, seed, p, llr_mag))

    def gen_bsc_codes(self, d_out, b0: int, B: int, d_cw, n_cw: int, seed: int, p: float):
        _check(lib().ldpc_engine_gen_bsc_codes(self._h, d_out, b0, B, d_cw, n_cw, seed, p))

    def sync(self):
        _check(lib().ldpc_engine_sync(self._h))

    def profile(self, stride: int):
        """HIP-event timing of every `stride`-th launch per kernel class (0: off)."""
        _check(lib().ldpc_engine_profile(self._h, int(stride)))

    def stats(self) -> dict:
        s = KernelStats()
        _check(lib().ldpc_engine_stats(self._h, C.byref(s)))
        return {k: {"launches": int(s.launches[i]), "sampled": int(s.sampled[i]), "ms": float(s.ms[i])}
                for i, k in enumerate(KCLASS)}

    def close(self):
        if getattr(self, "_h", None):
            lib().ldpc_engine_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
