"""ctypes wrapper of oracle/liboracle.so -- the CPU restatement (gx_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / CPU baseline, never by the product path.
Parity status: pinned -- tests/test_oracle_fixtures.py checks every algorithm against the
24 Graphalytics validation outputs of the reference (tests/golden/graphalytics) and
tests/test_golden_synthetic.py against committed scipy / networkx vectors
(tests/golden/make_golden.py).  The *_par functions are the multithreaded CPU baselines;
tests/test_oracle_parallel.py checks them bitwise against the serial checkers.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SO = HERE / "liboracle.so"
SRC = HERE / "gx_oracle.c"

_I64P = C.POINTER(C.c_int64)
_U64P = C.POINTER(C.c_uint64)
_DP = C.POINTER(C.c_double)

_lib = None


def build(force: bool = False) -> Path:
    if force or not SO.exists() or SO.stat().st_mtime < SRC.stat().st_mtime:
        subprocess.check_call(["gcc", "-O3", "-fPIC", "-shared", "-fopenmp", "-o", str(SO), str(SRC)])
    return SO


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(SO))
        L.orc_bfs.argtypes = [C.c_int64, _I64P, _I64P, C.c_int64, _I64P]
        L.orc_pagerank.argtypes = [C.c_int64, _I64P, _I64P, C.c_int, C.c_double, C.c_int, _DP, C.c_int]
        L.orc_sssp.argtypes = [C.c_int64, _I64P, _I64P, _DP, C.c_int64, _DP]
        L.orc_wcc.argtypes = [C.c_int64, _I64P, _I64P, _U64P]
        L.orc_cdlp.argtypes = [C.c_int64, _I64P, _I64P, C.c_int, C.c_int, _U64P, C.c_int]
        L.orc_lcc.argtypes = [C.c_int64, _I64P, _I64P, C.c_int, _DP, C.c_int]
        L.orc_max_threads.restype = C.c_int
        L.orc_mxv.argtypes = [C.c_int64, _I64P, _I64P, _DP, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                              C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_mxm_masked.argtypes = [C.c_int64, _I64P, _I64P, C.c_int, C.c_int, _I64P]
        L.orc_bfs_par.argtypes = [C.c_int64, _I64P, _I64P, C.c_int64, C.c_int, _I64P, C.c_int]
        L.orc_wcc_par.argtypes = [C.c_int64, _I64P, _I64P, _U64P, C.c_int]
        L.orc_sssp_par.argtypes = [C.c_int64, _I64P, _I64P, _DP, C.c_int64, C.c_double, _DP, C.c_int]
        _lib = L
    return _lib


def _i64(a: np.ndarray) -> np.ndarray:
    """int64 view of an index array (GrB_Index uint64 values are < 2^63): no copy, so the
    CPU baseline's timing holds the algorithm only."""
    a = np.ascontiguousarray(a)
    return a.view(np.int64) if a.dtype == np.uint64 else np.ascontiguousarray(a, dtype=np.int64)


def _arrs(csr):
    rp = _i64(csr.rowptr)
    ci = _i64(csr.colidx)
    return rp, ci, rp.ctypes.data_as(_I64P), ci.ctypes.data_as(_I64P)


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"oracle {what} failed: {rc}")


def max_threads() -> int:
    return lib().orc_max_threads()


def bfs(csr, src: int) -> np.ndarray:
    rp, ci, prp, pci = _arrs(csr)
    out = np.empty(csr.n, dtype=np.int64)
    _ok(lib().orc_bfs(csr.n, prp, pci, src, out.ctypes.data_as(_I64P)), "bfs")
    return out


def pagerank(csr, directed: bool, damping: float, iters: int, nthreads: int = 0) -> np.ndarray:
    rp, ci, prp, pci = _arrs(csr)
    out = np.empty(csr.n, dtype=np.float64)
    _ok(lib().orc_pagerank(csr.n, prp, pci, int(directed), damping, iters, out.ctypes.data_as(_DP),
                           nthreads), "pagerank")
    return out


def sssp(csr, src: int) -> np.ndarray:
    rp, ci, prp, pci = _arrs(csr)
    w = np.ascontiguousarray(csr.vals, dtype=np.float64)
    out = np.empty(csr.n, dtype=np.float64)
    _ok(lib().orc_sssp(csr.n, prp, pci, w.ctypes.data_as(_DP), src, out.ctypes.data_as(_DP)), "sssp")
    return out


def wcc(csr) -> np.ndarray:
    rp, ci, prp, pci = _arrs(csr)
    out = np.empty(csr.n, dtype=np.uint64)
    _ok(lib().orc_wcc(csr.n, prp, pci, out.ctypes.data_as(_U64P)), "wcc")
    return out


def cdlp(csr, directed: bool, iters: int, nthreads: int = 0) -> np.ndarray:
    rp, ci, prp, pci = _arrs(csr)
    out = np.empty(csr.n, dtype=np.uint64)
    _ok(lib().orc_cdlp(csr.n, prp, pci, int(directed), iters, out.ctypes.data_as(_U64P), nthreads), "cdlp")
    return out


def lcc(csr, directed: bool, nthreads: int = 0) -> np.ndarray:
    rp, ci, prp, pci = _arrs(csr)
    out = np.empty(csr.n, dtype=np.float64)
    _ok(lib().orc_lcc(csr.n, prp, pci, int(directed), out.ctypes.data_as(_DP), nthreads), "lcc")
    return out


def bfs_par(csr, src: int, symmetric: bool, nthreads: int = 0) -> np.ndarray:
    """Multithreaded direction-optimising BFS (CPU baseline); equals bfs()."""
    rp, ci, prp, pci = _arrs(csr)
    out = np.empty(csr.n, dtype=np.int64)
    _ok(lib().orc_bfs_par(csr.n, prp, pci, src, int(symmetric), out.ctypes.data_as(_I64P), nthreads), "bfs_par")
    return out


def wcc_par(csr, nthreads: int = 0) -> np.ndarray:
    """Multithreaded lock-free union-find WCC (CPU baseline); equals wcc()."""
    rp, ci, prp, pci = _arrs(csr)
    out = np.empty(csr.n, dtype=np.uint64)
    _ok(lib().orc_wcc_par(csr.n, prp, pci, out.ctypes.data_as(_U64P), nthreads), "wcc_par")
    return out


def sssp_par(csr, src: int, delta: float = 0.0, nthreads: int = 0) -> np.ndarray:
    """Multithreaded delta-stepping (CPU baseline); equals sssp() bitwise.  delta <= 0: 4 x the
    mean weight / the mean degree (the GPU default for undirected graphs)."""
    rp, ci, prp, pci = _arrs(csr)
    w = np.ascontiguousarray(csr.vals, dtype=np.float64)
    if delta <= 0:
        deg = max(1.0, csr.nnz / max(1, csr.n))
        delta = 4.0 * (float(w.mean()) if len(w) else 1.0) / deg
        delta = delta if delta > 0 else 1.0
    out = np.empty(csr.n, dtype=np.float64)
    _ok(lib().orc_sssp_par(csr.n, prp, pci, w.ctypes.data_as(_DP), src, delta, out.ctypes.data_as(_DP), nthreads),
        "sssp_par")
    return out


# op-level semirings / descriptors (include/gx.h)
PLUS_SECOND_FP64, MIN_SECOND_UINT64, ANY_PAIR_BOOL, MIN_PLUS_FP64, PLUS_PAIR_INT64 = range(5)
DESC_T0, DESC_MASK_COMP, DESC_REPLACE, DESC_ACCUM = 1, 2, 4, 8
OUT_DTYPE = {PLUS_SECOND_FP64: np.float64, MIN_SECOND_UINT64: np.uint64, ANY_PAIR_BOOL: np.uint8,
             MIN_PLUS_FP64: np.float64, PLUS_PAIR_INT64: np.int64}


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def mxv(csr, semiring: int, u=None, u_present=None, mask=None, desc: int = 0, w=None, w_present=None,
        vxm: bool = False):
    """orc_mxv: w<mask> (+)= A (+).(x) u (vxm: u (+).(x) A); returns (w, w_present) -- new arrays,
    initialised from the given w / w_present (ACCUM and kept entries read them)."""
    rp, ci, prp, pci = _arrs(csr)
    wt = None if csr.vals is None else np.ascontiguousarray(csr.vals, dtype=np.float64)
    out = np.array(w, dtype=OUT_DTYPE[semiring], copy=True) if w is not None else \
        np.zeros(csr.n, dtype=OUT_DTYPE[semiring])
    outp = None if w_present is None else np.array(w_present, dtype=np.uint8, copy=True)
    uu = None if u is None else np.ascontiguousarray(u)
    up = None if u_present is None else np.ascontiguousarray(u_present, dtype=np.uint8)
    mk = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    _ok(lib().orc_mxv(csr.n, prp, pci, None if wt is None else wt.ctypes.data_as(_DP), semiring, int(vxm), desc,
                      _ptr(mk), _ptr(uu), _ptr(up), _ptr(out), _ptr(outp)), "mxv")
    return out, outp


def mxm_masked(csr, semiring: int = PLUS_PAIR_INT64, desc: int = 0) -> np.ndarray:
    """orc_mxm_masked: C<A> = A (+).(x) A' (PLUS_PAIR), one count per stored entry of A."""
    rp, ci, prp, pci = _arrs(csr)
    c = np.zeros(csr.nnz, dtype=np.int64)
    _ok(lib().orc_mxm_masked(csr.n, prp, pci, semiring, desc, c.ctypes.data_as(_I64P)), "mxm_masked")
    return c
