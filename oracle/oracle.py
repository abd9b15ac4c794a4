"""ctypes wrapper of oracle/liboracle.so -- the CPU restatement (gx_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / CPU baseline, never by the product path.
Parity status: pinned -- tests/test_oracle_fixtures.py checks every algorithm against the
24 Graphalytics validation outputs of the reference (tests/golden/graphalytics) and
tests/test_oracle_synthetic.py against scipy / networkx.
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
        _lib = L
    return _lib


def _arrs(csr):
    rp = np.ascontiguousarray(csr.rowptr, dtype=np.int64)
    ci = np.ascontiguousarray(csr.colidx, dtype=np.int64)
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
