"""Graph formats of the Graphalytics GraphBLAS platform, without SuiteSparse or DuckDB.

* `.v` / `.e` / `.properties`: the Graphalytics dataset files.  `relabel()` restates
  bin/py/relabel.py:8-79: vertices get dense internal ids in `.v` file order (DuckDB
  `rowid`, relabel.py:37-45); edges keep their file order and optional weight; undirected
  graphs become a `symmetric` Matrix Market file that the reader expands to both
  directions (relabel.py:47-50).
* `.vtx` / `.mtx`: the text files relabel.py writes (relabel.py:52-79).
* `.vtb` / `.grb`: the binary files the converter writes and every executable reads
  (graphio.cpp:4-60; graphio.h:49-285) -- read/written natively by libgx.

A graph is held as `CSR(n, rowptr, colidx, vals)` with uint64 arrays (GrB_Index).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import numpy as np

from . import _native as N


@dataclass
class CSR:
    n: int
    rowptr: np.ndarray           # uint64[n+1]
    colidx: np.ndarray           # uint64[nnz]
    vals: Optional[np.ndarray] = None   # float64[nnz] or None (unweighted / iso)

    @property
    def nnz(self) -> int:
        return int(self.rowptr[-1])

    def as_c(self) -> N.gx_csr:
        """Borrowed gx_csr view (keep `self` alive while the struct is used)."""
        s = N.gx_csr()
        s.n = self.n
        s.nnz = self.nnz
        s.rowptr = N.as_u64p(self.rowptr)
        s.colidx = N.as_u64p(self.colidx) if self.nnz else C.cast(None, C.POINTER(C.c_uint64))
        s.vals = N.as_dp(self.vals) if self.vals is not None else C.cast(None, C.POINTER(C.c_double))
        return s

    def out_degree(self) -> np.ndarray:
        return np.diff(self.rowptr).astype(np.uint64)

    def transpose(self) -> "CSR":
        """In-edge CSR with rows sorted by column (stable counting sort)."""
        rows = np.repeat(np.arange(self.n, dtype=np.uint64), np.diff(self.rowptr).astype(np.int64))
        order = np.lexsort((rows, self.colidx))
        cols_t = rows[order]
        rp = np.zeros(self.n + 1, dtype=np.uint64)
        np.cumsum(np.bincount(self.colidx.astype(np.int64), minlength=self.n), out=rp[1:])
        return CSR(self.n, rp, cols_t.astype(np.uint64),
                   None if self.vals is None else self.vals[order].copy())


def csr_from_edges(n: int, src: np.ndarray, dst: np.ndarray, w: Optional[np.ndarray],
                   symmetric: bool) -> CSR:
    """Sorted CSR of an edge list; symmetric adds (j, i) for every off-diagonal (i, j)."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    if symmetric:
        off = src != dst
        src, dst = np.concatenate([src, dst[off]]), np.concatenate([dst, src[off]])
        if w is not None:
            w = np.concatenate([w, w[off]])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    if w is not None:
        w = np.asarray(w, dtype=np.float64)[order]
    # duplicates keep the last occurrence (gx_read_mtx semantics)
    if len(src):
        last = np.ones(len(src), dtype=bool)
        last[:-1] = (src[1:] != src[:-1]) | (dst[1:] != dst[:-1])
        src, dst = src[last], dst[last]
        if w is not None:
            w = w[last]
    rp = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(np.bincount(src, minlength=n), out=rp[1:])
    return CSR(n, rp, dst.astype(np.uint64), None if w is None else np.ascontiguousarray(w))


# ------------------------------------------------------------------ Graphalytics files

def read_properties(path) -> dict:
    """Parse a Graphalytics `.properties` file into a flat dict."""
    props = {}
    for line in Path(path).read_text().splitlines():
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        props[k.strip()] = v.strip()
    return props


@dataclass
class GraphalyticsGraph:
    name: str
    mapping: np.ndarray   # uint64 original ids in internal order (.vtx / .vtb)
    csr: CSR
    directed: bool
    weighted: bool
    props: dict

    def param(self, alg: str, key: str, default=None):
        return self.props.get(f"graph.{self.name}.{alg}.{key}", default)


def relabel(v_path, e_path, directed: bool, weighted: bool):
    """relabel.py:37-79 restated: returns (mapping, src, dst, weights) with 0-based ids."""
    ids = np.loadtxt(v_path, dtype=np.uint64, ndmin=1)
    index = {int(x): i for i, x in enumerate(ids)}
    src, dst, w = [], [], []
    for line in Path(e_path).read_text().splitlines():
        parts = line.split()
        if not parts:
            continue
        src.append(index[int(parts[0])])
        dst.append(index[int(parts[1])])
        if weighted:
            w.append(float(parts[2]))
    return (ids.astype(np.uint64), np.array(src, dtype=np.int64), np.array(dst, dtype=np.int64),
            np.array(w, dtype=np.float64) if weighted else None)


def load_graphalytics(directory, name: str, weighted: Optional[bool] = None) -> GraphalyticsGraph:
    """Load `<name>.v/.e/.properties` the way load-graph.sh + converter would store it."""
    d = Path(directory)
    props = read_properties(d / f"{name}.properties")
    directed = props.get(f"graph.{name}.directed", "false").lower() == "true"
    if weighted is None:
        weighted = f"graph.{name}.edge-properties.names" in props
    mapping, src, dst, w = relabel(d / f"{name}.v", d / f"{name}.e", directed, weighted)
    csr = csr_from_edges(len(mapping), src, dst, w, symmetric=not directed)
    return GraphalyticsGraph(name, mapping, csr, directed, weighted, props)


def write_vtx_mtx(out_dir, mapping, src, dst, w, directed: bool) -> None:
    """Write graph.vtx + graph.mtx exactly as relabel.py:52-79 lays them out."""
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    (out / "graph.vtx").write_text("".join(f"{int(x)}\n" for x in mapping))
    element = "real" if w is not None else "integer"
    sym = "general" if directed else "symmetric"
    grb = "GrB_FP64" if w is not None else "GrB_BOOL"
    n = len(mapping)
    lines = [f"%%MatrixMarket matrix coordinate {element} {sym}", f"%%GraphBLAS {grb}",
             f"{n} {n} {len(src)}"]
    for k in range(len(src)):
        val = repr(float(w[k])) if w is not None else "1"
        lines.append(f"{int(src[k]) + 1} {int(dst[k]) + 1} {val}")
    (out / "graph.mtx").write_text("\n".join(lines) + "\n")


# ------------------------------------------------------------------ native readers

def _take_csr(s: N.gx_csr) -> CSR:
    n, nnz = int(s.n), int(s.nnz)
    rp = np.ctypeslib.as_array(s.rowptr, shape=(n + 1,)).copy()
    ci = np.ctypeslib.as_array(s.colidx, shape=(nnz,)).copy() if nnz else np.zeros(0, np.uint64)
    vals = None
    if bool(s.vals):
        vals = np.ctypeslib.as_array(s.vals, shape=(nnz,)).copy() if nnz else np.zeros(0)
    N.lib().gx_csr_release(C.byref(s))
    return CSR(n, rp, ci, vals)


def read_grb(path) -> CSR:
    s = N.gx_csr()
    N.check(N.lib().gx_read_grb(str(path).encode(), C.byref(s)), "gx_read_grb")
    return _take_csr(s)


def write_grb(path, csr: CSR) -> None:
    s = csr.as_c()
    N.check(N.lib().gx_write_grb(str(path).encode(), C.byref(s)), "gx_write_grb")


def read_mtx(path) -> CSR:
    s = N.gx_csr()
    N.check(N.lib().gx_read_mtx(str(path).encode(), C.byref(s)), "gx_read_mtx")
    return _take_csr(s)


def _read_ids(fn, path) -> np.ndarray:
    p = C.POINTER(C.c_uint64)()
    cnt = C.c_uint64(0)
    N.check(fn(str(path).encode(), C.byref(p), C.byref(cnt)), fn.__name__)
    out = np.ctypeslib.as_array(p, shape=(cnt.value,)).copy() if cnt.value else np.zeros(0, np.uint64)
    N.lib().gx_host_free(C.cast(p, C.c_void_p))
    return out


def read_vtb(path) -> np.ndarray:
    return _read_ids(N.lib().gx_read_vtb, path)


def read_vtx(path) -> np.ndarray:
    return _read_ids(N.lib().gx_read_vtx, path)


def write_vtb(path, ids: np.ndarray) -> None:
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    N.check(N.lib().gx_write_vtb(str(path).encode(), N.as_u64p(ids), len(ids)), "gx_write_vtb")


def rmat(scale: int, edgefactor: int, seed: int, undirected: bool = True, weighted: bool = False,
         a: float = 0.57, b: float = 0.19, c: float = 0.19) -> CSR:
    """Seeded R-MAT graph (SURVEY.md 8d synthetic inputs), generated natively by libgx."""
    s = N.gx_csr()
    N.check(N.lib().gx_rmat_csr(scale, edgefactor, a, b, c, seed, int(undirected), int(weighted),
                                C.byref(s)), "gx_rmat_csr")
    return _take_csr(s)
