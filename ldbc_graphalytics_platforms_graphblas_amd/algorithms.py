"""Host-side mirror of the reference wrapper executables' algorithm entry points.

Each function has the name and argument meaning of the reference's wrapper
(src/main/c/src/algorithms/<alg>.cpp) and calls the libgx C ABI (include/gx.h) instead of
LAGraph.  Results are numpy arrays indexed by internal vertex id; the `serialize_*`
functions produce the exact text the reference serialisers write.
Errors raise `GxError` (the reference's OK() throws, utils.h:45-55).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _native as N
from .graphio import CSR

INT64_MAX = np.iinfo(np.int64).max


class Context:
    """One device context (gx_init): replaces LAGraph_Init (bfs.cpp:88)."""

    def __init__(self, device: int = 0):
        self._p = C.c_void_p()
        N.check(N.lib().gx_init(device, C.byref(self._p)), "gx_init")
        self.device = device

    @property
    def handle(self):
        return self._p

    def info(self):
        name = C.create_string_buffer(256)
        cus = C.c_int(0)
        N.check(N.lib().gx_device_info(self._p, name, 256, C.byref(cus)), "gx_device_info")
        return name.value.decode(), cus.value

    def set_kernel_timing(self, enable: bool) -> None:
        N.check(N.lib().gx_set_kernel_timing(self._p, int(enable)), "gx_set_kernel_timing")

    def kernel_stats(self, kernel: str):
        n = C.c_uint64(0)
        ms = C.c_double(0)
        N.check(N.lib().gx_kernel_stats(self._p, kernel.encode(), C.byref(n), C.byref(ms)), "gx_kernel_stats")
        return n.value, ms.value

    def reset_kernel_stats(self) -> None:
        N.check(N.lib().gx_reset_kernel_stats(self._p), "gx_reset_kernel_stats")

    def last_device_ms(self) -> float:
        ms = C.c_double(0)
        N.check(N.lib().gx_last_device_ms(self._p, C.byref(ms)), "gx_last_device_ms")
        return ms.value

    def close(self) -> None:
        if self._p:
            N.lib().gx_free(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Graph:
    """Device-resident adjacency (gx_graph_create): replaces LAGraph_New (bfs.cpp:78)."""

    def __init__(self, ctx: Context, csr: CSR, directed: bool):
        self.ctx = ctx
        self.n = csr.n
        self.nnz = csr.nnz
        self.directed = directed
        self.weighted = csr.vals is not None
        self._p = C.c_void_p()
        s = csr.as_c()
        N.check(N.lib().gx_graph_create(ctx.handle, C.byref(s), int(directed), C.byref(self._p)),
                "gx_graph_create")

    @property
    def handle(self):
        return self._p

    def close(self) -> None:
        if self._p:
            N.lib().gx_graph_free(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def LA_BFS(G: Graph, source_vertex: int) -> np.ndarray:
    """bfs.cpp:70-83: levels (int64), INT64_MAX for unreachable vertices."""
    out = np.empty(G.n, dtype=np.int64)
    N.check(N.lib().gx_bfs(G.handle, int(source_vertex), N.as_i64p(out)), "gx_bfs")
    return out


def LA_PR(G: Graph, damping_factor: float, iteration_num: int) -> np.ndarray:
    """pr.cpp:47-66: Graphalytics PageRank, fp64."""
    out = np.empty(G.n, dtype=np.float64)
    N.check(N.lib().gx_pagerank(G.handle, float(damping_factor), int(iteration_num), N.as_dp(out)),
            "gx_pagerank")
    return out


def LA_PR_csr(ctx: Context, csr: CSR, directed: bool, damping_factor: float, iteration_num: int,
              keep: bool = False):
    """pr.cpp:77-79 as bin/exe/pr runs it: upload + plan + iterations in one call
    (gx_pagerank_csr: the column upload overlapped with the plan).  keep=True returns
    (scores, the device graph's handle) -- free it with gx_graph_free -- as bin/exe/pr keeps the
    graph until after its end marker."""
    out = np.empty(csr.n, dtype=np.float64)
    s = csr.as_c()
    g = C.c_void_p()
    N.check(N.lib().gx_pagerank_csr(ctx.handle, C.byref(s), int(directed), float(damping_factor), int(iteration_num),
                                     N.as_dp(out), C.byref(g) if keep else None), "gx_pagerank_csr")
    return (out, g) if keep else out


def LA_SSSP(G: Graph, source_vertex: int) -> np.ndarray:
    """sssp.cpp:53-81: fp64 distances, +inf for unreachable vertices."""
    out = np.empty(G.n, dtype=np.float64)
    N.check(N.lib().gx_sssp(G.handle, int(source_vertex), N.as_dp(out)), "gx_sssp")
    return out


class SsspSplit:
    """gx_sssp_split on one device owning every vertex: the multi-GPU SSSP's per-rank path
    (1-D split, gx_sssp_split.hip) with no exchange; run(src) -> fp64 distances."""

    def __init__(self, G: Graph):
        self.G = G
        self.h = C.c_void_p()
        N.check(N.lib().gx_sssp_split_create(G.handle, 0, G.n, C.byref(self.h)), "gx_sssp_split_create")

    def run(self, source_vertex: int) -> np.ndarray:
        out = np.empty(self.G.n, dtype=np.float64)
        N.check(N.lib().gx_sssp_split_run(self.h, int(source_vertex), N.as_dp(out)), "gx_sssp_split_run")
        return out

    def close(self):
        if self.h:
            N.lib().gx_sssp_split_free(self.h)
            self.h = C.c_void_p()


def WeaklyConnectedComponents(G: Graph) -> np.ndarray:
    """wcc.cpp:39-66: component label = smallest internal vertex id of the component."""
    out = np.empty(G.n, dtype=np.uint64)
    N.check(N.lib().gx_wcc(G.handle, N.as_u64p(out)), "gx_wcc")
    return out


def LA_CDLP(G: Graph, itermax: int) -> np.ndarray:
    """cdlp.cpp:54-81: community labels (internal vertex ids)."""
    out = np.empty(G.n, dtype=np.uint64)
    N.check(N.lib().gx_cdlp(G.handle, int(itermax), N.as_u64p(out)), "gx_cdlp")
    return out


def LA_LCC(G: Graph) -> np.ndarray:
    """lcc.cpp:61-71: local clustering coefficient, fp64."""
    out = np.empty(G.n, dtype=np.float64)
    N.check(N.lib().gx_lcc(G.handle, N.as_dp(out)), "gx_lcc")
    return out


# ----------------------------------------------------------------- serialisers

# ---- op-level GraphBLAS calls (include/gx.h gx_mxv / gx_vxm / gx_mxm_masked) ----
PLUS_SECOND_FP64, MIN_SECOND_UINT64, ANY_PAIR_BOOL, MIN_PLUS_FP64, PLUS_PAIR_INT64 = range(5)
DESC_T0, DESC_MASK_COMP, DESC_REPLACE, DESC_ACCUM = 1, 2, 4, 8
_OUT_DTYPE = {PLUS_SECOND_FP64: np.float64, MIN_SECOND_UINT64: np.uint64, ANY_PAIR_BOOL: np.uint8,
              MIN_PLUS_FP64: np.float64, PLUS_PAIR_INT64: np.int64}


def _vp(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _op_vector(fn: str, G: Graph, semiring: int, u, u_present, mask, desc, w, w_present):
    out = np.array(w, dtype=_OUT_DTYPE[semiring], copy=True) if w is not None else \
        np.zeros(G.n, dtype=_OUT_DTYPE[semiring])
    outp = None if w_present is None else np.array(w_present, dtype=np.uint8, copy=True)
    uu = None if u is None else np.ascontiguousarray(u)
    up = None if u_present is None else np.ascontiguousarray(u_present, dtype=np.uint8)
    mk = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    N.check(getattr(N.lib(), fn)(G.handle, semiring, desc, _vp(mk), _vp(uu), _vp(up), _vp(out), _vp(outp)), fn)
    return out, outp


def mxv(G: Graph, semiring: int, u=None, u_present=None, mask=None, desc: int = 0, w=None, w_present=None):
    """gx_mxv: w<mask> (+)= A (+).(x) u  (GrB_mxv; A' with DESC_T0).  Returns (w, w_present)."""
    return _op_vector("gx_mxv", G, semiring, u, u_present, mask, desc, w, w_present)


def vxm(G: Graph, semiring: int, u=None, u_present=None, mask=None, desc: int = 0, w=None, w_present=None):
    """gx_vxm: w<mask> (+)= u (+).(x) A  (GrB_vxm; A' with DESC_T0).  Returns (w, w_present)."""
    return _op_vector("gx_vxm", G, semiring, u, u_present, mask, desc, w, w_present)


def mxm_masked(G: Graph, semiring: int = PLUS_PAIR_INT64, desc: int = 0) -> np.ndarray:
    """gx_mxm_masked: C<A> = A (+).(x) A' with PLUS_PAIR, one int64 per stored entry of A."""
    c = np.zeros(max(G.nnz, 1), dtype=np.int64)
    N.check(N.lib().gx_mxm_masked(G.handle, semiring, desc, N.as_i64p(c)), "gx_mxm_masked")
    return c[:G.nnz]


def _fmt_double(x: float) -> str:
    return "%.16e" % x   # ostream precision(16) + scientific (pr.cpp:26-27)


def serialize_bfs(levels: np.ndarray, mapping: np.ndarray) -> str:
    """SerializeBFSResult (bfs.cpp:11-68)."""
    return "".join(f"{int(m)} {int(l)}\n" for m, l in zip(mapping, levels))


def serialize_pr(rank: np.ndarray, mapping: np.ndarray) -> str:
    """SerializePageRankResult (pr.cpp:17-45)."""
    return "".join(f"{int(m)} {_fmt_double(x)}\n" for m, x in zip(mapping, rank))


def serialize_lcc(lcc: np.ndarray, mapping: np.ndarray) -> str:
    """SerializeLCCResult (lcc.cpp:17-59)."""
    return serialize_pr(lcc, mapping)


def serialize_sssp(dist: np.ndarray, mapping: np.ndarray) -> str:
    """SerializeSSSPResult (sssp.cpp:11-51): unreachable -> `infinity`."""
    return "".join(f"{int(m)} infinity\n" if np.isinf(x) else f"{int(m)} {_fmt_double(x)}\n"
                   for m, x in zip(mapping, dist))


def serialize_labels(labels: np.ndarray, mapping: np.ndarray) -> str:
    """SerializeCDLPResult (cdlp.cpp:21-52) / WCC: label printed as mapping[label]."""
    return "".join(f"{int(m)} {int(mapping[int(l)])}\n" for m, l in zip(mapping, labels))
