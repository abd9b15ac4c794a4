"""Full-size parity on every BASELINE config's graph (SURVEY.md 8d stand-ins; no network for
the real datasets):
- config 4, SYN-8_5 (datagen-8_5-fb: R-MAT scale 23, ef 40, seed 85; 8.4 M vertices, 628 M
  entries): PageRank rtol 1e-12; SSSP bit-exact (gx_sssp and the 1-D split's single-rank loop);
- config 2, SYN-7_5 (datagen-7_5-fb: scale 20, ef 32, seed 75): PageRank rtol 1e-12 with the
  default plan (1 Mi-entry blocks cut into units, narrow codes, CP=0); CDLP x10 bit-exact (the
  north-star's CDLP workload);
- config 3, SYN-g500-22 (graph500-22: scale 22, ef 16, seed 22): BFS and WCC bit-exact on the
  first call and the later ones (the hub-first copy serves from the second call);
- config 5, SYN-cit (cit-Patents: directed, scale 22, ef 4, seed 3): LCC bit-exact.

Each case runs against the oracle's multithreaded restatements (oracle/gx_oracle.c; their
equality with the serial ones is tests/test_oracle_parallel.py) on the box's host cores.
"""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

PR_RTOL = 1e-12   # fp64 PageRank: row sums in a different order than the oracle's


def _graph(scale, ef, seed, undirected, weighted=False):
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context, Graph
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    csr = rmat(scale, ef, seed, undirected=undirected, weighted=weighted)
    ctx = Context(0)
    G = Graph(ctx, csr, not undirected)
    return csr, ctx, G


@pytest.fixture(scope="module")
def syn85():
    csr, ctx, G = _graph(23, 40, 85, True, weighted=True)
    yield csr, G
    G.close()
    ctx.close()


@pytest.fixture(scope="module")
def syn75():
    csr, ctx, G = _graph(20, 32, 75, True)
    yield csr, G
    G.close()
    ctx.close()


@pytest.fixture(scope="module")
def g500():
    csr, ctx, G = _graph(22, 16, 22, True)
    yield csr, G
    G.close()
    ctx.close()


@pytest.fixture(scope="module")
def syncit():
    csr, ctx, G = _graph(22, 4, 3, False)
    yield csr, G
    G.close()
    ctx.close()


def _maxdeg(csr):
    return int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))


def test_pagerank_syn85(syn85):
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syn85
    got = A.LA_PR(G, 0.85, 10)
    ref = O.pagerank(csr, False, 0.85, 10, nthreads=O.max_threads())
    np.testing.assert_allclose(got, ref, rtol=PR_RTOL, atol=0)


@pytest.mark.parametrize("env", [{"GX_PR_UNIT_BY_COST": "0", "GX_PR_WIDE_COST": "12"}, {"GX_PR_QUEUE": "0", "GX_PR_BLOCK_NNZ": "8388608"},
                                 {"GX_PR_COMBINE": "1", "GX_PR_UNIT_NNZ": "524288"}])
def test_pagerank_syn85_plan_knobs(syn85, monkeypatch, env):
    """The huge-graph plan knobs at full size on a fresh graph (the plan is cached per graph):
    units cut by entries (the round-4 plan before the cost weighting), and the launch without
    the work queue on 8 Mi blocks."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context, Graph, LA_PR
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    csr, _ = syn85
    ctx = Context(0)
    G = Graph(ctx, csr, False)
    try:
        got = LA_PR(G, 0.85, 10)
    finally:
        G.close()
        ctx.close()
    ref = O.pagerank(csr, False, 0.85, 10, nthreads=O.max_threads())
    np.testing.assert_allclose(got, ref, rtol=PR_RTOL, atol=0)


def test_sssp_syn85(syn85):
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syn85
    src = _maxdeg(csr)
    ref = O.sssp_par(csr, src, 0.0, nthreads=O.max_threads())
    assert np.array_equal(A.LA_SSSP(G, src), ref)
    assert np.array_equal(A.LA_SSSP(G, src), ref)   # second call: the hub-first copy
    sp = A.SsspSplit(G)
    try:
        assert np.array_equal(sp.run(src), ref)
    finally:
        sp.close()


def test_pagerank_syn75(syn75):
    """Config 2 (pr.cpp:61): the default plan at full size, first and warm call."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syn75
    ref = O.pagerank(csr, False, 0.85, 10, nthreads=O.max_threads())
    for _ in range(2):
        np.testing.assert_allclose(A.LA_PR(G, 0.85, 10), ref, rtol=PR_RTOL, atol=0)


def test_cdlp_syn75(syn75):
    """The north-star CDLP workload (cdlp.cpp:54-81, LAGraph_cdlp.c:264-333): 10 iterations,
    bit-exact, on the caller's order (first call) and the hub-first relabelled copy (later)."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syn75
    ref = O.cdlp(csr, False, 10, nthreads=O.max_threads())
    for call in range(3):
        got = A.LA_CDLP(G, 10)
        assert np.array_equal(got, ref), f"call {call}: {int((got != ref).sum())} labels differ"


def test_bfs_g500(g500):
    """Config 3 BFS (bfs.cpp:80) from the max-degree vertex and from a low-degree one."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = g500
    deg = np.diff(csr.rowptr.astype(np.int64))
    srcs = [_maxdeg(csr), int(np.flatnonzero(deg == 1)[0])]
    for src in srcs:
        ref = O.bfs_par(csr, src, True, nthreads=O.max_threads())
        for call in range(3):
            got = A.LA_BFS(G, src)
            assert np.array_equal(got, ref), f"src {src} call {call}: {int((got != ref).sum())} differ"


def test_wcc_g500(g500):
    """Config 3 WCC (wcc.cpp:61): canonical min-id labels, first and later calls."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = g500
    ref = O.wcc_par(csr, nthreads=O.max_threads())
    for call in range(3):
        got = A.WeaklyConnectedComponents(G)
        assert np.array_equal(got, ref), f"call {call}: {int((got != ref).sum())} labels differ"


def test_lcc_syncit(syncit):
    """Config 5 (lcc.cpp:68): directed LCC over N(v) = in u out, bit-exact (integer counts
    and one division)."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syncit
    ref = O.lcc(csr, True, nthreads=O.max_threads())
    for call in range(2):
        got = A.LA_LCC(G)
        assert np.array_equal(got, ref), f"call {call}: {int((got != ref).sum())} values differ"


def test_bfs_wcc_cdlp_syncit(syncit):
    """The directed paths at config 5's size: BFS (Aᵀ built from the second call), WCC and CDLP
    (in + out multiset, reciprocal edges twice)."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syncit
    src = _maxdeg(csr)
    ref = O.bfs_par(csr, src, False, nthreads=O.max_threads())
    for call in range(2):
        assert np.array_equal(A.LA_BFS(G, src), ref), f"bfs call {call}"
    ref = O.wcc_par(csr, nthreads=O.max_threads())
    assert np.array_equal(A.WeaklyConnectedComponents(G), ref)
    ref = O.cdlp(csr, True, 10, nthreads=O.max_threads())
    for call in range(2):
        assert np.array_equal(A.LA_CDLP(G, 10), ref), f"cdlp call {call}"


def _multi(fn, ctx_handle, csr, *args):
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    out = np.zeros(csr.n)
    arr = (C.c_void_p * 1)(ctx_handle.value)
    s = csr.as_c()
    N.check(getattr(N.lib(), fn)(arr, 1, C.byref(s), *args, N.as_dp(out)), fn)
    return out


def test_multi_paths_at_full_size(syn75, syn85):
    """The executables' GX_NGPUS paths (one device, size-1 RCCL clique) at the config sizes:
    gx_pagerank_multi on SYN-7_5 (the device-built interleaved plan) and gx_sssp_multi on
    SYN-8_5 (the exchange protocol, one host read per round)."""
    csr, G = syn75
    got = _multi("gx_pagerank_multi", G.ctx.handle, csr, 0, 0.85, 10)
    np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, 10, nthreads=O.max_threads()), rtol=PR_RTOL, atol=0)
    csr, G = syn85
    src = _maxdeg(csr)
    got = _multi("gx_sssp_multi", G.ctx.handle, csr, 0, src)
    assert np.array_equal(got, O.sssp_par(csr, src, 0.0, nthreads=O.max_threads()))


def _multi_k(fn, k, csr, *args):
    """gx_<alg>_multi on k virtual devices of this GPU (k contexts on device 0)."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    ctxs = [Context(0) for _ in range(k)]
    try:
        out = np.zeros(csr.n)
        arr = (C.c_void_p * k)(*[c.handle.value for c in ctxs])
        s = csr.as_c()
        N.check(getattr(N.lib(), fn)(arr, k, C.byref(s), *args, N.as_dp(out)), fn)
        return out
    finally:
        for c in ctxs:
            c.close()


def test_multi_virtual_devices_syn75_syncit(syn75, syncit):
    """The N = 8 path of bin/exe/pr and bin/exe/lcc at config sizes, on 8 virtual devices of one
    GPU: PageRank on SYN-7_5 (undirected) and on SYN-cit (directed: A'
    on every device, the owner * chunk + local column map), LCC on SYN-cit (config 5's
    stand-in; probe-work ranges, one reduction)."""
    csr, _ = syn75
    got = _multi_k("gx_pagerank_multi", 8, csr, 0, 0.85, 10)
    np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, 10, nthreads=O.max_threads()), rtol=PR_RTOL, atol=0)
    csr, _ = syncit
    got = _multi_k("gx_pagerank_multi", 8, csr, 1, 0.85, 10)
    np.testing.assert_allclose(got, O.pagerank(csr, True, 0.85, 10, nthreads=O.max_threads()), rtol=PR_RTOL, atol=0)
    got = _multi_k("gx_lcc_multi", 8, csr, 1)
    assert np.array_equal(got, O.lcc(csr, True, nthreads=O.max_threads()))


def test_multi_virtual_devices_syn85(syn85):
    """Config 4 (PageRank + SSSP on datagen-8_5-fb, 8 GPUs) through the executables' entry
    points on 8 virtual devices: PageRank rtol 1e-12 (a huge graph: the block partition,
    pr_multi_blocks), SSSP bit-exact."""
    csr, _ = syn85
    src = _maxdeg(csr)
    got = _multi_k("gx_sssp_multi", 8, csr, 0, src)
    assert np.array_equal(got, O.sssp_par(csr, src, 0.0, nthreads=O.max_threads()))
    got = _multi_k("gx_pagerank_multi", 8, csr, 0, 0.85, 10)
    np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, 10, nthreads=O.max_threads()), rtol=PR_RTOL, atol=0)


def _multi_k_int(fn, k, csr, dtype, *args):
    """gx_<alg>_multi with an integer result on k virtual devices of this GPU."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    ctxs = [Context(0) for _ in range(k)]
    try:
        out = np.zeros(csr.n, dtype=dtype)
        arr = (C.c_void_p * k)(*[c.handle.value for c in ctxs])
        s = csr.as_c()
        ptr = out.ctypes.data_as(C.POINTER(C.c_int64 if dtype == np.int64 else C.c_uint64))
        N.check(getattr(N.lib(), fn)(arr, k, C.byref(s), *args, ptr), fn)
        return out
    finally:
        for c in ctxs:
            c.close()


def test_multi_virtual_devices_bfs_wcc_cdlp(g500, syn75):
    """bin/exe/{bfs,wcc,cdlp}'s GX_NGPUS path at config sizes on 8 virtual devices (round 6,
    VERDICT r05 next #10): BFS and WCC on SYN-g500-22 (config 3), CDLP x10 on SYN-7_5, bit-exact."""
    csr, _ = g500
    src = _maxdeg(csr)
    got = _multi_k_int("gx_bfs_multi", 8, csr, np.int64, 0, src)
    assert np.array_equal(got, O.bfs_par(csr, src, True, nthreads=O.max_threads()))
    got = _multi_k_int("gx_wcc_multi", 8, csr, np.uint64, 0)
    assert np.array_equal(got.astype(np.int64), O.wcc_par(csr, nthreads=O.max_threads()).astype(np.int64))
    csr, _ = syn75
    got = _multi_k_int("gx_cdlp_multi", 8, csr, np.uint64, 0, 10)
    assert np.array_equal(got.astype(np.int64), O.cdlp(csr, False, 10, nthreads=O.max_threads()).astype(np.int64))
