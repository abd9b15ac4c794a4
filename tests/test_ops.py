"""Op-level GraphBLAS ABI (include/gx.h gx_mxv / gx_vxm / gx_mxm_masked).

CPU: the oracle's restatement (orc_mxv, orc_mxm_masked) is pinned by composing the reference's
algorithms out of it -- PageRank from PLUS_SECOND mxv over A' (LAGr_PageRankGX, pr.cpp:61), BFS
from ANY_PAIR vxm under the complemented visited mask (bfs.cpp:80), SSSP from MIN_PLUS vxm
(sssp.cpp:78), WCC from MIN_SECOND mxv label propagation (wcc.cpp:61), LCC's triangle counts from
the PLUS_PAIR masked mxm (lcc.cpp:68) -- and checking each against the algorithm oracle that
tests/test_oracle_fixtures.py pins to the Graphalytics validation files; and by a dense numpy
restatement on small random graphs.
GPU: every semiring, mxv and vxm, with and without transpose, masks (plain / complemented,
replace or not), accumulation and presence, bit-exact against the oracle (PLUS_SECOND_FP64 sums
within 1e-12 relative: the GPU adds in another order).
"""
import numpy as np
import pytest

from oracle import oracle as O
from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat

SEMIRINGS = [O.PLUS_SECOND_FP64, O.MIN_SECOND_UINT64, O.ANY_PAIR_BOOL, O.MIN_PLUS_FP64, O.PLUS_PAIR_INT64]


def dense(csr):
    n = csr.n
    A = np.zeros((n, n))
    S = np.zeros((n, n), dtype=bool)
    rows = np.repeat(np.arange(n), np.diff(csr.rowptr.astype(np.int64)))
    cols = csr.colidx.astype(np.int64)
    S[rows, cols] = True
    A[rows, cols] = 1.0 if csr.vals is None else csr.vals
    return A, S


def numpy_mxv(csr, sr, u, up, vxm, t0):
    """Dense restatement of t = M (+).(x) u (no mask / accum): (values, presence)."""
    A, S = dense(csr)
    use_t = vxm != t0
    M, MS = (A.T, S.T) if use_t else (A, S)
    n = csr.n
    up = np.ones(n, bool) if up is None else up.astype(bool)
    t = np.zeros(n, dtype=O.OUT_DTYPE[sr])
    hit = np.zeros(n, bool)
    for i in range(n):
        js = np.nonzero(MS[i] & up)[0]
        hit[i] = len(js) > 0
        if sr == O.PLUS_SECOND_FP64:
            t[i] = sum((M[i, j] if vxm else u[j]) for j in js) if len(js) else 0.0
        elif sr == O.MIN_SECOND_UINT64:
            t[i] = min((sat_u64(M[i, j]) if vxm else u[j]) for j in js) if len(js) else np.iinfo(np.uint64).max
        elif sr == O.ANY_PAIR_BOOL:
            t[i] = 1 if len(js) else 0
        elif sr == O.MIN_PLUS_FP64:
            t[i] = min(u[j] + M[i, j] for j in js) if len(js) else np.inf
        else:
            t[i] = len(js)
    return t, hit


def sat_u64(x):
    """GraphBLAS's fp64 -> uint64 typecast (GB_cast_to_uint64_t): NaN and x <= 0 -> 0, x >= 2^64 ->
    UINT64_MAX, else truncation."""
    if not x > 0.0:
        return np.uint64(0)
    if x >= 18446744073709551616.0:
        return np.uint64(np.iinfo(np.uint64).max)
    return np.uint64(int(x))


def odd_weights(csr, seed=5):
    """The same graph with weights GraphBLAS must saturate: negative, NaN, above 2^64, fractional."""
    import copy
    rng = np.random.default_rng(seed)
    out = copy.copy(csr)
    pool = np.array([-3.5, np.nan, 2.0 ** 70, 0.75, 7.9, 1e19, 0.0, 42.0])
    out.vals = pool[rng.integers(0, len(pool), csr.nnz)]
    return out


def rand_u(sr, n, rng):
    if sr == O.MIN_SECOND_UINT64:
        return rng.integers(0, 1 << 40, n).astype(np.uint64)
    if sr in (O.PLUS_SECOND_FP64, O.MIN_PLUS_FP64):
        return rng.random(n)
    return None


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("undirected", [True, False])
def test_oracle_ops_match_dense_restatement(undirected, weighted):
    csr = rmat(6, 4, 11, undirected=undirected, weighted=weighted)
    rng = np.random.default_rng(3)
    for sr in SEMIRINGS:
        for vxm in (False, True):
            for t0 in (False, True):
                u = rand_u(sr, csr.n, rng)
                up = (rng.random(csr.n) < 0.7).astype(np.uint8)
                got, gp = O.mxv(csr, sr, u, up, desc=O.DESC_T0 if t0 else 0, w_present=np.zeros(csr.n, np.uint8),
                                vxm=vxm)
                want, hit = numpy_mxv(csr, sr, u, up, vxm, t0)
                np.testing.assert_array_equal(gp.astype(bool), hit)
                if sr == O.PLUS_SECOND_FP64:
                    np.testing.assert_allclose(got, want, rtol=1e-14)
                else:
                    np.testing.assert_array_equal(got, want)
    # C<A> = A A' (PLUS_PAIR)
    A, S = dense(csr)
    C = S.astype(np.int64) @ S.T.astype(np.int64)
    rows = np.repeat(np.arange(csr.n), np.diff(csr.rowptr.astype(np.int64)))
    np.testing.assert_array_equal(O.mxm_masked(csr), C[rows, csr.colidx.astype(np.int64)])


def test_oracle_mask_accum_replace():
    csr = rmat(6, 4, 5, undirected=False, weighted=True)
    n = csr.n
    rng = np.random.default_rng(9)
    u = rng.random(n)
    mask = (rng.random(n) < 0.5).astype(np.uint8)
    w0 = rng.random(n)
    wp0 = (rng.random(n) < 0.5).astype(np.uint8)
    t, hit = numpy_mxv(csr, O.MIN_PLUS_FP64, u, None, True, False)
    for desc in [0, O.DESC_MASK_COMP, O.DESC_REPLACE, O.DESC_ACCUM, O.DESC_ACCUM | O.DESC_MASK_COMP | O.DESC_REPLACE]:
        got, gp = O.mxv(csr, O.MIN_PLUS_FP64, u, None, mask, desc, w0, wp0, vxm=True)
        allowed = (mask != 0) != bool(desc & O.DESC_MASK_COMP)
        for i in range(n):
            if not allowed[i]:
                if desc & O.DESC_REPLACE:
                    assert gp[i] == 0 and got[i] == np.inf
                else:
                    assert gp[i] == wp0[i] and got[i] == w0[i]
            elif (desc & O.DESC_ACCUM) and wp0[i]:
                assert gp[i] == 1 and got[i] == (min(w0[i], t[i]) if hit[i] else w0[i])
            else:
                assert gp[i] == hit[i] and got[i] == (t[i] if hit[i] else np.inf)


# ---- the reference's algorithms composed from the ops (pins the op oracle to the fixtures) ----

def pagerank_from_mxv(mxv, csr, directed, d, iters):
    n = csr.n
    outdeg = np.diff(csr.rowptr.astype(np.int64)).astype(np.float64)
    r = np.full(n, 1.0 / n)
    sink = outdeg == 0
    for _ in range(iters):
        dangling = r[sink].sum()
        w = np.where(sink, 0.0, r / np.where(sink, 1.0, outdeg / d))
        t, _ = mxv(O.PLUS_SECOND_FP64, w, O.DESC_T0)   # t = A' w (pull over in-edges)
        r = (1 - d) / n + d / n * dangling + t
    return r


def bfs_from_vxm(vxm, n, src):
    level = np.full(n, np.iinfo(np.int64).max)
    level[src] = 0
    q = np.zeros(n, np.uint8)
    q[src] = 1
    visited = q.copy()
    depth = 0
    while q.any():
        depth += 1
        # q<!visited, replace> = q ANY.PAIR A
        nq, _ = vxm(O.ANY_PAIR_BOOL, None, q, visited, O.DESC_MASK_COMP | O.DESC_REPLACE)
        q = nq.astype(np.uint8)
        level[q != 0] = depth
        visited |= q
    return level


def sssp_from_vxm(vxm, n, src):
    dist = np.full(n, np.inf)
    dist[src] = 0.0
    present = np.zeros(n, np.uint8)
    present[src] = 1
    while True:   # Bellman-Ford: d = min(d, d MIN.PLUS A) until no change
        nd, npres = vxm(O.MIN_PLUS_FP64, dist, present, None, O.DESC_ACCUM, dist, present)
        if np.array_equal(nd, dist):
            return dist
        dist, present = nd, npres


def wcc_from_mxv(mxv, csr):
    """min-label propagation over A and A' (the LOR symmetrisation of wcc.cpp:54-55)."""
    lab = np.arange(csr.n, dtype=np.uint64)
    while True:
        a, _ = mxv(O.MIN_SECOND_UINT64, lab, 0, lab)
        b, _ = mxv(O.MIN_SECOND_UINT64, a, O.DESC_T0, a)
        if np.array_equal(b, lab):
            return lab
        lab = b


def oracle_ops():
    def mk(csr):
        return (lambda sr, u, desc, w=None: O.mxv(csr, sr, u, None, None, desc | (O.DESC_ACCUM if w is not None else 0),
                                                   w, None),
                lambda sr, u, up, mask, desc, w=None, wp=None: O.mxv(csr, sr, u, up, mask, desc, w, wp, vxm=True))
    return mk


@pytest.mark.parametrize("name", ["example-directed", "example-undirected", "test-pr-directed", "test-pr-undirected",
                                  "test-bfs-directed", "test-sssp-undirected", "test-wcc-directed"])
def test_algorithms_from_oracle_ops_match_pinned_oracle(fixture_graphs, name):
    g = fixture_graphs(name)
    csr = g.csr
    mxv, vxm = oracle_ops()(csr)
    np.testing.assert_allclose(pagerank_from_mxv(mxv, csr, g.directed, 0.85, 8),
                               O.pagerank(csr, g.directed, 0.85, 8), rtol=1e-13)
    for src in range(min(csr.n, 4)):
        np.testing.assert_array_equal(bfs_from_vxm(vxm, csr.n, src), O.bfs(csr, src))
        if csr.vals is not None:
            np.testing.assert_array_equal(sssp_from_vxm(vxm, csr.n, src), O.sssp(csr, src))
    np.testing.assert_array_equal(wcc_from_mxv(mxv, csr), O.wcc(csr))
    if not g.directed:
        # undirected LCC numerator: triangles at v = sum of C<A>(v, .) / 2
        c = O.mxm_masked(csr)
        rows = np.repeat(np.arange(csr.n), np.diff(csr.rowptr.astype(np.int64)))
        tri2 = np.bincount(rows, weights=c, minlength=csr.n)
        deg = np.diff(csr.rowptr.astype(np.int64)).astype(np.float64)
        with np.errstate(invalid="ignore", divide="ignore"):
            lcc = np.where(deg >= 2, tri2 / (deg * (deg - 1)), 0.0)
        np.testing.assert_allclose(lcc, O.lcc(csr, False), rtol=1e-15, atol=0)


# ---------------------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def gpu_ctx():
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    c = Context(0)
    yield c
    c.close()


def gpu_ops(G):
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    return (lambda sr, u, desc, w=None: A.mxv(G, sr, u, None, None, desc | (A.DESC_ACCUM if w is not None else 0), w),
            lambda sr, u, up, mask, desc, w=None, wp=None: A.vxm(G, sr, u, up, mask, desc, w, wp))


def test_oracle_min_second_saturates():
    """MIN_SECOND_UINT64 vxm takes the matrix value as uint64 the way GraphBLAS typecasts it
    (a plain cast is undefined for negative, NaN and huge weights)."""
    csr = odd_weights(rmat(6, 4, 11, undirected=False, weighted=True))
    u = np.arange(csr.n, dtype=np.uint64)
    for t0 in (False, True):
        want, hit = numpy_mxv(csr, O.MIN_SECOND_UINT64, u, None, True, t0)
        got, gp = O.mxv(csr, O.MIN_SECOND_UINT64, u, None, None, O.DESC_T0 if t0 else 0, None,
                        np.zeros(csr.n, np.uint8), vxm=True)
        np.testing.assert_array_equal(gp.astype(bool), hit)
        np.testing.assert_array_equal(got[hit], want[hit])


@pytest.mark.gpu
def test_gpu_min_second_saturates(gpu_ctx):
    """The device's MIN_SECOND_UINT64 vxm saturates fp64 -> uint64 like the oracle."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr = odd_weights(rmat(9, 8, 7, undirected=False, weighted=True))
    G = A.Graph(gpu_ctx, csr, directed=True)
    try:
        u = np.arange(csr.n, dtype=np.uint64)
        for desc in (0, A.DESC_T0):
            p0 = np.zeros(csr.n, np.uint8)
            got, gp = A.vxm(G, O.MIN_SECOND_UINT64, u, None, None, desc, None, p0)
            want, wp = O.mxv(csr, O.MIN_SECOND_UINT64, u, None, None, desc, None, p0, vxm=True)
            np.testing.assert_array_equal(gp, wp)
            np.testing.assert_array_equal(got, want)
    finally:
        G.close()


@pytest.mark.gpu
@pytest.mark.parametrize("undirected,weighted,scale", [(True, True, 10), (False, True, 10), (True, False, 12),
                                                      (False, False, 9)])
def test_gpu_ops_match_oracle(gpu_ctx, undirected, weighted, scale):
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr = rmat(scale, 8, 17 + scale, undirected=undirected, weighted=weighted)
    G = A.Graph(gpu_ctx, csr, directed=not undirected)
    rng = np.random.default_rng(scale)
    n = csr.n
    try:
        for sr in SEMIRINGS:
            for vxm in (False, True):
                for desc in [0, A.DESC_T0, A.DESC_MASK_COMP | A.DESC_REPLACE, A.DESC_ACCUM | A.DESC_T0,
                             A.DESC_ACCUM | A.DESC_MASK_COMP]:
                    u = rand_u(sr, n, rng)
                    up = None if desc & A.DESC_T0 else (rng.random(n) < 0.6).astype(np.uint8)
                    mask = (rng.random(n) < 0.5).astype(np.uint8) if desc & A.DESC_MASK_COMP else None
                    w0 = rand_u(sr, n, rng) if sr not in (O.ANY_PAIR_BOOL, O.PLUS_PAIR_INT64) else \
                        rng.integers(0, 2 if sr == O.ANY_PAIR_BOOL else 100, n).astype(O.OUT_DTYPE[sr])
                    wp0 = (rng.random(n) < 0.5).astype(np.uint8)
                    fn = A.vxm if vxm else A.mxv
                    got, gp = fn(G, sr, u, up, mask, desc, w0, wp0)
                    want, wp = O.mxv(csr, sr, u, up, mask, desc, w0, wp0, vxm=vxm)
                    np.testing.assert_array_equal(gp, wp, err_msg=f"presence sr={sr} vxm={vxm} desc={desc}")
                    if sr == O.PLUS_SECOND_FP64:
                        np.testing.assert_allclose(got, want, rtol=1e-12, atol=0,
                                                   err_msg=f"sr={sr} vxm={vxm} desc={desc}")
                    else:
                        np.testing.assert_array_equal(got, want, err_msg=f"sr={sr} vxm={vxm} desc={desc}")
        np.testing.assert_array_equal(A.mxm_masked(G), O.mxm_masked(csr))
    finally:
        G.close()


@pytest.mark.gpu
def test_gpu_algorithms_from_ops(gpu_ctx, fixture_graphs):
    """The same compositions as on the CPU, each op running on the device (PageRank's mxv is the
    k_pr_pull_units kernel itself)."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    for name in ["example-directed", "example-undirected", "test-pr-directed", "test-sssp-undirected"]:
        g = fixture_graphs(name)
        G = A.Graph(gpu_ctx, g.csr, directed=g.directed)
        try:
            mxv, vxm = gpu_ops(G)
            np.testing.assert_allclose(pagerank_from_mxv(mxv, g.csr, g.directed, 0.85, 8),
                                       O.pagerank(g.csr, g.directed, 0.85, 8), rtol=1e-12)
            for src in range(min(g.csr.n, 3)):
                np.testing.assert_array_equal(bfs_from_vxm(vxm, g.csr.n, src), O.bfs(g.csr, src))
                if g.csr.vals is not None:
                    np.testing.assert_array_equal(sssp_from_vxm(vxm, g.csr.n, src), O.sssp(g.csr, src))
            np.testing.assert_array_equal(wcc_from_mxv(mxv, g.csr), O.wcc(g.csr))
        finally:
            G.close()


@pytest.mark.gpu
def test_gpu_pr_mxv_on_large_graph(gpu_ctx):
    """PLUS_SECOND mxv over A' through the PageRank kernel on a graph with LONG rows and
    multi-unit blocks, plus the presence pass."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr = rmat(16, 16, 5, undirected=True)
    G = A.Graph(gpu_ctx, csr, directed=False)
    try:
        rng = np.random.default_rng(1)
        u = rng.random(csr.n)
        up = (rng.random(csr.n) < 0.9).astype(np.uint8)
        got, gp = A.mxv(G, A.PLUS_SECOND_FP64, u, up, None, A.DESC_T0, None, np.zeros(csr.n, np.uint8))
        want, wp = O.mxv(csr, O.PLUS_SECOND_FP64, u, up, None, O.DESC_T0, None, np.zeros(csr.n, np.uint8))
        np.testing.assert_array_equal(gp, wp)
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)
    finally:
        G.close()
