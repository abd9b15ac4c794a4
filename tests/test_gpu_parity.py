"""HIP path vs the oracle and vs the Graphalytics validation outputs (runs on the MI355X).

Bars: bit-exact for BFS levels, WCC labels, CDLP labels, SSSP distances and
LCC values (integer counts + one fp64 division); PageRank within 1e-12 relative of the fp64
oracle (the GPU sums each row in a different order) and 1e-4 of the validation files.
"""
import numpy as np
import pytest

from conftest import VALIDATION, FIXTURES, alg_params, check_against_validation, internal_index, \
    read_validation, split_validation
from oracle import oracle as O

pytestmark = pytest.mark.gpu

PR_RTOL = 1e-12


@pytest.fixture(scope="module")
def ctx():
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    c = Context(0)
    yield c
    c.close()


def gpu_run(ctx, g, alg, **p):
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    G = A.Graph(ctx, g.csr if not isinstance(g, tuple) else g[0], g.directed if not isinstance(g, tuple) else g[1])
    try:
        if alg == "BFS":
            return A.LA_BFS(G, p["source"])
        if alg == "SSSP":
            return A.LA_SSSP(G, p["source"])
        if alg == "PR":
            return A.LA_PR(G, p["damping"], p["iters"])
        if alg == "WCC":
            return A.WeaklyConnectedComponents(G)
        if alg == "CDLP":
            return A.LA_CDLP(G, p["iters"])
        if alg == "LCC":
            return A.LA_LCC(G)
    finally:
        G.close()
    raise AssertionError(alg)


@pytest.mark.parametrize("name", VALIDATION)
def test_gpu_matches_validation(ctx, name, fixture_graphs):
    graph, alg = split_validation(name)
    g = fixture_graphs(graph)
    p = alg_params(g, alg)
    if "source" in p:
        p["source"] = internal_index(g.mapping, p["source"])
    got = gpu_run(ctx, g, alg, **p)
    check_against_validation(alg, g.mapping, got, read_validation(FIXTURES / name))


class _G:
    def __init__(self, csr, directed):
        self.csr = csr
        self.directed = directed


def _rmat(scale, ef, seed, undirected=True, weighted=False):
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    return _G(rmat(scale, ef, seed, undirected=undirected, weighted=weighted), not undirected)


SYNTH = [
    # (scale, edgefactor, seed, undirected)
    (10, 8, 1, True),
    (12, 16, 2, True),
    (11, 8, 3, False),
    (14, 16, 4, True),
]


def _src(g):
    deg = np.diff(g.csr.rowptr.astype(np.int64))
    return int(np.argmax(deg))


@pytest.mark.parametrize("spec", SYNTH)
def test_bfs_synthetic(ctx, spec):
    g = _rmat(*spec)
    s = _src(g)
    np.testing.assert_array_equal(gpu_run(ctx, g, "BFS", source=s), O.bfs(g.csr, s))


@pytest.mark.parametrize("spec", SYNTH)
def test_pagerank_synthetic(ctx, spec):
    g = _rmat(*spec)
    want = O.pagerank(g.csr, g.directed, 0.85, 10)
    got = gpu_run(ctx, g, "PR", damping=0.85, iters=10)
    np.testing.assert_allclose(got, want, rtol=PR_RTOL, atol=0)


@pytest.mark.parametrize("spec", SYNTH)
def test_wcc_synthetic(ctx, spec):
    g = _rmat(*spec)
    np.testing.assert_array_equal(gpu_run(ctx, g, "WCC"), O.wcc(g.csr))


@pytest.mark.parametrize("spec", SYNTH)
def test_cdlp_synthetic(ctx, spec):
    g = _rmat(*spec)
    np.testing.assert_array_equal(gpu_run(ctx, g, "CDLP", iters=10), O.cdlp(g.csr, g.directed, 10))


@pytest.mark.parametrize("spec", SYNTH)
def test_lcc_synthetic(ctx, spec):
    g = _rmat(*spec)
    np.testing.assert_array_equal(gpu_run(ctx, g, "LCC"), O.lcc(g.csr, g.directed))


@pytest.mark.parametrize("spec", SYNTH)
def test_sssp_synthetic(ctx, spec):
    scale, ef, seed, und = spec
    g = _rmat(scale, ef, seed, undirected=und, weighted=True)
    s = _src(g)
    np.testing.assert_array_equal(gpu_run(ctx, g, "SSSP", source=s), O.sssp(g.csr, s))


def test_long_rows_pagerank(ctx):
    """A star plus a clique: rows far longer than the stream block (split segments)."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    n = 40000
    hub = np.zeros(n - 1, dtype=np.int64)
    leaves = np.arange(1, n, dtype=np.int64)
    src = np.concatenate([hub, leaves[:100]])
    dst = np.concatenate([leaves, leaves[100:200]])
    csr = csr_from_edges(n, src, dst, None, symmetric=True)
    g = _G(csr, False)
    want = O.pagerank(csr, False, 0.85, 5)
    got = gpu_run(ctx, g, "PR", damping=0.85, iters=5)
    np.testing.assert_allclose(got, want, rtol=PR_RTOL, atol=0)
    gd = _G(csr_from_edges(n, src, dst, None, symmetric=False), True)
    want = O.pagerank(gd.csr, True, 0.85, 5)
    got = gpu_run(ctx, gd, "PR", damping=0.85, iters=5)
    np.testing.assert_allclose(got, want, rtol=PR_RTOL, atol=0)


def test_empty_and_isolated(ctx):
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    csr = csr_from_edges(5, np.array([0]), np.array([1]), np.array([0.5]), symmetric=False)
    g = _G(csr, True)
    np.testing.assert_array_equal(gpu_run(ctx, g, "BFS", source=0), O.bfs(csr, 0))
    np.testing.assert_array_equal(gpu_run(ctx, g, "WCC"), O.wcc(csr))
    np.testing.assert_array_equal(gpu_run(ctx, g, "CDLP", iters=3), O.cdlp(csr, True, 3))
    np.testing.assert_array_equal(gpu_run(ctx, g, "LCC"), O.lcc(csr, True))
    np.testing.assert_array_equal(gpu_run(ctx, g, "SSSP", source=0), O.sssp(csr, 0))
    np.testing.assert_allclose(gpu_run(ctx, g, "PR", damping=0.85, iters=3),
                               O.pagerank(csr, True, 0.85, 3), rtol=PR_RTOL)
    e = csr_from_edges(4, np.zeros(0, np.int64), np.zeros(0, np.int64), None, symmetric=True)
    ge = _G(e, False)
    np.testing.assert_allclose(gpu_run(ctx, ge, "PR", damping=0.85, iters=4),
                               O.pagerank(e, False, 0.85, 4), rtol=PR_RTOL)
    np.testing.assert_array_equal(gpu_run(ctx, ge, "CDLP", iters=2), O.cdlp(e, False, 2))
    np.testing.assert_array_equal(gpu_run(ctx, ge, "WCC"), O.wcc(e))


def test_dense_tiers(ctx):
    """A 700-clique inside a sparse random graph (directed and undirected): oriented rows of
    up to 699 entries exercise LCC's workgroup tier, and degrees past 512 the CDLP mid tiers."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    rng = np.random.default_rng(7)
    n, k = 5000, 700
    a, b = np.triu_indices(k, 1)
    flip = rng.random(len(a)) < 0.5   # direct each clique edge one way or the other
    src = np.concatenate([np.where(flip, a, b), rng.integers(0, n, 20000)])
    dst = np.concatenate([np.where(flip, b, a), rng.integers(0, n, 20000)])
    keep = src != dst
    for directed in (False, True):
        csr = csr_from_edges(n, src[keep], dst[keep], None, symmetric=not directed)
        g = _G(csr, directed)
        np.testing.assert_array_equal(gpu_run(ctx, g, "LCC"), O.lcc(csr, directed))
        np.testing.assert_array_equal(gpu_run(ctx, g, "CDLP", iters=4), O.cdlp(csr, directed, 4))


@pytest.mark.parametrize("laneperm", ["0", "1"])
def test_pagerank_long_row_segments(ctx, monkeypatch, laneperm):
    """A hub row of 150 000 entries, longer than a column-sorted block: LONG segments
    combined by the last arriver, beside sorted blocks of random edges (with and without the
    LDS-bank lane permutation)."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    monkeypatch.setenv("GX_PR_LANEPERM", laneperm)
    n = 150001
    rng = np.random.default_rng(3)
    a, b = rng.integers(1, n, 200000), rng.integers(1, n, 200000)
    keep = a != b
    src = np.concatenate([np.zeros(n - 1, np.int64), a[keep]])
    dst = np.concatenate([np.arange(1, n, dtype=np.int64), b[keep]])
    csr = csr_from_edges(n, src, dst, None, symmetric=True)
    np.testing.assert_allclose(gpu_run(ctx, _G(csr, False), "PR", damping=0.85, iters=6),
                               O.pagerank(csr, False, 0.85, 6), rtol=PR_RTOL, atol=0)


@pytest.mark.parametrize("env", [{}, {"GX_PR_LANEPERM": "0"}, {"GX_PR_BLOCK_NNZ": "2097152", "GX_PR_UNIT_NNZ": "16384"},
                                 {"GX_PR_CP": "1"}, {"GX_PR_CP": "5", "GX_PR_NT_COL": "1000"}, {"GX_PR_NARROW": "0"},
                                 {"GX_PR_NARROW": "0", "GX_PR_CP": "5"}, {"GX_PR_SORT_GROUP_BITS": "1"},
                                 {"GX_PR_WIDE_KEYS": "1"},
                                 {"GX_PR_KERNEL": "adaptive"},
                                 {"GX_PR_SORTED_ROWS": "16384", "GX_PR_UNIT_NNZ": "16384"},
                                 {"GX_PR_SORTED_ROWS": "64"}, {"GX_PR_SORTED_ROWS": "2048"},
                                 {"GX_PR_UNIT_NNZ": "8192", "GX_PR_BLOCK_NNZ": "65536"},
                                 {"GX_PR_UNIT_NNZ": "8192", "GX_PR_BLOCK_NNZ": "524288"},
                                 {"GX_PR_UNIT_NNZ": "8192", "GX_PR_BLOCK_NNZ": "65536", "GX_PR_LONG_NNZ": "1024"},
                                 {"GX_PR_UNIT_NNZ": "1024", "GX_PR_BLOCK_NNZ": "8192"},
                                 {"GX_PR_UNIT_NNZ": "1024", "GX_PR_BLOCK_NNZ": "8192", "GX_PR_SORTED_ROWS": "64",
                                  "GX_PR_LANEPERM": "0"},
                                 {"GX_PR_NARROW_MIN": "4096"}, {"GX_PR_NARROW_MIN": "1073741824"},
                                 {"GX_PR_WIDE_COST": "64", "GX_PR_ROW_COST": "0", "GX_PR_UNIT_NNZ": "8192"},
                                 {"GX_PR_ROW_COST": "1024", "GX_PR_BLOCK_NNZ": "65536"},
                                 {"GX_PR_QUEUE": "1"}, {"GX_PR_QUEUE": "0"},
                                 {"GX_PR_COMBINE": "1", "GX_PR_UNIT_NNZ": "8192", "GX_PR_BLOCK_NNZ": "65536"},
                                 {"GX_PR_COMBINE": "1", "GX_PR_UNIT_NNZ": "1024", "GX_PR_BLOCK_NNZ": "8192",
                                  "GX_PR_SORTED_ROWS": "64"},
                                 {"GX_PR_COMBINE": "1", "GX_PR_QUEUE": "1", "GX_PR_UNIT_NNZ": "1024",
                                  "GX_PR_BLOCK_NNZ": "65536", "GX_PR_LONG_NNZ": "1024"},
                                 {"GX_PR_QUEUE": "1", "GX_PR_UNIT_NNZ": "1024", "GX_PR_BLOCK_NNZ": "8192",
                                  "GX_PR_LONG_NNZ": "1024", "GX_PR_CP": "5", "GX_PR_NT_COL": "1000"},
                                 {"GX_PR_PACE": "1", "GX_PR_PACE_H": "1024", "GX_PR_PACE_W": "10"},
                                 {"GX_PR_PACE": "1", "GX_PR_PACE_H": "0", "GX_PR_PACE_W": "11", "GX_PR_PACE_D": "0",
                                  "GX_PR_UNIT_NNZ": "8192", "GX_PR_BLOCK_NNZ": "65536"},
                                 {"GX_PR_PACE": "1", "GX_PR_PACE_H": "4096", "GX_PR_PACE_W": "12", "GX_PR_CP": "5",
                                  "GX_PR_NT_COL": "1000", "GX_PR_UNIT_NNZ": "8192", "GX_PR_BLOCK_NNZ": "524288"}])
def test_pagerank_plan_variants(ctx, monkeypatch, env):
    """The default plan, non-temporal index loads and sparse narrow gathers (GX_PR_CP=1 / 5, the large-graph default), the plan's key sort in groups of two segments or with 64-bit keys, without the lane permutation, blocks cut into many units, tiny blocks, 16 Ki- / 2 Ki- / 64-row blocks, split
    blocks (several workgroups per sorted block, combined through slabs by the last arriver, or
    by the stripes of the combine kernel, GX_PR_COMBINE=1)
    and the CSR-Adaptive kernel all give the oracle's scores (directed and undirected)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for g in (_rmat(14, 16, 4), _rmat(11, 8, 3, undirected=False)):
        np.testing.assert_allclose(gpu_run(ctx, g, "PR", damping=0.85, iters=10),
                                   O.pagerank(g.csr, g.directed, 0.85, 10), rtol=PR_RTOL, atol=0)


@pytest.mark.parametrize("unit", [None, "8192"])
def test_pagerank_narrow_fillers(ctx, monkeypatch, unit):
    """Narrow 2-byte codes whose column steps need fillers: a 6-regular multiplicative graph
    (v ~ 5v, 7v, 11v mod n, every degree equal, so the hub-first order is the identity) gives
    every block column steps of all sizes; the per-block split puts some blocks' prefixes in
    narrow codes with fillers and leaves the rest wide.  Also with blocks cut into units."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    if unit:
        monkeypatch.setenv("GX_PR_UNIT_NNZ", unit)
    n = 200003   # prime: v -> m v is a permutation
    v = np.arange(1, n, dtype=np.int64)
    src = np.concatenate([v, v, v])
    dst = np.concatenate([(5 * v) % n, (7 * v) % n, (11 * v) % n])
    keep = src != dst
    csr = csr_from_edges(n, src[keep], dst[keep], None, symmetric=True)
    np.testing.assert_allclose(gpu_run(ctx, _G(csr, False), "PR", damping=0.85, iters=8),
                               O.pagerank(csr, False, 0.85, 8), rtol=PR_RTOL, atol=0)


def test_pagerank_narrow_exact_supergroups(ctx, monkeypatch):
    """Blocks whose narrow codes fill whole 512-code supergroups exactly (complete bipartite
    graph K(512, 1024), 64-row blocks: 65 536 and 32 768 codes, no fillers): the base of the
    supergroup after a block's last code belongs to the next block and must not be written."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    monkeypatch.setenv("GX_PR_SORTED_ROWS", "64")
    monkeypatch.setenv("GX_PR_BLOCK_NNZ", "131072")
    monkeypatch.setenv("GX_PR_UNIT_NNZ", "16384")
    a = np.repeat(np.arange(512, dtype=np.int64), 1024)
    b = np.tile(np.arange(512, 1536, dtype=np.int64), 512)
    csr = csr_from_edges(1536, a, b, None, symmetric=True)
    np.testing.assert_allclose(gpu_run(ctx, _G(csr, False), "PR", damping=0.85, iters=5),
                               O.pagerank(csr, False, 0.85, 5), rtol=PR_RTOL, atol=0)


def test_pagerank_escape_groups(ctx, monkeypatch):
    """A perfect matching on 2^21 + 64 vertices in 64-row blocks: the columns of a block's one
    256-entry supergroup span more than 2^18 ids, so it escapes to plain column ids (permuted
    with the rest of its 64-entry groups by the lane permutation)."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    monkeypatch.setenv("GX_PR_SORTED_ROWS", "64")
    n = (1 << 21) + 64
    perm = np.random.default_rng(9).permutation(n)
    csr = csr_from_edges(n, perm[0::2], perm[1::2], None, symmetric=True)
    np.testing.assert_allclose(gpu_run(ctx, _G(csr, False), "PR", damping=0.85, iters=4),
                               O.pagerank(csr, False, 0.85, 4), rtol=PR_RTOL, atol=0)


@pytest.mark.parametrize("laneperm", ["1", "0"])
def test_pagerank_mixed_escape_rounds(ctx, monkeypatch, laneperm):
    """Escape and packed supergroups in the same round: 1 Ki rows each linked to the 96 lowest
    ids (packed supergroups) and to a partner far away (a perfect matching over 2^20 ids: the
    tail supergroups of a block escape), in 1 Ki-row blocks cut into 8 Ki-entry units."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    monkeypatch.setenv("GX_PR_SORTED_ROWS", "1024")
    monkeypatch.setenv("GX_PR_UNIT_NNZ", "8192")
    monkeypatch.setenv("GX_PR_LANEPERM", laneperm)
    n = 1 << 20
    perm = np.random.default_rng(10).permutation(n)
    dense_r = np.repeat(np.arange(96, 4096, dtype=np.int64), 96)
    dense_c = np.tile(np.arange(96, dtype=np.int64), 4096 - 96)
    csr = csr_from_edges(n, np.concatenate([perm[0::2], dense_r]), np.concatenate([perm[1::2], dense_c]), None,
                         symmetric=True)
    np.testing.assert_allclose(gpu_run(ctx, _G(csr, False), "PR", damping=0.85, iters=4),
                               O.pagerank(csr, False, 0.85, 4), rtol=PR_RTOL, atol=0)


@pytest.mark.parametrize("env", [{"GX_SSSP_PULL": "0"}, {"GX_SSSP_PULL": "2"},
                                 {"GX_SSSP_PULL": "2", "GX_SSSP_DSCALE": "2"},
                                 {"GX_SSSP_PULL": "2", "GX_SSSP_DSCALE": "200"},
                                 {"GX_SSSP_PULL_FRAC": "50", "GX_SSSP_DSCALE": "5"},
                                 {"GX_SSSP_FUSE": "0"}, {"GX_SSSP_FUSE": "300", "GX_SSSP_DSCALE": "0.5"},
                                 {"GX_SSSP_FUSE_MAX": "3", "GX_SSSP_DSCALE": "1"},
                                 {"GX_SSSP_DELTA": "0.01"}, {"GX_SSSP_DELTA": "1000"},
                                 {"GX_SSSP_DENSE": "0"}, {"GX_SSSP_DENSE": "1000000"},
                                 {"GX_SSSP_DENSE": "1000000", "GX_SSSP_FUSE": "0", "GX_SSSP_DSCALE": "0.5"},
                                 {"GX_SSSP_DENSE": "1000000", "GX_SSSP_DELTA": "0.01"}])
def test_sssp_pull_heavy_phase(ctx, monkeypatch, env):
    """Heavy phases pushed, always pulled, and pulled only for big settled lists, over narrow
    and wide buckets, with buckets opened one at a time or fused (GX_SSSP_FUSE entries,
    GX_SSSP_FUSE_MAX buckets), give the oracle's distances bit for bit -- also with integer
    weights (ties at bucket boundaries) and on a directed graph (where the pull is never used)."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = _rmat(13, 16, 5, weighted=True)
    s = _src(g)
    np.testing.assert_array_equal(gpu_run(ctx, g, "SSSP", source=s), O.sssp(g.csr, s))
    rng = np.random.default_rng(11)
    n = 5000
    a = rng.integers(0, n, 60000)
    b = rng.integers(0, n, 60000)
    a, b = np.unique(np.stack([np.minimum(a, b), np.maximum(a, b)]), axis=1)   # one weight per edge
    w = rng.integers(1, 8, len(a)).astype(np.float64)
    csr = csr_from_edges(n, a, b, w, symmetric=True)
    np.testing.assert_array_equal(gpu_run(ctx, _G(csr, False), "SSSP", source=0), O.sssp(csr, 0))
    gd = _rmat(12, 8, 6, undirected=False, weighted=True)
    s = _src(gd)
    np.testing.assert_array_equal(gpu_run(ctx, gd, "SSSP", source=s), O.sssp(gd.csr, s))


@pytest.mark.parametrize("graph_replay", ["1", "0"])
def test_sssp_repeated_runs_reuse_work_buffers(ctx, monkeypatch, graph_replay):
    """Runs from several sources on one resident graph reuse the cached work buffers (and the
    captured step graph): every run starts from a clean state."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    monkeypatch.setenv("GX_SSSP_GRAPH", graph_replay)
    g = _rmat(12, 16, 7, weighted=True)
    G = A.Graph(ctx, g.csr, g.directed)
    try:
        deg = np.diff(g.csr.rowptr.astype(np.int64))
        for s in (int(np.argmax(deg)), 0, int(np.argmax(deg)), g.csr.n - 1):
            np.testing.assert_array_equal(A.LA_SSSP(G, s), O.sssp(g.csr, s))
    finally:
        G.close()


@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_bfs_directed_transpose_policy(ctx, monkeypatch, mode):
    """Directed BFS: top-down only (0), bottom-up over the cached transpose from the second run
    (1, default) or from the first (2) -- every run gives the oracle's levels."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    monkeypatch.setenv("GX_BFS_TRANSPOSE", mode)
    for spec in ((13, 8, 21), (12, 4, 22)):
        g = _rmat(*spec, undirected=False)
        G = A.Graph(ctx, g.csr, g.directed)
        try:
            deg = np.diff(g.csr.rowptr.astype(np.int64))
            for s in (int(np.argmax(deg)), 1, int(np.argmax(deg))):
                np.testing.assert_array_equal(A.LA_BFS(G, s), O.bfs(g.csr, s))
        finally:
            G.close()


def test_wcc_directed_sparse_many_components(ctx):
    """Directed WCC (sampling + one link pass): sparse R-MAT graphs with many components, and
    chains whose edges all point away from the component minimum (seen from one end only)."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    for spec in ((14, 2, 31), (13, 1, 32), (15, 4, 33)):
        g = _rmat(*spec, undirected=False)
        np.testing.assert_array_equal(gpu_run(ctx, g, "WCC"), O.wcc(g.csr))
    n = 20000
    perm = np.random.default_rng(5).permutation(n)
    src, dst = perm[1:], perm[:-1]          # one long chain in random id order
    keep = np.arange(n - 1) % 97 != 0        # cut into ~200 components
    csr = csr_from_edges(n, src[keep], dst[keep], None, symmetric=False)
    np.testing.assert_array_equal(gpu_run(ctx, _G(csr, True), "WCC"), O.wcc(csr))


def _tier_graph(directed: bool):
    """CDLP tier boundaries in one graph: a star of 10 000 leaves (the huge tier), hubs of
    degree ~3 000 and ~6 000 (the 4 096- and 8 192-degree workgroup tiers), and rows of
    degree exactly 128 and 129 (the two light-tier table instances), over a sparse random
    background.  Several leaves share a few labels, so labels agree after a few iterations
    and the wave-aggregated insert sees groups of more than one lane."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    rng = np.random.default_rng(11)
    n = 30000
    src, dst = [], []
    def star(center, leaves):
        src.append(np.full(len(leaves), center, np.int64))
        dst.append(np.asarray(leaves, np.int64))
    # centers 0-4 take no other edge; leaves and background live in [5, n)
    star(0, np.arange(5, 10005))                                  # huge tier (> 8 192)
    star(1, rng.choice(np.arange(5, n), 3000, replace=False))     # 2 049-4 096
    star(2, rng.choice(np.arange(5, n), 6000, replace=False))     # 4 097-8 192
    star(3, rng.choice(np.arange(5, n), 128, replace=False))      # exactly 128
    star(4, rng.choice(np.arange(5, n), 129, replace=False))      # exactly 129
    # background: vertices also link to a few shared labels
    src.append(rng.integers(5, n, 40000))
    dst.append(rng.integers(5, 55, 40000))
    s, d = np.concatenate(src), np.concatenate(dst)
    keep = s != d
    return csr_from_edges(n, s[keep], d[keep], None, symmetric=not directed)


@pytest.mark.parametrize("directed", [False, True])
def test_cdlp_tier_boundaries(ctx, directed):
    """CDLP over every degree tier and the 128/129 light-tier split, against the oracle."""
    csr = _tier_graph(directed)
    deg = np.diff(csr.rowptr.astype(np.int64))
    if not directed:
        assert {128, 129} <= set(deg.tolist()) and deg.max() > 8192
    g = _G(csr, directed)
    for iters in (1, 3, 6):
        np.testing.assert_array_equal(gpu_run(ctx, g, "CDLP", iters=iters), O.cdlp(csr, directed, iters))


@pytest.mark.parametrize("active,lag", [("1", "2"), ("0", "2"), ("1", "1")])
def test_cdlp_active_set(ctx, monkeypatch, active, lag):
    """From the third iteration gx_cdlp recomputes only the neighbours of the last iteration's
    changes (GX_CDLP_ACTIVE=0: every vertex): labels equal the oracle's at every count, on
    graphs whose labels settle and on ones that keep oscillating (directed and undirected),
    with the fixed-point exit read two iterations late (the default) or one (GX_CDLP_LAG=1)."""
    monkeypatch.setenv("GX_CDLP_ACTIVE", active)
    monkeypatch.setenv("GX_CDLP_LAG", lag)
    for g in (_rmat(14, 16, 4), _rmat(12, 4, 8), _rmat(11, 8, 3, undirected=False), _G(_tier_graph(False), False),
              _G(_tier_graph(True), True)):
        for iters in (2, 3, 5, 12):
            np.testing.assert_array_equal(gpu_run(ctx, g, "CDLP", iters=iters), O.cdlp(g.csr, g.directed, iters))


def _shuffle_rows(csr, seed=0):
    """The same graph with every row's columns in a random order."""
    import copy
    rng = np.random.default_rng(seed)
    out = copy.copy(csr)
    rp = csr.rowptr.astype(np.int64)
    keys = np.repeat(np.arange(len(rp) - 1), np.diff(rp)) * 2.0 + rng.random(int(rp[-1]))
    out.colidx = csr.colidx[np.argsort(keys, kind="stable")]
    return out


@pytest.mark.parametrize("first_sorted", ["1", "0"])
@pytest.mark.parametrize("sparse,only", [("1", "1"), ("1", "2"), ("1", "0"), ("0", "1")])
def test_cdlp_row_order_and_sparse(ctx, monkeypatch, first_sorted, sparse, only):
    """The first iteration of an undirected graph with sorted rows takes each row's first
    column (GX_CDLP_FIRST_SORTED=0: the tier kernels' minimum); rows in random order take the
    tier kernels.  Sparse iterations recompute listed active vertices (GX_CDLP_SPARSE=0: the
    tier kernels' act checks); sparse-only iterations launch no tier kernel but the huge ones
    (GX_CDLP_SPARSE_ONLY=2: every active iteration, so overflowing ones take the fallback
    lists).  Same labels as the oracle either way."""
    monkeypatch.setenv("GX_CDLP_FIRST_SORTED", first_sorted)
    monkeypatch.setenv("GX_CDLP_SPARSE", sparse)
    monkeypatch.setenv("GX_CDLP_SPARSE_ONLY", only)
    g = _rmat(13, 8, 21)
    shuffled = _shuffle_rows(g.csr)
    assert not np.array_equal(shuffled.colidx, g.csr.colidx)
    for csr in (g.csr, shuffled):
        for iters in (1, 2, 4, 9):
            np.testing.assert_array_equal(gpu_run(ctx, _G(csr, False), "CDLP", iters=iters), O.cdlp(csr, False, iters))
    t = _tier_graph(True)
    for iters in (4, 9):
        np.testing.assert_array_equal(gpu_run(ctx, _G(t, True), "CDLP", iters=iters), O.cdlp(t, True, iters))


def _reciprocal_graph():
    """A directed graph for the first-iteration shortcut: short rows (one thread compares both
    rows) with and without reciprocal edges, self loops, isolated vertices, vertices with only
    in- or only out-edges, and long rows (more than 16 entries, one wave each) whose smallest
    reciprocal neighbour sits past the first 64 entries of the shorter row or is absent."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    rng = np.random.default_rng(5)
    n = 5000
    src, dst = [rng.integers(0, n, 12000)], [rng.integers(0, n, 12000)]
    r = rng.integers(0, n, 3000)                      # reciprocal pairs
    src += [r, (r * 7 + 3) % n]
    dst += [(r * 7 + 3) % n, r]
    loops = rng.integers(0, n, 200)                   # self loops
    src.append(loops)
    dst.append(loops)
    # vertex 10: 300 out-edges to 1000.., 250 in-edges from 900..; the in-row is the shorter
    # one and its first reciprocal entry (1000) is its 101st
    src += [np.full(300, 10), np.arange(900, 1150)]
    dst += [np.arange(1000, 1300), np.full(250, 10)]
    # vertex 11: 100 out, 90 in, no reciprocal neighbour
    src += [np.full(100, 11), np.arange(2000, 2090)]
    dst += [np.arange(3000, 3100), np.full(90, 11)]
    # vertex 12: 17 out-edges, 2 in-edges, one reciprocal (4321): past every per-lane limit
    src += [np.full(17, 12), np.array([4321, 4000])]
    dst += [np.arange(4310, 4327), np.full(2, 12)]
    s, d = np.concatenate(src).astype(np.int64), np.concatenate(dst).astype(np.int64)
    ok = ~np.isin(s, [10, 11, 12]) & ~np.isin(d, [10, 11, 12])
    ok[-(300 + 250 + 100 + 90 + 17 + 2):] = True      # the crafted rows keep only their own edges
    ok &= (s < 4990) | (d < 4990)                     # a few vertices isolated
    ok &= ~np.isin(s, np.arange(4990, n)) & ~np.isin(d, np.arange(4990, n))
    return csr_from_edges(n, s[ok], d[ok], None, symmetric=False)


@pytest.mark.parametrize("first_sorted,small,med", [("1", "8", "32"), ("1", "4", "64"), ("1", "16", "0"),
                                                   ("1", "8", "100000"), ("0", "8", "32")])
def test_cdlp_first_directed(ctx, monkeypatch, first_sorted, small, med):
    """The first iteration of a directed graph whose rows (A and A') are strictly sorted is the
    smallest reciprocal neighbour, else the smallest neighbour of either direction
    (k_cdlp_first_dir: rows up to GX_CDLP_FIRST_SMALL entries in one lane, up to
    GX_CDLP_FIRST_MED merged by 16-lane groups, longer ones by the wave; GX_CDLP_FIRST_SORTED=0:
    the tier kernels' count); rows in random order take the tier kernels.  Same labels as the
    oracle every time."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    monkeypatch.setenv("GX_CDLP_FIRST_SORTED", first_sorted)
    monkeypatch.setenv("GX_CDLP_FIRST_SMALL", small)
    monkeypatch.setenv("GX_CDLP_FIRST_MED", med)
    rc = _reciprocal_graph()
    want1 = O.cdlp(rc, True, 1)
    assert want1[10] == 1000 and want1[11] == 2000 and want1[12] == 4321
    cases = [rc, _rmat(13, 8, 21, undirected=False).csr, _tier_graph(True), _shuffle_rows(rc)]
    ctx.set_kernel_timing(True)
    try:
        for i, csr in enumerate(cases):
            G = A.Graph(ctx, csr, True)
            try:
                for iters in (1, 2, 5):
                    ctx.reset_kernel_stats()
                    np.testing.assert_array_equal(A.LA_CDLP(G, iters), O.cdlp(csr, True, iters))
                    ran = ctx.kernel_stats("cdlp_first")[0]
                    if first_sorted == "0" or i == 3:
                        assert ran == 0
                    elif i == 0:
                        assert ran == 1   # the crafted graph is duplicate-free, so its rows qualify
            finally:
                G.close()
    finally:
        ctx.set_kernel_timing(False)


@pytest.mark.parametrize("directed", [False, True])
def test_cdlp_huge_table_epochs(ctx, directed):
    """The huge tier's global tables are emptied by a new epoch per iteration, and cleared for
    real once the 63 epochs are used up: many calls on one graph (the tables live in its cache)
    run through the wrap, every result equal to the oracle's."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    t = _tier_graph(directed)
    G = A.Graph(ctx, t, directed)
    try:
        want = {k: O.cdlp(t, directed, k) for k in (2, 3, 4, 5)}
        for call in range(40):
            k = 2 + call % 4
            np.testing.assert_array_equal(A.LA_CDLP(G, k), want[k])
    finally:
        G.close()


@pytest.mark.parametrize("bound", ["1", "0"])
def test_cdlp_recount_bound(ctx, monkeypatch, bound):
    """Vertices whose label provably keeps a strict majority skip their recount in active
    iterations (GX_CDLP_BOUND, the default: the count when the label was last computed minus
    the changed neighbour entries k_cdlp_mark counts since), in every sparse role and the huge
    tier (degree > 8192).  Repeated calls on one graph (the relabelled copy from the second),
    iteration counts through the sparse phase, equal to the oracle's."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    monkeypatch.setenv("GX_CDLP_BOUND", bound)
    for g in (_rmat(16, 48, 7), _G(_tier_graph(False), False), _rmat(15, 40, 5, undirected=False),
              _rmat(14, 16, 4), _rmat(12, 4, 8)):
        deg = np.diff(g.csr.rowptr.astype(np.int64))
        G = A.Graph(ctx, g.csr, g.directed)
        try:
            for k in (3, 6, 10, 10):
                np.testing.assert_array_equal(A.LA_CDLP(G, k), O.cdlp(g.csr, g.directed, k))
        finally:
            G.close()
        assert g.directed or deg.max() > 8192 or g.csr.n < 30000


@pytest.mark.parametrize("keep,only,asub", [("1", "1", None), ("1", "2", None), ("1", "0", None), ("0", "1", None),
                                            ("1", "1", "2"), ("1", "2", "2")])
@pytest.mark.parametrize("relabel", ["1", "0"])
@pytest.mark.parametrize("sorted_", ["1", "0"])
def test_cdlp_own_label_check(ctx, monkeypatch, keep, only, asub, relabel, sorted_):
    """Dense active iterations take the own-label check (GX_CDLP_KEEP, the default): vertices
    whose label more than half of their neighbours hold keep it, the rest go to the sparse
    kernels' lists and k_cdlp_tiny; with tiny lists (GX_CDLP_ASUB=2) they overflow and the
    iteration stays dense (every tier kernel).  Sparse-only iterations (GX_CDLP_SPARSE_ONLY=2)
    run the check without tier kernels.  Same labels as the oracle, directed and undirected,
    on the caller's order and the relabelled copy; the count on column-sorted blocks
    (GX_CDLP_KEEP_SORTED, the default on the relabelled copy) or on 64-entry slabs."""
    monkeypatch.setenv("GX_CDLP_KEEP", keep)
    monkeypatch.setenv("GX_CDLP_KEEP_SORTED", sorted_)
    monkeypatch.setenv("GX_CDLP_SPARSE_ONLY", only)
    monkeypatch.setenv("GX_CDLP_RELABEL", relabel)
    if asub:
        monkeypatch.setenv("GX_CDLP_ASUB", asub)
    for g in (_rmat(14, 16, 4), _rmat(12, 4, 8), _rmat(11, 8, 3, undirected=False), _rmat(13, 48, 5),
              _rmat(12, 24, 6, undirected=False), _G(_tier_graph(False), False), _G(_tier_graph(True), True)):
        for iters in (3, 4, 7):
            np.testing.assert_array_equal(gpu_run(ctx, g, "CDLP", iters=iters), O.cdlp(g.csr, g.directed, iters))


@pytest.mark.parametrize("relabel", ["1", "0"])
def test_cdlp_layouts(ctx, monkeypatch, relabel):
    """gx_cdlp on the hub-first relabelled graph (GX_CDLP_RELABEL, the default) or the caller's
    order: label values stay the caller's vertex ids, so both layouts match the oracle
    exactly."""
    monkeypatch.setenv("GX_CDLP_RELABEL", relabel)
    for g in (_rmat(12, 16, 2), _rmat(11, 8, 3, undirected=False), _G(_tier_graph(False), False),
              _G(_tier_graph(True), True)):
        for iters in (1, 3, 10):
            np.testing.assert_array_equal(gpu_run(ctx, g, "CDLP", iters=iters), O.cdlp(g.csr, g.directed, iters))


@pytest.mark.parametrize("env", [{"GX_WCC_HOOK0": "0", "GX_WCC_MINHOOK": "0"}, {"GX_WCC_MINHOOK": "0"},
                                 {"GX_WCC_MINHOOK": "3"}, {}])
def test_wcc_sampling_modes(ctx, monkeypatch, env):
    """Afforest's sampling rounds with CAS links only, with the plain-store first round, and
    with min-hook passes before the second round's links: the same canonical labels, on
    undirected and directed graphs, sparse ones with many components and shuffled rows."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for g in (_rmat(14, 16, 4), _rmat(14, 2, 31), _rmat(13, 1, 32, undirected=False), _rmat(12, 8, 3, undirected=False)):
        np.testing.assert_array_equal(gpu_run(ctx, g, "WCC"), O.wcc(g.csr))
    g = _rmat(13, 4, 9)
    shuffled = _shuffle_rows(g.csr, seed=3)
    np.testing.assert_array_equal(gpu_run(ctx, _G(shuffled, False), "WCC"), O.wcc(shuffled))
    n = 20000
    perm = np.random.default_rng(5).permutation(n)
    keep = np.arange(n - 1) % 97 != 0
    csr = csr_from_edges(n, perm[1:][keep], perm[:-1][keep], None, symmetric=True)
    np.testing.assert_array_equal(gpu_run(ctx, _G(csr, False), "WCC"), O.wcc(csr))


@pytest.mark.parametrize("device,nextbits,grid,qbits", [("1", "1", None, "1"), ("1", "1", None, "0"),
                                                        ("1", "0", None, "1"), ("1", "1", "3", "1"),
                                                        ("1", "0", "8192", "1"), ("0", "1", None, "1")])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_bfs_level_driver(ctx, monkeypatch, device, nextbits, grid, qbits, fused):
    """BFS levels planned on the device (GX_BFS_DEVICE=1, batches of levels, done flag read a
    batch late) or by the host: the oracle's levels on power-law graphs (top-down and
    bottom-up levels), a 3 000-level chain (many batches) and an isolated source.  On the device
    path a bottom-up level writes the next level's frontier bitmap (GX_BFS_NEXTBITS=1) or a
    bitmap pass rebuilds it from the levels, and a top-down level after it builds its queue from
    that bitmap (GX_BFS_QBITS=1) or from the levels; GX_BFS_GRID caps the grid-stride kernels'
    grids (3 workgroups: many rounds per wave).  A level runs as two launches branching on the
    plan's direction (GX_BFS_FUSED=1, the default) or as the four direction kernels."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    monkeypatch.setenv("GX_BFS_DEVICE", device)
    monkeypatch.setenv("GX_BFS_FUSED", fused)
    monkeypatch.setenv("GX_BFS_NEXTBITS", nextbits)
    monkeypatch.setenv("GX_BFS_QBITS", qbits)
    if grid:
        monkeypatch.setenv("GX_BFS_GRID", grid)
    for g in (_rmat(14, 16, 4), _rmat(12, 8, 3, undirected=False)):
        s = _src(g)
        np.testing.assert_array_equal(gpu_run(ctx, g, "BFS", source=s), O.bfs(g.csr, s))
    # a directed graph with its transpose (bottom-up levels): two calls on one graph
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    gd = _rmat(12, 8, 3, undirected=False)
    G = A.Graph(ctx, gd.csr, True)
    try:
        s = _src(gd)
        for _ in range(3):
            np.testing.assert_array_equal(A.LA_BFS(G, s), O.bfs(gd.csr, s))
    finally:
        G.close()
    n = 3000
    perm = np.random.default_rng(2).permutation(n)
    csr = csr_from_edges(n + 1, perm[:-1], perm[1:], None, symmetric=True)   # vertex n isolated
    for s in (int(perm[0]), int(perm[n // 2]), n):
        np.testing.assert_array_equal(gpu_run(ctx, _G(csr, False), "BFS", source=s), O.bfs(csr, s))


@pytest.mark.parametrize("alpha,beta", [("1", "1000"), ("1000", "1"), ("24", "48")])
def test_bfs_direction_thresholds(ctx, monkeypatch, alpha, beta):
    """Beamer's switch thresholds (GX_BFS_ALPHA / GX_BFS_BETA): bottom-up from the first level
    and kept to the end, top-down almost throughout, and a mid setting; levels bit-exact."""
    monkeypatch.setenv("GX_BFS_ALPHA", alpha)
    monkeypatch.setenv("GX_BFS_BETA", beta)
    for g in (_rmat(14, 16, 4), _rmat(12, 8, 3, undirected=False)):
        s = _src(g)
        for _ in range(2):   # the second call runs on the hub-first copy / with the transpose
            np.testing.assert_array_equal(gpu_run(ctx, g, "BFS", source=s), O.bfs(g.csr, s))


@pytest.mark.parametrize("env", [{"GX_HUB": "1"}, {"GX_HUB": "2"}, {"GX_HUB": "2", "GX_HUB_SORT": "0"},
                                 {"GX_HUB": "2", "GX_WCC_ROUNDS": "2"}, {"GX_HUB": "2", "GX_REMAP": "scatter"}])
def test_hub_first_copy(ctx, monkeypatch, env):
    """BFS, WCC and SSSP on the hub-first relabelled copy of an undirected graph (built from
    the second call on a graph, GX_HUB=1, or from the first, GX_HUB=2; rows sorted by hub-first
    id, or in the parent's order with GX_HUB_SORT=0; WCC with one sampling round on the sorted
    copy, or two): results come back in the caller's vertex order -- levels and distances
    gathered through the permutation (or scattered through its inverse, GX_REMAP=scatter), WCC labels renamed to each component's smallest caller
    id -- on graphs with many components, isolated vertices and unreachable ones, over three
    calls on one graph."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n = 30000
    perm = np.random.default_rng(11).permutation(n)
    keep = np.arange(n - 1) % 53 != 0
    chains = csr_from_edges(n, perm[1:][keep], perm[:-1][keep], None, symmetric=True)
    for csr in (_rmat(13, 8, 21).csr, _rmat(12, 2, 22).csr, chains):
        G = A.Graph(ctx, csr, False)
        try:
            src = int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))
            ref_bfs, ref_wcc = O.bfs(csr, src), O.wcc(csr)
            for _ in range(3):
                np.testing.assert_array_equal(A.LA_BFS(G, src), ref_bfs)
                np.testing.assert_array_equal(A.LA_BFS(G, 1), O.bfs(csr, 1))
                np.testing.assert_array_equal(A.WeaklyConnectedComponents(G), ref_wcc)
        finally:
            G.close()
    for csr in (_rmat(13, 8, 23, weighted=True).csr, _rmat(12, 2, 24, weighted=True).csr):
        G = A.Graph(ctx, csr, False)
        try:
            src = int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))
            ref = O.sssp(csr, src)
            for _ in range(3):
                np.testing.assert_array_equal(A.LA_SSSP(G, src), ref)
        finally:
            G.close()


@pytest.mark.parametrize("kmax", ["128", "300", "1024", "4096"])
def test_lcc_dense_core(ctx, monkeypatch, kmax):
    """LCC with the dense core counted on the matrix cores (GX_LCC_CORE = the core's largest
    size; the vertices of closure degree above a cut, padded to 128): the core's triangles by
    the masked int8 MFMA product, the others by the hash kernels, which skip core in-neighbours.
    Bit-exact against the oracle on R-MAT graphs (directed ones have reciprocal edges, weight 2)
    and on a 700-clique, where the degree cut falls among equal degrees."""
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges
    monkeypatch.setenv("GX_LCC_CORE", kmax)
    graphs = [_rmat(14, 16, 4), _rmat(13, 8, 3, undirected=False), _rmat(12, 32, 9, undirected=False)]
    rng = np.random.default_rng(11)
    n, k = 6000, 700
    a, b = np.triu_indices(k, 1)
    flip = rng.random(len(a)) < 0.5
    both = rng.random(len(a)) < 0.3   # some clique edges stored both ways (weight 2)
    src = np.concatenate([np.where(flip, a, b), b[both], rng.integers(0, n, 30000)])
    dst = np.concatenate([np.where(flip, b, a), a[both], rng.integers(0, n, 30000)])
    keep = src != dst
    for directed in (False, True):
        graphs.append(_G(csr_from_edges(n, src[keep], dst[keep], None, symmetric=not directed), directed))
    for g in graphs:
        np.testing.assert_array_equal(gpu_run(ctx, g, "LCC"), O.lcc(g.csr, g.directed))


@pytest.mark.parametrize("env", [{}, {"GX_PR_FUSED": "0"}, {"GX_PLAN_TIMES": "1"}, {"GX_UPLOAD_PACK": "0"}])
def test_pagerank_csr_fused(ctx, monkeypatch, env):
    """gx_pagerank_csr (bin/exe/pr's one call): the columns uploaded by a host thread while the
    plan takes each 8 Mi-entry chunk as it lands, from the source side.  Against the oracle at
    1e-12 on undirected graphs of one and of several chunks (scale 19: 16.6 M entries, 2 chunks),
    a weighted one (weights not uploaded), a directed one (unfused path), an edgeless one."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import CSR
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    graphs = [(_rmat(12, 8, 5).csr, False), (_rmat(19, 16, 6).csr, False), (_rmat(13, 8, 7, weighted=True).csr, False),
              (_rmat(12, 8, 8, undirected=False).csr, True),
              (CSR(5, np.zeros(6, dtype=np.uint64), np.zeros(0, dtype=np.uint64), None), False)]
    for csr, directed in graphs:
        got = A.LA_PR_csr(ctx, csr, directed, 0.85, 10)
        np.testing.assert_allclose(got, O.pagerank(csr, directed, 0.85, 10), rtol=PR_RTOL, atol=0)


@pytest.mark.parametrize("pack", ["1", "0"])
def test_upload_packed_columns(ctx, monkeypatch, pack):
    """Columns travel as packed 24-bit values (host_pack24, widened by k_unpack24) when the graph
    has fewer than 2^24 vertices, else (or GX_UPLOAD_PACK=0) as 4 bytes: edge counts around the
    16-entry packing groups and the 4-entry widening groups, columns at the 24-bit limit's
    edges, and a graph of several staging chunks (11 M entries a chunk), through gx_graph_create
    (BFS, SSSP, PR) and gx_pagerank_csr."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import CSR, csr_from_edges
    monkeypatch.setenv("GX_UPLOAD_PACK", pack)
    rng = np.random.default_rng(5)
    for m in (1, 3, 4, 5, 15, 16, 17, 31, 33, 47, 49):
        n = 300
        src = rng.integers(0, n, m)
        dst = rng.integers(0, n, m)
        dst[0] = n - 1
        csr = csr_from_edges(n, src, dst, rng.random(m) + 0.5, symmetric=False)
        g = _G(csr, True)
        s = int(src[0])
        np.testing.assert_array_equal(gpu_run(ctx, g, "BFS", source=s), O.bfs(csr, s))
        np.testing.assert_array_equal(gpu_run(ctx, g, "SSSP", source=s), O.sssp(csr, s))
        np.testing.assert_allclose(gpu_run(ctx, g, "PR", damping=0.85, iters=5), O.pagerank(csr, True, 0.85, 5),
                                   rtol=PR_RTOL, atol=0)
    # columns up to 2^24 - 1: every byte of the packed value in use
    n = (1 << 24) - 1
    rp = np.array([0] + [2] * 2 + [4] * (n - 2), dtype=np.uint64)
    ci = np.array([n - 1, 1 << 16, 0, (1 << 23) + 5], dtype=np.uint64)
    big = CSR(n, rp, ci, None)
    np.testing.assert_array_equal(gpu_run(ctx, _G(big, True), "BFS", source=0), O.bfs(big, 0))
    np.testing.assert_allclose(gpu_run(ctx, _G(big, True), "PR", damping=0.85, iters=3), O.pagerank(big, True, 0.85, 3),
                               rtol=PR_RTOL, atol=0)
    csr = _rmat(21, 16, 9).csr   # ~ 60 M entries: several chunks
    np.testing.assert_allclose(A.LA_PR_csr(ctx, csr, False, 0.85, 5), O.pagerank(csr, False, 0.85, 5,
                                                                                   nthreads=O.max_threads()),
                               rtol=PR_RTOL, atol=0)


def test_pagerank_csr_rejects_bad_columns(ctx):
    """A column >= n fails with GX_INVALID_INDEX (found by the upload thread, reported by the
    call), with one chunk and with the bad entry in the second chunk, and the context stays
    usable."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    for csr in (_rmat(12, 8, 5).csr, _rmat(19, 16, 6).csr):
        bad = type(csr)(csr.n, csr.rowptr.copy(), csr.colidx.copy(), None)
        bad.colidx[-3] = csr.n + 7
        with pytest.raises(N.GxError):
            A.LA_PR_csr(ctx, bad, False, 0.85, 10)
        got = A.LA_PR_csr(ctx, csr, False, 0.85, 10)
        np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, 10), rtol=PR_RTOL, atol=0)
