"""SSSP on the 1-D split (gx_sssp_split.hip, config 4's partition) against the oracle.

GPU: one rank owning every vertex (gx_sssp_split_run, rounds on the device) and 2-5 ranks
simulated on one device through the lock-step driver (distributed.sssp with LocalComm: the
pairs all-gather is a concatenation) -- bit-exact distances, whatever the bucket width.
The gloo world-2 run of the same driver is in test_distributed_algs.py.
"""
import numpy as np
import pytest
import torch

from conftest import ROOT  # noqa: F401  (sys.path)
from ldbc_graphalytics_platforms_graphblas_amd import distributed as D
from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges, rmat
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    c = Context(0)
    yield c
    c.close()


def _src(csr):
    return int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))


GRAPHS = [(10, 8, 1, True), (13, 16, 2, True), (12, 8, 3, False), (14, 6, 4, False)]


ENVS = [{}, {"GX_SSSP_DSCALE": "0.25"}, {"GX_SSSP_DSCALE": "40"}, {"GX_SSSP_PULL": "2"}, {"GX_SSSP_PULL": "0"},
        {"GX_SSSP_FUSE": "1"}, {"GX_SSSP_FUSE": "1", "GX_SSSP_DSCALE": "0.05"}]


@pytest.mark.parametrize("scale,ef,seed,und", GRAPHS)
@pytest.mark.parametrize("env", ENVS)
def test_split_run_one_rank(ctx, monkeypatch, scale, ef, seed, und, env):
    """Every schedule: bucket widths (0.05 x the default puts most vertices past the 32-bucket
    ring window, through the overflow), pulled / pushed heavy phases, no bucket fusion."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    csr = rmat(scale, ef, seed, undirected=und, weighted=True)
    G = A.Graph(ctx, csr, not und)
    sp = A.SsspSplit(G)
    try:
        for src in (_src(csr), 0):
            assert np.array_equal(sp.run(src), O.sssp(csr, src))
    finally:
        sp.close()
        G.close()


def test_split_run_unreachable_and_isolated(ctx):
    """Two components, isolated vertices and a source without edges."""
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    rng = np.random.default_rng(5)
    n = 3000
    a, b = rng.integers(0, 1000, 6000), rng.integers(0, 1000, 6000)
    c, d = rng.integers(1500, 2500, 4000), rng.integers(1500, 2500, 4000)
    src = np.concatenate([a, c])
    dst = np.concatenate([b, d])
    keep = src != dst
    w = rng.random(int(keep.sum())) * 3.0
    csr = csr_from_edges(n, src[keep], dst[keep], w, symmetric=True)
    G = A.Graph(ctx, csr, False)
    sp = A.SsspSplit(G)
    try:
        for s in (int(src[0]), 1200, int(c[0])):
            assert np.array_equal(sp.run(s), O.sssp(csr, s))
    finally:
        sp.close()
        G.close()


@pytest.mark.parametrize("nranks,env", [(2, {}), (4, {}), (5, {}), (3, {"GX_SSSP_PULL": "2"}),
                                        (3, {"GX_SSSP_FUSE": "1", "GX_SSSP_DSCALE": "0.05"})])
def test_split_simulated_ranks(ctx, monkeypatch, nranks, env):
    """The per-round protocol with 2, 4 and 5 ranks on one device (rank ranges balanced by
    entries), also with an always-pulled heavy phase and through the overflow."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Graph
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    dev = torch.device("cuda", 0)
    for csr, directed in [(rmat(13, 8, 31, undirected=True, weighted=True), False),
                          (rmat(12, 6, 32, undirected=False, weighted=True), True)]:
        g = Graph(ctx, csr, directed)
        try:
            be = D.GpuBackend(g)
            rng = D.vertex_ranges(csr.rowptr, nranks)
            ranks = [D.LocalRank(be, int(rng[k]), int(rng[k + 1]), dev, k) for k in range(nranks)]
            src = _src(csr)
            got = D.sssp(ranks, D.LocalComm(), csr.n, src).cpu().numpy()
            assert np.array_equal(got, O.sssp(csr, src))
        finally:
            g.close()


def test_split_empty_rank(ctx):
    """A rank owning no vertex still takes part in every round."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Graph
    dev = torch.device("cuda", 0)
    csr = rmat(11, 8, 33, undirected=True, weighted=True)
    g = Graph(ctx, csr, False)
    try:
        be = D.GpuBackend(g)
        n = csr.n
        bounds = [0, n // 3, n // 3, n]
        ranks = [D.LocalRank(be, bounds[k], bounds[k + 1], dev, k) for k in range(3)]
        src = _src(csr)
        assert np.array_equal(D.sssp(ranks, D.LocalComm(), n, src).cpu().numpy(), O.sssp(csr, src))
    finally:
        g.close()
