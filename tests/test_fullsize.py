"""Full-size parity on config 4's graph (SYN-8_5: the seeded R-MAT stand-in for
datagen-8_5-fb, scale 23, edgefactor 40, 8.4 M vertices, 628 M stored entries).

One bounded case per path on the MI355X, against the oracle's multithreaded restatements
(oracle/gx_oracle.c; their equality with the serial ones is tests/test_oracle_parallel.py):
- PageRank (gx_pagerank, 10 iterations): rtol 1e-12 of the fp64 oracle;
- SSSP (gx_sssp and the 1-D split's single-rank loop gx_sssp_split_run): bit-exact.
The graph is generated once (~16 s), the oracle runs on the box's host cores.
"""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)
from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

PR_RTOL = 1e-12


@pytest.fixture(scope="module")
def syn85():
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context, Graph
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    csr = rmat(23, 40, 85, undirected=True, weighted=True)
    ctx = Context(0)
    G = Graph(ctx, csr, False)
    yield csr, G
    G.close()
    ctx.close()


def test_pagerank_syn85(syn85):
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syn85
    got = A.LA_PR(G, 0.85, 10)
    ref = O.pagerank(csr, False, 0.85, 10, nthreads=O.max_threads())
    np.testing.assert_allclose(got, ref, rtol=PR_RTOL, atol=0)


def test_sssp_syn85(syn85):
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    csr, G = syn85
    src = int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))
    ref = O.sssp_par(csr, src, 0.0, nthreads=O.max_threads())
    assert np.array_equal(A.LA_SSSP(G, src), ref)
    sp = A.SsspSplit(G)
    try:
        assert np.array_equal(sp.run(src), ref)
    finally:
        sp.close()
