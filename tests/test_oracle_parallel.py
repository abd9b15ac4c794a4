"""The multithreaded CPU baselines (bench.py's cpu_baseline leg) return bitwise the results of
the serial oracle functions they stand beside (oracle/gx_oracle.c *_par)."""
import numpy as np
import pytest

from oracle import oracle as O
from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat


@pytest.mark.parametrize("undirected", [True, False])
@pytest.mark.parametrize("threads", [1, 4, 8])
def test_parallel_baselines_match_serial(undirected, threads):
    csr = rmat(12, 8, 21, undirected=undirected, weighted=True)
    deg = np.diff(csr.rowptr.astype(np.int64))
    for src in [int(np.argmax(deg)), 0, csr.n - 1]:
        np.testing.assert_array_equal(O.bfs_par(csr, src, undirected, nthreads=threads), O.bfs(csr, src))
        for delta in [0.0, 0.01, 1.0, 100.0]:
            np.testing.assert_array_equal(O.sssp_par(csr, src, delta, nthreads=threads), O.sssp(csr, src))
    np.testing.assert_array_equal(O.wcc_par(csr, nthreads=threads), O.wcc(csr))


def test_parallel_baselines_on_fixtures(fixture_graphs):
    for name in ["example-directed", "example-undirected", "test-bfs-directed", "test-bfs-undirected",
                 "test-sssp-directed", "test-sssp-undirected", "test-wcc-directed", "test-wcc-undirected"]:
        g = fixture_graphs(name)
        for src in range(g.csr.n):
            np.testing.assert_array_equal(O.bfs_par(g.csr, src, not g.directed, nthreads=4), O.bfs(g.csr, src))
            if g.csr.vals is not None:
                np.testing.assert_array_equal(O.sssp_par(g.csr, src, 0.0, nthreads=4), O.sssp(g.csr, src))
        np.testing.assert_array_equal(O.wcc_par(g.csr, nthreads=4), O.wcc(g.csr))
