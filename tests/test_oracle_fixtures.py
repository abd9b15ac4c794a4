"""Pin the CPU oracle (oracle/gx_oracle.c) to the reference's own golden vectors: the 24
Graphalytics validation outputs in example-data-sets/graphs."""
import pytest

from conftest import VALIDATION, FIXTURES, alg_params, check_against_validation, internal_index, \
    read_validation, split_validation
from oracle import oracle as O


def run_oracle(g, alg):
    p = alg_params(g, alg)
    if alg == "BFS":
        return O.bfs(g.csr, internal_index(g.mapping, p["source"]))
    if alg == "SSSP":
        return O.sssp(g.csr, internal_index(g.mapping, p["source"]))
    if alg == "PR":
        return O.pagerank(g.csr, g.directed, p["damping"], p["iters"])
    if alg == "WCC":
        return O.wcc(g.csr)
    if alg == "CDLP":
        return O.cdlp(g.csr, g.directed, p["iters"])
    if alg == "LCC":
        return O.lcc(g.csr, g.directed)
    raise AssertionError(alg)


def test_inventory():
    assert len(VALIDATION) == 24


@pytest.mark.parametrize("name", VALIDATION)
def test_oracle_matches_validation(name, fixture_graphs):
    graph, alg = split_validation(name)
    g = fixture_graphs(graph)
    expected = read_validation(FIXTURES / name)
    check_against_validation(alg, g.mapping, run_oracle(g, alg), expected)


def test_pagerank_thread_count_invariant(fixture_graphs):
    g = fixture_graphs("test-pr-directed")
    a = O.pagerank(g.csr, True, 0.85, 14, nthreads=1)
    b = O.pagerank(g.csr, True, 0.85, 14, nthreads=4)
    assert (a == b).all()
