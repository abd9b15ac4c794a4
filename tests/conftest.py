import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

FIXTURES = ROOT / "tests" / "golden" / "graphalytics"
GOLDEN = ROOT / "tests" / "golden"

# the 24 Graphalytics validation outputs shipped with the reference
# (example-data-sets/graphs/<graph>-<ALG>), SURVEY.md Appendix B
VALIDATION = sorted(p.name for p in FIXTURES.iterdir()
                    if "-" in p.name and p.name.rsplit("-", 1)[1] in {"BFS", "PR", "SSSP", "WCC", "CDLP", "LCC"})


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: larger synthetic inputs")


def split_validation(name: str):
    graph, alg = name.rsplit("-", 1)
    return graph, alg


def read_validation(path):
    """<original id> <value> per line -> dict id -> str value."""
    out = {}
    for line in Path(path).read_text().splitlines():
        parts = line.split()
        if len(parts) >= 2:
            out[int(parts[0])] = parts[1]
    return out


def alg_params(g, alg: str):
    p = {}
    if alg == "BFS":
        p["source"] = int(g.param("bfs", "source-vertex"))
    elif alg == "SSSP":
        p["source"] = int(g.param("sssp", "source-vertex"))
    elif alg == "CDLP":
        p["iters"] = int(g.param("cdlp", "max-iterations"))
    elif alg == "PR":
        p["damping"] = float(g.param("pr", "damping-factor"))
        p["iters"] = int(g.param("pr", "num-iterations"))
    return p


def internal_index(mapping, orig_id: int) -> int:
    hits = np.nonzero(mapping == np.uint64(orig_id))[0]
    assert len(hits) == 1
    return int(hits[0])


def check_against_validation(alg: str, mapping, values, expected: dict):
    """Graphalytics validation rules: exact (BFS, CDLP), equivalence (WCC),
    relative epsilon 1e-4 (PR, SSSP, LCC); infinity must match infinity."""
    assert len(expected) == len(mapping)
    if alg == "WCC":
        # equivalence: same partition; and, bit-exact, min original id per component
        ours = {int(m): int(mapping[int(v)]) for m, v in zip(mapping, values)}
        assert ours == {k: int(v) for k, v in expected.items()}
        return
    for m, v in zip(mapping, values):
        e = expected[int(m)]
        if alg in ("BFS",):
            assert int(v) == int(e), (m, v, e)
        elif alg == "CDLP":
            assert int(mapping[int(v)]) == int(e), (m, v, e)
        else:
            if e == "infinity":
                assert np.isinf(v), (m, v)
            else:
                ev = float(e)
                assert abs(float(v) - ev) <= 1e-4 * max(abs(ev), 1e-300) or (ev == 0.0 and v == 0.0), (m, v, e)


@pytest.fixture(scope="session")
def fixture_graphs():
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import load_graphalytics
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_graphalytics(FIXTURES, name)
        return cache[name]

    return get


def has_gpu() -> bool:
    try:
        from ldbc_graphalytics_platforms_graphblas_amd import device_count
        return device_count() > 0
    except Exception:
        return False
