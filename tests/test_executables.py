"""The Graphalytics executables (bin/exe/*) behind their unchanged process contract.

The load path (load-graph.sh:50-67) is relabel.py -> converter; the run path
(execute-job.sh:68-151) invokes bin/exe/<alg> with the argument vector rebuilt below
(execute-job.sh:70-139).  Outputs are checked with the Graphalytics validation rules against
the 24 reference validation files; stdout must carry the two processing-time markers the
Java collector parses (GraphblasCollector.java:54-95).
"""
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import FIXTURES, ROOT, VALIDATION, check_against_validation, read_validation, split_validation

EXE = ROOT / "bin" / "exe"
RELABEL = ROOT / "bin" / "py" / "relabel.py"


def load_dir(tmp_path_factory, graph, fixture_graphs):
    """load-graph.sh: relabel.py then converter, into a per-graph directory."""
    g = fixture_graphs(graph)
    d = tmp_path_factory.mktemp(graph)
    subprocess.check_call([sys.executable, str(RELABEL), "--graph-name", graph,
                           "--input-vertex-path", str(FIXTURES / f"{graph}.v"),
                           "--input-edge-path", str(FIXTURES / f"{graph}.e"),
                           "--output-path", str(d), "--weighted", str(g.weighted).lower(),
                           "--directed", str(g.directed).lower()], stdout=subprocess.DEVNULL)
    subprocess.check_call([str(EXE / "converter"), "--data-dir", str(d)], stdout=subprocess.DEVNULL)
    return d, g


def job_argv(alg, d, out, g, log):
    """The COMMAND execute-job.sh builds for each algorithm (execute-job.sh:70-139)."""
    directed = str(g.directed).lower()
    common = ["--binary", "true", "--jobid", "job-1", "--input-dir", str(d), "--output-file", str(out),
              "--directed", directed]
    tail = ["--log-path", str(log), "--threadnum", "4"]
    if alg in ("bfs", "sssp"):
        return [str(EXE / alg)] + common + ["--source-vertex", g.param(alg, "source-vertex")] + tail
    if alg == "pr":
        return [str(EXE / alg)] + common + ["--damping-factor", str(float(g.param("pr", "damping-factor"))),
                                            "--max-iteration", g.param("pr", "num-iterations")] + tail
    if alg == "cdlp":
        return [str(EXE / alg)] + common + ["--max-iteration", g.param("cdlp", "max-iterations")] + tail
    return [str(EXE / alg)] + common + tail


def test_converter_roundtrip(tmp_path_factory, fixture_graphs):
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    for graph in ["example-directed", "example-undirected", "test-sssp-undirected"]:
        d, g = load_dir(tmp_path_factory, graph, fixture_graphs)
        back = graphio.read_grb(d / "graph.grb")
        np.testing.assert_array_equal(back.rowptr, g.csr.rowptr)
        np.testing.assert_array_equal(back.colidx, g.csr.colidx)
        np.testing.assert_array_equal(graphio.read_vtb(d / "graph.vtb"), g.mapping)
        if g.weighted:
            np.testing.assert_array_equal(back.vals, g.csr.vals)


def test_relabel_standalone_load_graph_flags(tmp_path, fixture_graphs):
    """relabel.py copied alone into a reference-like checkout, run with
    the abbreviated flags load-graph.sh:51-58 passes (--input-vertex / --input-edge), gives
    the same files as the package's restatement, for every fixture graph."""
    import shutil
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    ref_py = tmp_path / "ref" / "bin" / "py"
    ref_py.mkdir(parents=True)
    shutil.copy(RELABEL, ref_py / "relabel.py")
    graphs = sorted({p.stem for p in FIXTURES.glob("*.properties")})
    assert len(graphs) == 14
    for graph in graphs:
        g = fixture_graphs(graph)
        out, want = tmp_path / "out" / graph, tmp_path / "want" / graph
        subprocess.check_call([sys.executable, str(ref_py / "relabel.py"), "--graph-name", graph,
                               "--input-vertex", str(FIXTURES / f"{graph}.v"),
                               "--input-edge", str(FIXTURES / f"{graph}.e"),
                               "--output-path", str(out), "--weighted", str(g.weighted).lower(),
                               "--directed", str(g.directed).lower()],
                              stdout=subprocess.DEVNULL, cwd=tmp_path, env={"PATH": "/usr/bin:/bin"})
        m, s, d_, w = graphio.relabel(FIXTURES / f"{graph}.v", FIXTURES / f"{graph}.e", g.directed, g.weighted)
        graphio.write_vtx_mtx(want, m, s, d_, w, g.directed)
        for f in ("graph.vtx", "graph.mtx"):
            assert (out / f).read_text() == (want / f).read_text(), f"{graph}/{f}"


def parse_output(path, alg):
    ids, vals = [], []
    for line in path.read_text().splitlines():
        a, b = line.split()
        ids.append(int(a))
        vals.append(b)
    return np.array(ids, dtype=np.uint64), vals


@pytest.mark.gpu
@pytest.mark.parametrize("name", VALIDATION)
def test_executable_matches_validation(name, tmp_path_factory, fixture_graphs):
    graph, ALG = split_validation(name)
    alg = ALG.lower()
    d, g = load_dir(tmp_path_factory, graph, fixture_graphs)
    out = d / f"out-{alg}"
    res = subprocess.run(job_argv(alg, d, out, g, d), capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    starts = re.findall(r"Processing starts at: (\d+)", res.stdout)
    ends = re.findall(r"Processing ends at: (\d+)", res.stdout)
    assert len(starts) == 1 and len(ends) == 1 and int(ends[0]) >= int(starts[0])
    # ComputationTimer's lines (computation_timer.hpp:17-50), inside the markers
    tname = {"BFS": "BFS", "PR": "PageRank", "SSSP": "SSSP", "WCC": "WeaklyConnectedComponents", "CDLP": "CDLP",
             "LCC": "LCC"}[ALG]
    assert re.search(rf"^{tname} starts$", res.stdout, re.M), res.stdout
    assert re.search(rf"^{tname} duration: \d+(\.\d+)?s$", res.stdout, re.M), res.stdout
    ids, vals = parse_output(out, alg)
    np.testing.assert_array_equal(ids, g.mapping)
    expected = read_validation(FIXTURES / name)
    if ALG in ("WCC", "CDLP"):
        # labels are printed as original ids: map back to internal indices for the checker
        index = {int(m): i for i, m in enumerate(g.mapping)}
        labels = np.array([index[int(v)] for v in vals], dtype=np.uint64)
        check_against_validation(ALG, g.mapping, labels, expected)
        assert [int(v) for v in vals] == [int(expected[int(m)]) for m in g.mapping]   # bit-exact
    elif ALG == "BFS":
        check_against_validation(ALG, g.mapping, [int(v) for v in vals], expected)
    else:
        got = [np.inf if v == "infinity" else float(v) for v in vals]
        check_against_validation(ALG, g.mapping, got, expected)
        for v in vals:   # %.16e formatting (pr.cpp:26-27) or the literal `infinity` (sssp.cpp:45)
            assert v == "infinity" or re.fullmatch(r"-?\d\.\d{16}e[+-]\d\d", v), v


@pytest.mark.gpu
def test_source_vertex_not_found(tmp_path_factory, fixture_graphs):
    d, g = load_dir(tmp_path_factory, "example-directed", fixture_graphs)
    argv = job_argv("bfs", d, d / "o", g, d)
    argv[argv.index("--source-vertex") + 1] = "987654"
    res = subprocess.run(argv, capture_output=True, text=True, timeout=60)
    assert res.returncode != 0 and "Source vertex not found in mapping" in res.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["example-directed", "example-undirected", "test-pr-directed", "test-pr-undirected"])
def test_pagerank_executable_gx_ngpus(graph, tmp_path_factory, fixture_graphs):
    """bin/exe/pr with GX_NGPUS=1: the single-process multi-GPU path (gx_pagerank_multi: 1-D
    row blocks, an in-process RCCL clique, grouped all-gathers), equal to the oracle at 1e-12
    and to the Graphalytics validation file."""
    import os
    from oracle import oracle as O
    d, g = load_dir(tmp_path_factory, graph, fixture_graphs)
    out = d / "out-pr-multi"
    env = dict(os.environ, GX_NGPUS="1")
    res = subprocess.run(job_argv("pr", d, out, g, d), capture_output=True, text=True, timeout=120, env=env)
    assert res.returncode == 0, res.stderr
    assert len(re.findall(r"Processing (starts|ends) at: \d+", res.stdout)) == 2
    ids, vals = parse_output(out, "pr")
    np.testing.assert_array_equal(ids, g.mapping)
    got = np.array([float(v) for v in vals])
    want = O.pagerank(g.csr, g.directed, float(g.param("pr", "damping-factor")), int(g.param("pr", "num-iterations")))
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)
    check_against_validation("PR", g.mapping, list(got), read_validation(FIXTURES / f"{graph}-PR"))


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["example-directed", "example-undirected", "test-sssp-directed",
                                   "test-sssp-undirected"])
def test_sssp_executable_gx_ngpus(graph, tmp_path_factory, fixture_graphs):
    """bin/exe/sssp with GX_NGPUS=1 (gx_sssp_multi: the 1-D split with in-process RCCL
    all-gathers of counts and pairs, BASELINE config 4's SSSP half): bit-exact against the
    oracle and within the Graphalytics rule of the validation file."""
    import os
    from oracle import oracle as O
    d, g = load_dir(tmp_path_factory, graph, fixture_graphs)
    out = d / "out-sssp-multi"
    env = dict(os.environ, GX_NGPUS="1")
    res = subprocess.run(job_argv("sssp", d, out, g, d), capture_output=True, text=True, timeout=120, env=env)
    assert res.returncode == 0, res.stderr
    assert "GX_NGPUS" not in res.stderr
    assert re.search(r"^SSSP duration: \d+(\.\d+)?s$", res.stdout, re.M), res.stdout
    ids, vals = parse_output(out, "sssp")
    np.testing.assert_array_equal(ids, g.mapping)
    got = np.array([np.inf if v == "infinity" else float(v) for v in vals])
    src = int(np.flatnonzero(g.mapping == np.uint64(g.param("sssp", "source-vertex")))[0])
    assert np.array_equal(got, O.sssp(g.csr, src))
    check_against_validation("SSSP", g.mapping, list(got), read_validation(FIXTURES / f"{graph}-SSSP"))


@pytest.mark.gpu
@pytest.mark.parametrize("alg,graph", [("pr", "example-directed"), ("pr", "test-pr-undirected"),
                                       ("sssp", "example-undirected"), ("sssp", "test-sssp-directed"),
                                       ("lcc", "example-directed"), ("lcc", "test-lcc-undirected"),
                                       ("lcc", "example-undirected"), ("bfs", "example-directed"),
                                       ("bfs", "test-bfs-undirected"), ("wcc", "example-undirected"),
                                       ("wcc", "test-wcc-directed"), ("cdlp", "example-directed"),
                                       ("cdlp", "test-cdlp-undirected")])
@pytest.mark.parametrize("ngpus", [1, 2, 3])
def test_executable_gx_ngpus_virtual(alg, graph, ngpus, tmp_path_factory, fixture_graphs):
    """bin/exe/* with GX_NGPUS=N: N = 1 is a size-1 in-process RCCL clique (PageRank: the
    single-GPU call), N > 1 runs N virtual devices on this box's one GPU (GX_MULTI_SIM=1), the
    same partition and kernels an N-GPU node runs, with the collectives as device copies.
    Against the oracle (PR rtol 1e-12, the others bit-exact) and the Graphalytics rule of the
    validation file."""
    import os
    from oracle import oracle as O
    d, g = load_dir(tmp_path_factory, graph, fixture_graphs)
    out = d / f"out-{alg}-n{ngpus}"
    env = dict(os.environ, GX_NGPUS=str(ngpus), GX_MULTI_SIM="1")
    res = subprocess.run(job_argv(alg, d, out, g, d), capture_output=True, text=True, timeout=120, env=env)
    assert res.returncode == 0, res.stderr
    assert "GX_NGPUS" not in res.stderr
    assert len(re.findall(r"Processing (starts|ends) at: \d+", res.stdout)) == 2
    ids, vals = parse_output(out, alg)
    np.testing.assert_array_equal(ids, g.mapping)
    if alg in ("bfs", "wcc", "cdlp"):
        expected = read_validation(FIXTURES / f"{graph}-{alg.upper()}")
        if alg == "bfs":
            check_against_validation("BFS", g.mapping, [int(v) for v in vals], expected)
        else:
            index = {int(m): i for i, m in enumerate(g.mapping)}
            labels = np.array([index[int(v)] for v in vals], dtype=np.uint64)
            check_against_validation(alg.upper(), g.mapping, labels, expected)
        assert [int(v) for v in vals] == [int(expected[int(m)]) for m in g.mapping]   # bit-exact
        return
    got = np.array([np.inf if v == "infinity" else float(v) for v in vals])
    if alg == "pr":
        want = O.pagerank(g.csr, g.directed, float(g.param("pr", "damping-factor")),
                          int(g.param("pr", "num-iterations")))
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)
    elif alg == "sssp":
        src = int(np.flatnonzero(g.mapping == np.uint64(g.param("sssp", "source-vertex")))[0])
        assert np.array_equal(got, O.sssp(g.csr, src))
    else:
        assert np.array_equal(got, O.lcc(g.csr, g.directed))
    check_against_validation(alg.upper(), g.mapping, list(got), read_validation(FIXTURES / f"{graph}-{alg.upper()}"))


REF_EXECUTE_JOB = __import__("pathlib").Path("/root/reference/bin/sh/execute-job.sh")


@pytest.mark.skipif(not REF_EXECUTE_JOB.exists(), reason="the reference checkout is not on this machine")
@pytest.mark.parametrize("alg", ["bfs", "wcc", "pr", "cdlp", "lcc", "sssp"])
def test_job_argv_matches_reference_execute_job(alg, tmp_path):
    """job_argv() restates the COMMAND that execute-job.sh:68-139 builds; this pins it to the
    script itself, run in place (not copied): a symlink to it under a temporary root makes its
    rootdir (execute-job.sh:5) resolve there, where a stub bin/exe/<alg> records its argv.  The
    script's quirks are covered: --num-threads becomes --threadnum, --job-id --jobid, and the
    sssp lines without a trailing backslash (execute-job.sh:130, 135) still split into words."""
    import os
    (tmp_path / "bin" / "sh").mkdir(parents=True)
    (tmp_path / "bin" / "exe").mkdir(parents=True)
    os.symlink(REF_EXECUTE_JOB, tmp_path / "bin" / "sh" / "execute-job.sh")
    log = tmp_path / "log"
    log.mkdir()
    stub = tmp_path / "bin" / "exe" / alg
    stub.write_text('#!/bin/bash\nprintf "%s\\n" "$@" > "$(dirname "$0")/argv.txt"\n')
    stub.chmod(0o755)
    d, out = tmp_path / "graph", tmp_path / "out"

    class G:   # the job's parameters, as Graphalytics passes them
        directed = True

        @staticmethod
        def param(a, key):
            return {"source-vertex": "6", "damping-factor": "0.85", "num-iterations": "10",
                    "max-iterations": "10"}[key]

    res = subprocess.run(["bash", str(tmp_path / "bin" / "sh" / "execute-job.sh"), "--job-id", "job-1",
                          "--log-path", str(log), "--algorithm", alg, "--source-vertex", "6",
                          "--max-iteration", "10", "--damping-factor", "0.85", "--input-dir", str(d),
                          "--output-file", str(out), "--num-threads", "4", "--directed", "true"],
                         capture_output=True, text=True, timeout=60)
    assert res.returncode == 0, res.stderr
    got = (tmp_path / "bin" / "exe" / "argv.txt").read_text().split("\n")[:-1]
    want = job_argv(alg, d, out, G, log)
    assert got == want[1:], (got, want)
