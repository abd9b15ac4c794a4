"""The C-ABI library loads and exports every symbol include/gx.h declares (no GPU needed),
and the host-only entry points (graph I/O, R-MAT) work on the CPU."""
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, FIXTURES

HEADER = ROOT / "include" / "gx.h"


def declared_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gx_[a-z0-9_]+)\s*\(", text)))


def test_header_lists_the_entry_points():
    syms = declared_symbols()
    for s in ["gx_init", "gx_bfs", "gx_pagerank", "gx_sssp", "gx_wcc", "gx_cdlp", "gx_lcc",
              "gx_read_grb", "gx_pr_part_step"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    L = N.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    bound = {name for name, _, _ in N.SIGNATURES}
    assert bound == set(declared_symbols())


def test_init_without_gpu_fails_loudly():
    from conftest import has_gpu
    if has_gpu():
        pytest.skip("GPU present")
    from ldbc_graphalytics_platforms_graphblas_amd import GxError
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    with pytest.raises(GxError):
        Context(0)


def test_grb_roundtrip(tmp_path, fixture_graphs):
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    for name in ["example-directed", "example-undirected", "test-pr-directed"]:
        g = fixture_graphs(name)
        p = tmp_path / f"{name}.grb"
        graphio.write_grb(p, g.csr)
        back = graphio.read_grb(p)
        assert back.n == g.csr.n
        np.testing.assert_array_equal(back.rowptr, g.csr.rowptr)
        np.testing.assert_array_equal(back.colidx, g.csr.colidx)
        if g.csr.vals is None:
            assert back.vals is None
        else:
            np.testing.assert_array_equal(back.vals, g.csr.vals)
        # header: 512 bytes of ASCII, then fmt=0 (BY_ROW), kind 2 / 102 (sparse [+iso])
        raw = p.read_bytes()
        assert raw.startswith(b"SuiteSparse:GraphBLAS matrix")
        fmt, kind = np.frombuffer(raw[512:520], dtype=np.int32)
        assert fmt == 0 and kind == (2 if g.weighted else 102)


def test_vtb_roundtrip(tmp_path):
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    ids = np.array([5, 1, 99, 2**40], dtype=np.uint64)
    graphio.write_vtb(tmp_path / "g.vtb", ids)
    np.testing.assert_array_equal(graphio.read_vtb(tmp_path / "g.vtb"), ids)
    assert (tmp_path / "g.vtb").stat().st_size == 32


def test_mtx_reader_matches_relabel(tmp_path, fixture_graphs):
    """relabel.py-style .vtx/.mtx parsed by gx_read_mtx equals the Python relabel CSR."""
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    for name in ["example-directed", "example-undirected", "test-cdlp-undirected"]:
        g = fixture_graphs(name)
        mapping, src, dst, w = graphio.relabel(FIXTURES / f"{name}.v", FIXTURES / f"{name}.e",
                                               g.directed, g.weighted)
        graphio.write_vtx_mtx(tmp_path / name, mapping, src, dst, w, g.directed)
        csr = graphio.read_mtx(tmp_path / name / "graph.mtx")
        np.testing.assert_array_equal(csr.rowptr, g.csr.rowptr)
        np.testing.assert_array_equal(csr.colidx, g.csr.colidx)
        np.testing.assert_array_equal(graphio.read_vtx(tmp_path / name / "graph.vtx"), mapping)


def test_hypersparse_and_csc_grb(tmp_path):
    """binread accepts hypersparse and by-column matrices (graphio.h:150-250)."""
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    # 4x4, entries (0,1) (0,3) (2,1): CSC hypersparse with columns {1, 3}
    header = b"x" * 512
    fields = (np.array([1, 101], np.int32).tobytes() + np.array([0.0625]).tobytes() +
              np.array([4, 4], np.uint64).tobytes() + np.array([-1], np.int64).tobytes() +
              np.array([2, 3], np.uint64).tobytes() + np.array([0], np.int32).tobytes() +
              np.array([1], np.uint64).tobytes())
    Ap = np.array([0, 2, 3], np.uint64).tobytes()
    Ah = np.array([1, 3], np.uint64).tobytes()
    Ai = np.array([0, 2, 0], np.uint64).tobytes()
    (tmp_path / "h.grb").write_bytes(header + fields + Ap + Ah + Ai + b"\x01")
    csr = graphio.read_grb(tmp_path / "h.grb")
    np.testing.assert_array_equal(csr.rowptr, [0, 2, 2, 3, 3])
    np.testing.assert_array_equal(csr.colidx, [1, 3, 1])
    assert csr.vals is None


def test_rmat_deterministic():
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    a = rmat(10, 8, 7)
    b = rmat(10, 8, 7)
    np.testing.assert_array_equal(a.rowptr, b.rowptr)
    np.testing.assert_array_equal(a.colidx, b.colidx)
    # undirected: symmetric, no self loops, sorted unique rows
    rows = np.repeat(np.arange(a.n), np.diff(a.rowptr.astype(np.int64)))
    pairs = set(zip(rows.tolist(), a.colidx.tolist()))
    assert all((c, r) in pairs for r, c in pairs)
    assert all(r != c for r, c in pairs)
    for i in range(a.n):
        row = a.colidx[a.rowptr[i]:a.rowptr[i + 1]]
        assert (np.diff(row.astype(np.int64)) > 0).all()
    w = rmat(9, 4, 3, weighted=True)
    assert w.vals is not None and (w.vals > 0).all() and (w.vals <= 1).all()


def _grb_fields(fmt, kind, n, nvec, nvals, typecode, typesize):
    return (b"x" * 512 + np.array([fmt, kind], np.int32).tobytes() + np.array([0.0625]).tobytes() +
            np.array([n, n], np.uint64).tobytes() + np.array([-1], np.int64).tobytes() +
            np.array([nvec, nvals], np.uint64).tobytes() + np.array([typecode], np.int32).tobytes() +
            np.array([typesize], np.uint64).tobytes())


def test_iso_fp64_grb_is_weighted(tmp_path):
    """An iso FP64 matrix (SuiteSparse stores one when every weight is equal) keeps its
    weight on every entry, so SSSP runs on it as the reference's does (graphio.h:191-216)."""
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    # 3x3 CSR sparse iso FP64 (kind 102), entries (0,1) (1,2) (2,0), all weight 2.5
    raw = (_grb_fields(0, 102, 3, 3, 3, 10, 8) + np.array([0, 1, 2, 3], np.uint64).tobytes() +
           np.array([1, 2, 0], np.uint64).tobytes() + np.array([2.5]).tobytes())
    (tmp_path / "iso.grb").write_bytes(raw)
    csr = graphio.read_grb(tmp_path / "iso.grb")
    np.testing.assert_array_equal(csr.rowptr, [0, 1, 2, 3])
    np.testing.assert_array_equal(csr.colidx, [1, 2, 0])
    np.testing.assert_array_equal(csr.vals, [2.5, 2.5, 2.5])
    # iso BOOL stays unweighted
    raw = (_grb_fields(0, 102, 3, 3, 3, 0, 1) + np.array([0, 1, 2, 3], np.uint64).tobytes() +
           np.array([1, 2, 0], np.uint64).tobytes() + b"\x01")
    (tmp_path / "b.grb").write_bytes(raw)
    assert graphio.read_grb(tmp_path / "b.grb").vals is None


@pytest.mark.parametrize("fmt", [0, 1])
def test_bitmap_and_full_grb(tmp_path, fmt):
    """Bitmap (kind 4) and full (kind 8) matrices, by row and by column (graphio.h:175-186,
    211-216, 250-277): Ab presence bytes then Ax, or Ax alone."""
    from ldbc_graphalytics_platforms_graphblas_amd import graphio
    dense = np.array([[0, 1.5, 0], [2.0, 0, 3.0], [0, 0, 4.0]])
    present = dense != 0
    cells = dense if fmt == 0 else dense.T   # major order: rows for BY_ROW, columns for BY_COL
    pres = present if fmt == 0 else present.T
    raw = (_grb_fields(fmt, 4, 3, 3, int(present.sum()), 10, 8) + pres.astype(np.int8).tobytes() +
           cells.astype(np.float64).tobytes())
    (tmp_path / "bm.grb").write_bytes(raw)
    csr = graphio.read_grb(tmp_path / "bm.grb")
    np.testing.assert_array_equal(csr.rowptr, [0, 1, 3, 4])
    np.testing.assert_array_equal(csr.colidx, [1, 0, 2, 2])
    np.testing.assert_array_equal(csr.vals, [1.5, 2.0, 3.0, 4.0])
    # full iso BOOL: every cell an edge (self-loops included), unweighted
    raw = _grb_fields(fmt, 108, 3, 3, 9, 0, 1) + b"\x01"
    (tmp_path / "full.grb").write_bytes(raw)
    csr = graphio.read_grb(tmp_path / "full.grb")
    np.testing.assert_array_equal(csr.rowptr, [0, 3, 6, 9])
    np.testing.assert_array_equal(csr.colidx, [0, 1, 2] * 3)
    assert csr.vals is None
