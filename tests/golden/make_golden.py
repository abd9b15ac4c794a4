#!/usr/bin/env python3
"""Generate tests/golden/synthetic_*.npz: small seeded graphs + expected outputs computed by
independent libraries (NOT by our oracle), used to cross-check the oracle and the HIP path.

  BFS   scipy.sparse.csgraph.shortest_path(unweighted=True)     (hop levels, inf -> INT64_MAX)
  SSSP  scipy.sparse.csgraph.dijkstra                           (fp64 path sums)
  WCC   scipy.sparse.csgraph.connected_components('weak')       (relabelled to min vertex id)
  LCC   networkx.clustering on the undirected graph             (undirected graphs only)

PR and CDLP have no independent implementation with the Graphalytics semantics here; they are
pinned by the reference's own validation files (tests/golden/graphalytics).
Run from the repo root:  python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import networkx as nx
import numpy as np
import scipy.sparse as sp
from scipy.sparse import csgraph

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from ldbc_graphalytics_platforms_graphblas_amd.graphio import csr_from_edges  # noqa: E402

OUT = Path(__file__).resolve().parent
INT64_MAX = np.iinfo(np.int64).max


def rmat_edges(scale, ef, seed, rng_directed):
    rng = np.random.default_rng(seed)
    n = 1 << scale
    m = ef * n
    src = np.zeros(m, dtype=np.int64)
    dst = np.zeros(m, dtype=np.int64)
    for _ in range(scale):
        r = rng.random(m)
        src = (src << 1) | (r >= 0.76)          # c + d quadrants
        dst = (dst << 1) | (((r >= 0.57) & (r < 0.76)) | (r >= 0.95))
    perm = rng.permutation(n)
    src, dst = perm[src], perm[dst]
    keep = src != dst
    return n, src[keep], dst[keep], rng.random(int(keep.sum())) * 0.999 + 0.001


def make(name, scale, ef, seed, directed):
    n, src, dst, w = rmat_edges(scale, ef, seed, directed)
    if not directed:   # one weight per unordered pair
        a, b = np.minimum(src, dst), np.maximum(src, dst)
        key = a * n + b
        _, first = np.unique(key, return_index=True)
        src, dst, w = a[first], b[first], w[first]
    else:
        key = src * n + dst
        _, first = np.unique(key, return_index=True)
        src, dst, w = src[first], dst[first], w[first]
    csr = csr_from_edges(n, src, dst, w, symmetric=not directed)
    A = sp.csr_matrix((csr.vals, csr.colidx.astype(np.int64), csr.rowptr.astype(np.int64)), shape=(n, n))
    deg = np.diff(csr.rowptr.astype(np.int64))
    source = int(np.argmax(deg))
    hops = csgraph.shortest_path(A, directed=True, unweighted=True, indices=source)
    bfs = np.full(n, INT64_MAX, dtype=np.int64)
    fin = np.isfinite(hops)
    bfs[fin] = hops[fin].astype(np.int64)
    dist = csgraph.dijkstra(A, directed=True, indices=source)
    _, lab = csgraph.connected_components(A, directed=True, connection="weak")
    minid = np.full(lab.max() + 1, n, dtype=np.int64)
    np.minimum.at(minid, lab, np.arange(n))
    wcc = minid[lab].astype(np.uint64)
    out = dict(n=np.int64(n), directed=np.int64(directed), rowptr=csr.rowptr, colidx=csr.colidx, vals=csr.vals,
               source=np.int64(source), bfs=bfs, sssp=dist, wcc=wcc)
    if not directed:
        G = nx.Graph()
        G.add_nodes_from(range(n))
        G.add_edges_from(zip(src.tolist(), dst.tolist()))
        cl = nx.clustering(G)
        out["lcc"] = np.array([cl[v] for v in range(n)], dtype=np.float64)
    np.savez_compressed(OUT / f"synthetic_{name}.npz", **out)
    print(name, n, csr.nnz)


if __name__ == "__main__":
    make("und_s9", 9, 8, 101, directed=False)
    make("dir_s9", 9, 6, 202, directed=True)
    make("und_s11", 11, 4, 303, directed=False)
