#!/usr/bin/env python3
"""Probe: warm-call device time of BFS / WCC / SSSP / LCC on a graph in its generated vertex
order against the same graph relabelled hub-first (out-degree descending), to size what a
relabelled copy would buy the gather-bound kernels (PR's x gathers went 393 -> 283 us per
launch from the same reordering).

    python tools/relabel_probe.py sssp:SYN-8_5 bfs:SYN-g500-22 wcc:SYN-g500-22
"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import PRESETS  # noqa: E402
from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A  # noqa: E402
from ldbc_graphalytics_platforms_graphblas_amd.graphio import CSR, rmat  # noqa: E402


def hub_order(csr):
    """(perm, relabelled CSR): row order[i] becomes row i, columns renamed, rows unsorted."""
    n = csr.n
    rp = csr.rowptr.astype(np.int64)
    deg = np.diff(rp)
    order = np.argsort(-deg, kind="stable")
    perm = np.empty(n, dtype=np.int64)
    perm[order] = np.arange(n, dtype=np.int64)
    nd = deg[order]
    nrp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nd, out=nrp[1:])
    idx = np.repeat(rp[order] - nrp[:-1], nd) + np.arange(int(nrp[-1]), dtype=np.int64)
    nci = perm[csr.colidx.astype(np.int64)[idx]].astype(np.uint64)
    vals = None if csr.vals is None else np.ascontiguousarray(csr.vals[idx])
    return perm, CSR(n, nrp.astype(np.uint64), nci, vals)


def timed(ctx, G, fn, reps=5):
    fn(G)
    fn(G)
    ms = []
    for _ in range(reps):
        out = fn(G)
        ms.append(ctx.last_device_ms())
    return out, float(np.median(ms))


def main():
    ctx = A.Context(0)
    for spec in sys.argv[1:]:
        alg, gname = spec.split(":")
        P = PRESETS[gname]
        csr = rmat(P["scale"], P["ef"], P["seed"], undirected=P["undirected"], weighted=(alg == "sssp"))
        directed = not P["undirected"]
        deg = np.diff(csr.rowptr.astype(np.int64))
        src = int(np.argmax(deg))
        t0 = time.time()
        perm, hub = hub_order(csr)
        t_rel = time.time() - t0
        fns = {"bfs": lambda G, s: A.LA_BFS(G, s), "sssp": lambda G, s: A.LA_SSSP(G, s),
               "wcc": lambda G, s: A.WeaklyConnectedComponents(G), "lcc": lambda G, s: A.LA_LCC(G)}
        f = fns[alg]
        G0 = A.Graph(ctx, csr, directed)
        out0, ms0 = timed(ctx, G0, lambda G: f(G, src))
        G0.close()
        G1 = A.Graph(ctx, hub, directed)
        out1, ms1 = timed(ctx, G1, lambda G: f(G, int(perm[src])))
        G1.close()
        back = out1[perm]
        if alg == "wcc":
            same = len(np.unique(out0)) == len(np.unique(back))
        elif alg == "lcc":
            same = np.allclose(out0, back, rtol=1e-12, atol=0)
        else:
            same = np.array_equal(out0, back)
        print(f"{alg} {gname}: generated order {ms0:.3f} ms, hub-first {ms1:.3f} ms "
              f"({ms0 / ms1:.2f}x; host relabel {t_rel:.1f} s; results {'agree' if same else 'DIFFER'})", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
