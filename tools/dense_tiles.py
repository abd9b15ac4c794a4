#!/usr/bin/env python3
"""Does the LCC / masked-SpGEMM operand form dense tiles?  (MFMA only where
the SpGEMM forms dense tiles.)  Counts, for the degree-oriented closure O of a stand-in graph in
hub-first order, the share of entries that sit in T x T tiles of at least a given fill, and
the share of the triangle-counting work (sum over (v, u) in O of |O(u)|) those tiles carry.

    python tools/dense_tiles.py [--graph SYN-cit|SYN-7_5] [--tile 16]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="SYN-cit")
    ap.add_argument("--tile", type=int, default=16)
    a = ap.parse_args()
    from bench import PRESETS
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    P = PRESETS[a.graph]
    csr = rmat(P["scale"], P["ef"], P["seed"], undirected=P["undirected"])
    n = csr.n
    rp = csr.rowptr.astype(np.int64)
    src = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    dst = csr.colidx.astype(np.int64)
    # closure S = A u A^T without self loops, then the degree orientation (low -> high degree, ties by id)
    u = np.concatenate([src, dst]); v = np.concatenate([dst, src])
    keep = u != v
    key = np.unique(u[keep] * n + v[keep])
    u, v = key // n, key % n
    deg = np.bincount(u, minlength=n)
    order = np.lexsort((np.arange(n), -deg))        # hub-first
    pos = np.empty(n, np.int64); pos[order] = np.arange(n)
    pu, pv = pos[u], pos[v]
    o = pv > pu                                       # oriented toward the later (lower-degree) position
    ou, ov = pu[o], pv[o]
    T = a.tile
    tid = (ou // T) * ((n + T - 1) // T) + ov // T
    tiles, cnt = np.unique(tid, return_counts=True)
    fill = cnt / float(T * T)
    # work: each (v, u) in O probes |O(u)|
    odeg = np.bincount(ou, minlength=n)
    work = odeg[ov]
    tw = np.bincount(np.searchsorted(tiles, tid), weights=work, minlength=len(tiles))
    print(f"{a.graph}: n={n} oriented entries={len(ou)} tiles {T}x{T} touched={len(tiles)} "
          f"mean fill {cnt.mean() / (T * T):.4f}")
    for f in (0.05, 0.125, 0.25, 0.5):
        m = fill >= f
        print(f"  tiles with fill >= {f:5.3f}: {m.sum():>8} tiles, {cnt[m].sum() / len(ou) * 100:5.2f} % of entries, "
              f"{tw[m].sum() / max(1.0, tw.sum()) * 100:5.2f} % of the probe work")


if __name__ == "__main__":
    main()
