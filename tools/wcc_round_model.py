#!/usr/bin/env python3
"""CPU model of Afforest's sampling rounds on the hub-first copy (gx_wcc.hip).

After round 0 (every vertex hooked to its first neighbour) the forest's roots are the minima of
the components of {(v, first neighbour of v)}.  The model counts them and the round-1 hooks
(v's root vs its second neighbour's root) that k_afforest_minhook would issue, for the copy's
rows in the parent's entry order (columns = original ids) and sorted by hub-first id.

    python tools/wcc_round_model.py [--scale 22 --ef 16 --seed 22]
"""
import argparse
import sys
from pathlib import Path

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def roots_after_round0(n, v, first):
    g = sp.coo_matrix((np.ones(len(v)), (v, first)), shape=(n, n)).tocsr()
    nc, lab = connected_components(g, directed=False)
    mins = np.full(nc, n, dtype=np.int64)
    np.minimum.at(mins, lab, np.arange(n))
    return mins[lab]


def report(name, n, deg, r, first_of, second_of):
    has = deg > 0
    vals, cnts = np.unique(r[has], return_counts=True)
    giant = vals[np.argmax(cnts)]
    out = has & (r != giant)
    v2 = np.nonzero(deg > 1)[0]
    a, b = r[v2], r[second_of(v2)]
    want = a != b
    high = np.maximum(a, b)[want]
    h, c = np.unique(high, return_counts=True)
    top = np.sort(c)[::-1][:5].tolist()
    print(f"{name}: roots {len(vals)}, giant {cnts.max()}, outside giant {int(out.sum())} "
          f"({int(deg[out].sum())} entries); round-1 hooks {int(want.sum())} at {len(h)} roots, hottest {top}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--ef", type=int, default=16)
    ap.add_argument("--seed", type=int, default=22)
    a = ap.parse_args()
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    csr = rmat(a.scale, a.ef, a.seed, undirected=True)
    n = csr.n
    rp = csr.rowptr.astype(np.int64)
    ci = csr.colidx.astype(np.int64)
    deg_o = np.diff(rp)
    order = np.argsort(-deg_o, kind="stable")          # hub-first position -> vertex
    perm = np.empty(n, dtype=np.int64)
    perm[order] = np.arange(n)
    deg = deg_o[order]                                  # degree of hub-first vertex x
    has = np.nonzero(deg > 0)[0]
    # parent's entry order: the first neighbour of x is perm[smallest original neighbour]
    first_p = lambda x: perm[ci[rp[order[x]]]]
    second_p = lambda x: perm[ci[rp[order[x]] + 1]]
    report("parent order", n, deg, roots_after_round0(n, has, first_p(has)), first_p, second_p)
    # sorted rows: the first neighbour is the smallest hub-first id
    # vectorised: the two smallest hub-first ids per row
    rows = np.repeat(np.arange(n), deg_o)
    hub_cols = perm[ci]
    key = perm[rows] * (n + 1) + hub_cols
    s = np.sort(key)
    xr, cc = s // (n + 1), s % (n + 1)
    start = np.searchsorted(xr, np.arange(n))
    first_s = lambda x: cc[start[x]]
    second_s = lambda x: cc[start[x] + 1]
    report("sorted rows", n, deg, roots_after_round0(n, has, first_s(has)), first_s, second_s)


if __name__ == "__main__":
    main()
