#!/usr/bin/env python3
"""Offline model of PageRank's wide tail under two vertex orders (round 6).

The round-6 probes (profiles/r06_pr_probes_wide_tail.txt) put the wide entries' gathers at
~125 us of SYN-8_5's ~685 us probe launch: 5 % of the entries, each a gather into the sparse tail
of x.  Those entries are columns (sources) of low degree met inside hub blocks.  Among vertices of
equal degree the hub-first order breaks ties by id, so a block's tail columns are scattered over
x.  The "tail key" order breaks the ties by s(c) = the hub-first position of c's highest-degree
neighbour instead: vertices whose strongest neighbour is the same hub become adjacent in x, and
that hub's block sees them as a dense run.

For each order this cuts the relabelled rows as the huge-graph plan does (16 320 rows / 32 Mi
entries per block), sorts every block's entries by column and counts
- narrow-able entries (step from the previous sorted entry of the block <= 3),
- wide entries (the rest) and their x line requests: distinct 128-B lines per 64-entry group
  of the block's wide entries (the line model of tools/pr_line_model.py).

python tools/pr_tail_order_model.py [scale edgefactor seed]   (default 23 40 85: SYN-8_5)"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat  # noqa: E402


def cut(hdeg, R=16320, B=32 << 20):
    n = len(hdeg)
    pre = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(hdeg, out=pre[1:])
    starts, r = [], 0
    while r < n:
        e = int(np.searchsorted(pre, pre[r] + B, side="right")) - 1
        e = max(r + 1, min(e, r + R, n))
        starts.append(r)
        r = e
    starts.append(n)
    return np.asarray(starts, dtype=np.int64)


def model(name, order, rp, ci, deg):
    t = time.time()
    n = len(deg)
    perm = np.empty(n, dtype=np.int64)
    perm[order] = np.arange(n)
    st = cut(deg[order])
    bpos = np.searchsorted(st, np.arange(n), side="right") - 1   # block of each position
    bvert = bpos[perm].astype(np.uint64)                         # block of each vertex's row
    erow = np.repeat(np.arange(n, dtype=np.int64), deg)
    key = (bvert[erow] << np.uint64(32)) | perm[ci].astype(np.uint64)
    del erow
    key.sort()
    blk = (key >> np.uint64(32)).astype(np.int64)
    col = (key & np.uint64(0xFFFFFFFF)).astype(np.int64)
    del key
    step = np.empty_like(col)
    step[0] = 0
    step[1:] = col[1:] - col[:-1]
    first = np.ones(len(col), dtype=bool)
    first[1:] = blk[1:] != blk[:-1]
    step[first] = 0
    wide = step > 3
    nw = int(wide.sum())
    wc, wb = col[wide], blk[wide]
    # 64-entry groups of each block's wide entries
    idx = np.arange(nw, dtype=np.int64)
    bstart = np.zeros(nw, dtype=np.int64)
    if nw:
        newb = np.ones(nw, dtype=bool)
        newb[1:] = wb[1:] != wb[:-1]
        bstart = np.maximum.accumulate(np.where(newb, idx, 0))
    g = (idx - bstart) // 64
    lines = wc >> 4
    newl = np.ones(nw, dtype=bool)
    newl[1:] = (lines[1:] != lines[:-1]) | (g[1:] != g[:-1]) | (wb[1:] != wb[:-1])
    req = int(newl.sum())
    print(f"{name}: {len(st) - 1} blocks; entries {len(col)}; narrow-able {len(col) - nw} "
          f"({(len(col) - nw) / len(col):.3f}); wide {nw} ({nw / len(col):.3f}); wide x line requests {req} "
          f"({req / max(nw, 1):.3f} per wide entry) [{time.time() - t:.0f} s]", flush=True)


def main():
    args = [int(a) for a in sys.argv[1:]]
    scale, ef, seed = args[:3] if len(args) >= 3 else (23, 40, 85)
    t = time.time()
    csr = rmat(scale, ef, seed)
    rp = csr.rowptr.astype(np.int64)
    ci = csr.colidx.astype(np.int64)
    deg = np.diff(rp)
    n = len(deg)
    print(f"R-MAT {scale}/{ef}/{seed}: n {n} nnz {rp[-1]} ({time.time() - t:.0f} s)", flush=True)
    hub = np.argsort(-deg, kind="stable")
    model("hub-first (degree, id)", hub, rp, ci, deg)
    perm0 = np.empty(n, dtype=np.int64)
    perm0[hub] = np.arange(n)
    s = np.full(n, n, dtype=np.int64)
    nz = deg > 0
    s[nz] = np.minimum.reduceat(perm0[ci], rp[:-1][nz])
    tail = np.lexsort((np.arange(n), s, -deg))
    model("tail key (degree, strongest neighbour, id)", tail, rp, ci, deg)


if __name__ == "__main__":
    main()
