#!/usr/bin/env python3
"""Where k_pr_pull_units' x line fetches come from.

Counts the distinct (block, 128-B line of x) pairs of the sorted-block plan -- each is one
line fetch from the Infinity Cache / HBM when the block's sweep misses L2 -- split by the
column class (hub columns < H, tail columns >= H) and by the block's row count, on the
hub-first relabelled graph.  Optionally evaluates an alternative cut of the tail entries
(--tail-rows R2: the entries with columns >= H regrouped into blocks of R2 rows).

    python tools/pr_tail_model.py --scale 23 --ef 40 --seed 85 [--B 8388608 --R 16320] [--H 524288]
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def cut(rp, B, R):
    """Runs of <= B entries and <= R rows (pr_plan_sorted's sorted blocks; no LONG rows here)."""
    n = len(rp) - 1
    out = []
    r = 0
    while r < n:
        lim = min(n, r + R)
        k = int(np.searchsorted(rp[r + 1:lim + 1] - rp[r], B, side="right"))
        e = r + max(1, k)
        out.append((r, e))
        r = e
    return out


def sweep_groups(rp, ci, blocks, gsize=32):
    """Line fetches if the blocks ran in sweep groups of `gsize` (one XCD each, sweeping x in
    lockstep, so a line is fetched once per group): blocks in size order, consecutive groups."""
    sizes = [rp[b] - rp[a] for (a, b) in blocks]
    order = np.argsort(sizes)[::-1]
    total = 0
    for g0 in range(0, len(order), gsize):
        lines = np.unique(np.concatenate([np.unique(ci[rp[blocks[i][0]]:rp[blocks[i][1]]] >> 4)
                                          for i in order[g0:g0 + gsize]]))
        total += len(lines)
    return total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=23)
    ap.add_argument("--ef", type=int, default=40)
    ap.add_argument("--seed", type=int, default=85)
    ap.add_argument("--B", type=int, default=8 << 20)
    ap.add_argument("--R", type=int, default=16320)
    ap.add_argument("--H", type=int, nargs="*", default=[65536, 524288])
    ap.add_argument("--tail-rows", type=int, nargs="*", default=[])
    ap.add_argument("--groups", type=int, nargs="*", default=[], help="sweep-group sizes to model")
    args = ap.parse_args()
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    t0 = time.time()
    csr = rmat(args.scale, args.ef, args.seed, undirected=True)
    n = csr.n
    deg = np.diff(csr.rowptr.astype(np.int64))
    order = np.argsort(-deg, kind="stable")
    perm = np.empty(n, dtype=np.int64)
    perm[order] = np.arange(n)
    rp = np.zeros(n + 1, dtype=np.int64)
    rp[1:] = np.cumsum(deg[order])
    # relabelled columns, row by row in hub order (int32 to save memory)
    ci = np.empty(int(rp[-1]), dtype=np.int32)
    src_rp = csr.rowptr.astype(np.int64)
    step = 1 << 16
    for i0 in range(0, n, step):
        rows = order[i0:i0 + step]
        idx = np.concatenate([np.arange(src_rp[v], src_rp[v + 1]) for v in rows]) if len(rows) else np.zeros(0, np.int64)
        ci[rp[i0]:rp[min(n, i0 + step)]] = perm[csr.colidx[idx].astype(np.int64)]
    del csr
    print(f"graph {time.time() - t0:.0f} s: n={n} nnz={int(rp[-1])} live={int((deg > 0).sum())}", flush=True)
    blocks = cut(rp, args.B, args.R)
    H = sorted(args.H)
    tot = {h: [0, 0, 0, 0] for h in H}   # entries hub/tail, lines hub/tail
    by_rows = {}
    for (a, b) in blocks:
        lines = np.unique(ci[rp[a]:rp[b]] >> 4)
        cols = ci[rp[a]:rp[b]]
        cls = "rows=R" if b - a >= args.R else "entries=B"
        br = by_rows.setdefault(cls, [0, 0, 0, {}])
        br[0] += 1
        br[1] += len(cols)
        br[2] += len(lines)
        for h in H:
            t = cols >= h
            tl = lines >= (h >> 4)
            q = br[3].setdefault(h, [0, 0, 0, 0])
            q[0] += int((~t).sum())
            q[1] += int(t.sum())
            q[2] += int((~tl).sum())
            q[3] += int(tl.sum())
        for h in H:
            t = cols >= h
            tl = lines >= (h >> 4)
            tot[h][0] += int((~t).sum())
            tot[h][1] += int(t.sum())
            tot[h][2] += int((~tl).sum())
            tot[h][3] += int(tl.sum())
    print(f"B={args.B} R={args.R}: {len(blocks)} blocks")
    for cls, (nb, ne, nl, q) in by_rows.items():
        print(f"  blocks limited by {cls}: {nb}, entries {ne / 1e6:.1f} M, distinct lines {nl / 1e6:.2f} M "
              f"({ne / max(1, nl):.1f} entries per line fetch)")
        for h, (eh, et, lh, lt) in q.items():
            print(f"     H={h}: columns < H {eh / 1e6:.1f} M entries / {lh / 1e6:.2f} M lines; "
                  f">= H {et / 1e6:.1f} M / {lt / 1e6:.2f} M")
    for h in H:
        eh, et, lh, lt = tot[h]
        print(f"  H={h}: hub entries {eh / 1e6:.1f} M lines {lh / 1e6:.2f} M ({eh / max(1, lh):.1f}/line); "
              f"tail entries {et / 1e6:.1f} M lines {lt / 1e6:.2f} M ({et / max(1, lt):.1f}/line); "
              f"x line bytes {(lh + lt) * 128 / 1e9:.2f} GB")
    for gs in args.groups:
        f = sweep_groups(rp, ci, blocks, gs)
        print(f"  sweep groups of {gs} blocks in lockstep: {f / 1e6:.2f} M line fetches ({f * 128 / 1e9:.2f} GB)",
              flush=True)
    # alternative: tail entries (columns >= H) regrouped by taller row ranges
    for R2 in args.tail_rows:
        for h in H:
            lt = 0
            nb = 0
            for a in range(0, n, R2):
                b = min(n, a + R2)
                cols = ci[rp[a]:rp[b]]
                lt += len(np.unique(cols[cols >= h] >> 4))
                nb += 1
            print(f"  tail re-cut R2={R2} H={h}: {nb} tail blocks, tail lines {lt / 1e6:.2f} M "
                  f"({lt * 128 / 1e9:.2f} GB)")


if __name__ == "__main__":
    main()
