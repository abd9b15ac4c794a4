#!/usr/bin/env python3
"""Offline model of k_pr_pull_sorted's x-gather line requests.

Each 64-entry group of a column-sorted block is one wave-instruction; every distinct 128-B
line of x it touches is one L1 miss -> one L2 request.  The model counts them for a block
layout (entries per block, rows per block) and a vertex order, so layouts can be compared on
the CPU before they are built (the GPU count on SYN-7_5 was 13.6 M x requests per launch,
15.5 M with the index stream: profiles/pmc_pr_pull.json).

    python tools/pr_line_model.py [--scale 20 --ef 32 --seed 75] [--order hub|...]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def blocks_of(rp, B, R):
    """pr_plan_sorted's cut: runs of rows with <= B entries and <= R rows; rows > B are LONG."""
    rows = len(rp) - 1
    out, long_rows = [], []
    r = 0
    deg = np.diff(rp)
    while r < rows:
        if deg[r] > B:
            long_rows.append(r)
            r += 1
            continue
        start = r
        # vectorised scan: the largest end with nz <= B and end - start <= R, stopping at a LONG row
        lim = min(rows, start + R)
        cum = rp[start + 1:lim + 1] - rp[start]
        k = int(np.searchsorted(cum, B, side="right"))
        end = start + max(1, k)
        seg = deg[start:end]
        big = np.nonzero(seg > B)[0]
        if len(big):
            end = start + int(big[0])
        out.append((start, end))
        r = end
    return out, long_rows


def count_requests(rp, ci, blocks, line_shift=4, group=64):
    """x line requests of the sorted blocks: sum over 64-entry groups of distinct lines."""
    total = 0
    ents = 0
    for (a, b) in blocks:
        cols = np.sort(ci[rp[a]:rp[b]])
        m = len(cols)
        ents += m
        lines = cols >> line_shift
        g = np.arange(m) // group
        # distinct (group, line) pairs in a sorted array: count changes
        new = np.ones(m, dtype=bool)
        new[1:] = (lines[1:] != lines[:-1]) | (g[1:] != g[:-1])
        total += int(new.sum())
    return total, ents


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--ef", type=int, default=32)
    ap.add_argument("--seed", type=int, default=75)
    ap.add_argument("--B", type=int, nargs="*", default=[65536])
    ap.add_argument("--R", type=int, nargs="*", default=[4096])
    args = ap.parse_args()
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import hub_relabel
    csr = rmat(args.scale, args.ef, args.seed, undirected=True)
    _, hub = hub_relabel(csr)
    rp = hub.rowptr.astype(np.int64)
    ci = hub.colidx.astype(np.int64)
    deg = np.diff(rp)
    print(f"n={hub.n} nnz={hub.nnz} nonzero-degree={int((deg > 0).sum())}")
    # column-degree profile: share of entries whose column is below c
    cdeg = np.bincount(ci, minlength=hub.n)
    cum = np.cumsum(cdeg) / max(1, hub.nnz)
    for c in (1024, 4096, 16384, 65536, 262144, 524288):
        if c <= hub.n:
            print(f"  columns < {c:>7}: {cum[c - 1] * 100:5.1f} % of entries")
    for B in args.B:
        for R in args.R:
            blocks, longr = blocks_of(rp, B, R)
            req, ents = count_requests(rp, ci, blocks)
            print(f"B={B:>7} R={R:>5}: blocks={len(blocks):>5} long={len(longr):>3} "
                  f"entries={ents} x-requests={req / 1e6:.2f} M ({ents / max(1, req):.2f} entries/request)")


if __name__ == "__main__":
    main()
