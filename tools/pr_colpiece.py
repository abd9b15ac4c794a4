#!/usr/bin/env python3
"""One rank's SpMV under a column (2-D) partition of config 4's PageRank, timed on one GPU
(VERDICT r03 next #6).

Rank p of P owns the columns whose hub-first position is p mod P (dealt round-robin like the
1-D rows, so every rank gets the same mix of hub and tail columns) and ALL rows: its SpMV
gathers only its x slice (n / P doubles) and writes partial sums for every row, which a
reduce-scatter would then combine.  The piece is planned by the product's partition path
(gx_pr_part_create: column-sorted blocks, units, narrow codes) with the columns renamed to the
slice, so x_full holds the slice at its front; the launch time is what a rank's kernel costs.
The values are not a PageRank (no exchange is simulated); only the time is reported.

    python tools/pr_colpiece.py [--scale 23 --ef 40 --seed 85] [--pieces 8] [--piece 0] [--steps 20]
"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def column_piece(csr, P, p):
    n = csr.n
    rp = csr.rowptr.astype(np.int64)
    deg = np.diff(rp)
    order = np.argsort(-deg, kind="stable")
    pos = np.empty(n, dtype=np.int64)
    pos[order] = np.arange(n)
    colpos = pos[csr.colidx.astype(np.int64)]
    keep = (colpos % P) == p
    row = np.repeat(pos, deg)[keep]            # rows in hub-first order
    col = colpos[keep] // P                    # the slice's local column
    del colpos
    key = np.sort((row << 32) | col)
    row, col = key >> 32, key & 0xffffffff
    counts = np.bincount(row, minlength=n)
    lrp = np.zeros(n + 1, dtype=np.uint64)
    lrp[1:] = np.cumsum(counts)
    outdeg = deg[order].astype(np.uint64)      # every row's global out-degree (hub-first order)
    return lrp, col.astype(np.uint64), outdeg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=23)
    ap.add_argument("--ef", type=int, default=40)
    ap.add_argument("--seed", type=int, default=85)
    ap.add_argument("--pieces", type=int, default=8)
    ap.add_argument("--piece", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    t0 = time.time()
    csr = rmat(args.scale, args.ef, args.seed, undirected=True)
    n = csr.n
    lrp, lci, outdeg = column_piece(csr, args.pieces, args.piece)
    nnz_piece = int(lrp[-1])
    del csr
    t_build = time.time() - t0
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = Context(0)
    lib = N.lib()
    part = C.c_void_p()
    ranges = np.array([0, n], dtype=np.uint64)
    N.check(lib.gx_pr_part_create(ctx.handle, n, 1, 0, N.as_u64p(ranges), N.as_u64p(lrp), N.as_u64p(lci),
                                  N.as_u64p(outdeg), 0.85, C.byref(part)), "gx_pr_part_create")
    chunk = C.c_uint64()
    N.check(lib.gx_pr_part_chunk(part, C.byref(chunk)), "gx_pr_part_chunk")
    stream = torch.cuda.Stream(dev)
    xa = torch.zeros(chunk.value, dtype=torch.float64, device=dev)
    xb = torch.zeros(chunk.value, dtype=torch.float64, device=dev)
    sp = C.c_void_p(stream.cuda_stream)
    N.check(lib.gx_pr_part_init(part, C.c_void_p(xa.data_ptr()), sp), "gx_pr_part_init")
    for _ in range(3):
        N.check(lib.gx_pr_part_step(part, C.c_void_p(xa.data_ptr()), C.c_void_p(xb.data_ptr()), None, sp), "step")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    for i in range(args.steps):
        a, b = (xa, xb) if i % 2 == 0 else (xb, xa)
        N.check(lib.gx_pr_part_step(part, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), None, sp), "step")
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    us = ev0.elapsed_time(ev1) * 1e3 / args.steps
    lib.gx_pr_part_free(part)
    ctx.close()
    print(json.dumps({"graph": f"rmat({args.scale},{args.ef},{args.seed})", "n": n, "pieces": args.pieces,
                      "piece": args.piece, "nnz_piece": nnz_piece, "x_slice_doubles": (n + args.pieces - 1) // args.pieces,
                      "us_per_launch": us, "build_s": t_build}), flush=True)


if __name__ == "__main__":
    main()
