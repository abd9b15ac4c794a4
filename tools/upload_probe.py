#!/usr/bin/env python3
"""gx_graph_create (the upload half of the Graphalytics processing time) under the upload
knobs, on one graph generated once.

    GX_PLAN_TIMES=1 python tools/upload_probe.py [--scale 23 --ef 40 --seed 85]

Settings are "BUFS/THREADS/NT" (GX_UPLOAD_BUFS, GX_UPLOAD_THREADS with 0 = the default,
GX_UPLOAD_NT); each is timed --reps times and the best is printed, one JSON line in all.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=23)
    ap.add_argument("--ef", type=int, default=40)
    ap.add_argument("--seed", type=int, default=85)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--torch", action="store_true", help="import torch and run CPU and GPU ops first, as bench.py does")
    ap.add_argument("--settings", nargs="*", default=["2/0/0", "2/0/1", "4/0/0", "4/0/1", "3/8/1", "4/12/1"])
    args = ap.parse_args()
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context, Graph
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    csr = rmat(args.scale, args.ef, args.seed, undirected=True)
    if args.torch:
        import torch
        torch.cuda.set_device(0)
        torch.ones(1 << 24).sum().item()
        x = torch.ones(1 << 28, device="cuda")
        (x * 2).sum().item()
        del x
    ctx = Context(0)
    out = {"graph": f"rmat({args.scale},{args.ef},{args.seed})", "nnz": int(csr.nnz), "torch": args.torch}
    for s in args.settings:
        b, t, nt = s.split("/")
        os.environ["GX_UPLOAD_BUFS"], os.environ["GX_UPLOAD_THREADS"], os.environ["GX_UPLOAD_NT"] = b, t, nt
        best = None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            G = Graph(ctx, csr, False)
            ms = (time.perf_counter() - t0) * 1e3
            G.close()
            best = ms if best is None else min(best, ms)
        out[s] = round(best, 2)
        print(f"{s}: {best:.2f} ms", file=sys.stderr, flush=True)
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
