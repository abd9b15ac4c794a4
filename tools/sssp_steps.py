#!/usr/bin/env python3
"""Per-step log of one warm gx_sssp run (GX_SSSP_VERBOSE=2: one step per batch, its bucket,
phase, items, edges, improvements and device time) on a bench stand-in, after two untimed calls
(the second builds the hub-first copy the warm calls run on).

    python tools/sssp_steps.py [--graph SYN-8_5] > steps.txt
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="SYN-8_5")
    a = ap.parse_args()
    import bench
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    p = bench.PRESETS[a.graph]
    csr = rmat(p["scale"], p["ef"], p["seed"], undirected=p["undirected"], weighted=True)
    ctx = A.Context(0)
    G = A.Graph(ctx, csr, not p["undirected"])
    src = int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))
    import time
    t0 = time.perf_counter()
    ref = A.LA_SSSP(G, src)
    t1 = time.perf_counter()
    A.LA_SSSP(G, src)   # builds the hub-first copy
    t2 = time.perf_counter()
    A.LA_SSSP(G, src)
    t3 = time.perf_counter()
    print(f"first call {1e3 * (t1 - t0):.1f} ms, second (hub-first copy built) {1e3 * (t2 - t1):.1f} ms, "
          f"warm {1e3 * (t3 - t2):.1f} ms", flush=True)
    os.environ["GX_SSSP_VERBOSE"] = "2"
    got = A.LA_SSSP(G, src)
    assert np.array_equal(got, ref)
    G.close()
    ctx.close()


if __name__ == "__main__":
    main()
