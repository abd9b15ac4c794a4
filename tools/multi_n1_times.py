#!/usr/bin/env python3
"""Wall time of the executables' multi-GPU entry points with one context against the single-GPU
calls on the config graphs (SYN-8_5 PageRank and SSSP, SYN-cit LCC): the fixed cost of the
N > 1 machinery (clique, per-round exchanges) at N = 1.  python tools/multi_n1_times.py"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import bench
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
    ctx = A.Context(0)
    arr = (C.c_void_p * 1)(ctx.handle.value)
    t = time.perf_counter()
    N.check(N.lib().gx_multi_prepare(arr, 1), "gx_multi_prepare")
    print(f"gx_multi_prepare (clique of one context) {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    for gname, alg in (("SYN-8_5", "pr"), ("SYN-8_5", "sssp"), ("SYN-cit", "lcc")):
        p = bench.PRESETS[gname]
        csr = rmat(p["scale"], p["ef"], p["seed"], undirected=p["undirected"], weighted=(alg == "sssp"))
        directed = not p["undirected"]
        s = csr.as_c()
        out = np.zeros(csr.n)
        src = int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))
        def multi():
            if alg == "pr":
                return N.lib().gx_pagerank_multi(arr, 1, C.byref(s), int(directed), 0.85, 10, N.as_dp(out))
            if alg == "sssp":
                return N.lib().gx_sssp_multi(arr, 1, C.byref(s), int(directed), src, N.as_dp(out))
            return N.lib().gx_lcc_multi(arr, 1, C.byref(s), int(directed), N.as_dp(out))
        G = A.Graph(ctx, csr, directed)
        def single():
            if alg == "pr":
                return A.LA_PR(G, 0.85, 10)
            if alg == "sssp":
                return A.LA_SSSP(G, src)
            return A.LA_LCC(G)
        for name, f in (("multi N=1 (whole call: upload + plan + run)", multi), ("single (warm call)", single)):
            f()
            t = time.perf_counter()
            for _ in range(3):
                rc = f()
                if name.startswith("multi"):
                    N.check(rc, alg)
            print(f"{gname} {alg}: {name} {(time.perf_counter() - t) / 3 * 1e3:.1f} ms", flush=True)
        G.close()
    ctx.close()


if __name__ == "__main__":
    main()
