#!/usr/bin/env python3
"""Whole-call wall time of bin/exe/pr's multi-GPU entry point (gx_pagerank_multi) on SYN-8_5
against the single-GPU call (gx_pagerank_csr), one MI355X: N = 1 (routed to the single call) and
k virtual devices (k contexts on device 0: every device's upload, plan, pieces and exchanges run
one after the other on the one GPU), with the partitioned upload ("rows") or the whole graph
on every device ("whole"), and 1 or 2 pipelined pieces.  Each k-device result is checked
against the single call's (rtol 1e-12).

python tools/multi_pr_times.py [k ...]          (default 8)
GX_PLAN_TIMES=1 adds the partitioned upload's input-columns counter on stderr."""
import ctypes as C
import os
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
    ks = [int(a) for a in sys.argv[1:]] or [8]
    p = bench.PRESETS["SYN-8_5"]
    csr = rmat(p["scale"], p["ef"], p["seed"], undirected=p["undirected"])
    s = csr.as_c()
    ctxs = [A.Context(0) for _ in range(max(ks))]
    try:
        def call(k, env):
            for key, val in env.items():
                os.environ[key] = val
            out = np.zeros(csr.n)
            arr = (C.c_void_p * k)(*[c.handle.value for c in ctxs[:k]])
            N.check(N.lib().gx_multi_prepare(arr, k), "gx_multi_prepare")
            t = time.perf_counter()
            N.check(N.lib().gx_pagerank_multi(arr, k, C.byref(s), 0, 0.85, 10, N.as_dp(out)), "gx_pagerank_multi")
            dt = time.perf_counter() - t
            for key in env:
                del os.environ[key]
            return dt, out

        # the single-GPU call (bin/exe/pr's N = 1 path), warm
        ref = np.zeros(csr.n)
        times = []
        for _ in range(4):
            t = time.perf_counter()
            N.check(N.lib().gx_pagerank_csr(ctxs[0].handle, C.byref(s), 0, 0.85, 10, N.as_dp(ref), None),
                    "gx_pagerank_csr")
            times.append(time.perf_counter() - t)
        print(f"SYN-8_5 gx_pagerank_csr (whole call): {min(times[1:]) * 1e3:.1f} ms "
              f"(runs {', '.join(f'{x * 1e3:.1f}' for x in times)})", flush=True)
        variants = [(1, {})]
        for k in ks:
            variants += [(k, {"GX_PR_MULTI_UPLOAD": u, "GX_PR_MULTI_PIECES": str(pc)})
                         for u in ("rows", "whole") for pc in (1, 2)]
        # MULTI_ONLY=k:upload:pieces runs that variant alone (for rocprofv3 kernel statistics)
        only = os.environ.get("MULTI_ONLY")
        if only:
            k, u, pc = only.split(":")
            variants = [(int(k), {"GX_PR_MULTI_UPLOAD": u, "GX_PR_MULTI_PIECES": pc})]
        for k, env in variants:
            res = [call(k, env) for _ in range(3)]
            best = min(r[0] for r in res[1:])
            err = float(np.max(np.abs(res[-1][1] - ref) / np.abs(ref)))
            label = ", ".join(f"{a}={b}" for a, b in env.items()) or "default"
            print(f"SYN-8_5 gx_pagerank_multi k={k} ({label}): {best * 1e3:.1f} ms "
                  f"(runs {', '.join(f'{r[0] * 1e3:.1f}' for r in res)}); max rel err vs single {err:.1e}", flush=True)
            assert err <= 1e-12, err
    finally:
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()
