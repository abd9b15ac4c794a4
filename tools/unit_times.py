#!/usr/bin/env python3
"""Summarise a GX_PR_UNIT_TIMES dump (per-workgroup s_memrealtime stamps, 100 MHz) of one
k_pr_pull_units launch: launch span, start skew, the slowest units and time per entry."""
import sys
import numpy as np

for path in sys.argv[1:]:
    rows = [l.split() for l in open(path).read().splitlines()[1:]]
    kind = np.array([r[1] for r in rows])
    ents = np.array([int(r[5]) for r in rows], dtype=np.int64)
    nrow = np.array([int(r[6]) for r in rows], dtype=np.int64)
    nun = np.array([int(r[4]) for r in rows], dtype=np.int64)
    t0 = np.array([int(r[7]) for r in rows], dtype=np.int64)
    tg = np.array([int(r[8]) for r in rows], dtype=np.int64)
    t1 = np.array([int(r[9]) for r in rows], dtype=np.int64)
    base = t0.min()
    us = lambda x: x / 100.0
    dur = t1 - t0
    print(f"== {path}: {len(rows)} workgroups, span {us(t1.max() - base):.1f} us, "
          f"last start {us(t0.max() - base):.1f} us, median dur {us(np.median(dur)):.1f} us")
    cus = 256
    busy = [int((((t0 - base) <= t * 100) & ((t1 - base) > t * 100)).sum()) for t in range(0, int(us(t1.max() - base)), 10)]
    print(f"   sum of item durations / {cus} CUs {us(dur.sum()) / cus:.1f} us (the balanced span); "
          f"items in flight every 10 us: {busy}")
    u = kind == "unit"
    g = tg - t0
    rate = ents[u] / np.maximum(1, g[u])   # entries per 10 ns
    print(f"   units: entries/us median {np.median(rate) * 100:.0f}, p10 {np.percentile(rate, 10) * 100:.0f}, "
          f"p90 {np.percentile(rate, 90) * 100:.0f}; gather share of duration {np.median(g[u] / np.maximum(1, dur[u])):.2f}")
    order = np.argsort(-(t1 - base))[:12]
    print("   last to finish: wg kind blk unit/n entries rows start gather end")
    for i in order:
        r = rows[i]
        print(f"     {r[0]:>5} {r[1]:4} {r[2]:>4} {r[3]:>2}/{r[4]:<2} {int(r[5]):>7} {int(r[6]):>5} "
              f"{us(t0[i] - base):7.1f} {us(g[i]):7.1f} {us(t1[i] - base):7.1f}")
    # time per entry by block row count bucket
    for lo, hi in ((0, 64), (64, 512), (512, 2048), (2048, 5000)):
        m = u & (nrow >= lo) & (nrow < hi)
        if m.any():
            print(f"   rows [{lo},{hi}): {m.sum():4} units, {ents[m].sum() / 1e6:6.2f} M entries, "
                  f"entries/us {np.median(ents[m] / np.maximum(1, g[m])) * 100:.0f}, gather us median {us(np.median(g[m])):.1f} max {us(g[m].max()):.1f}")
