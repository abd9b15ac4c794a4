"""How much of x each rank's PageRank blocks read ("before building,
measure per rank which fraction of x its blocks reference").

The N-rank block partition (pr_partition.block_relabel: the single-GPU plan's blocks dealt
whole, LPT) gives every vertex an owner.  Rank r's SpMV reads x[c] for every column c of its
rows; x[c] arrives from owner(c) when owner(c) != r, and only live columns (out-degree > 0) are
exchanged at all.  Reported per N:
- frac_read: distinct columns rank r reads / n (mean, min, max over ranks);
- allgather_in: doubles into a rank per iteration with the padded all-gather ((N-1) x chunk);
- needed_in: doubles into a rank if each peer sent only the live columns r reads (mean, max);
- ratio = max needed_in / allgather_in.

CPU only (the graph comes from libgx's seeded R-MAT generator).
Usage: python tools/pr_xref.py [scale edgefactor seed] [N ...]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat  # noqa: E402
from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import _deal_blocks  # noqa: E402


def owners(deg: np.ndarray, nparts: int, rows_per_block: int = 16320, block_nnz: int = 32 << 20) -> np.ndarray:
    """owner[v] under block_relabel's cut and deal (same blocks, no relabelled copy)."""
    n = len(deg)
    hub = np.argsort(-deg, kind="stable")
    hdeg = deg[hub]
    pre = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(hdeg, out=pre[1:])
    starts, r = [], 0
    while r < n:
        lim = min(n, r + rows_per_block)
        e = int(np.searchsorted(pre, pre[r] + block_nnz, side="right")) - 1
        e = max(r + 1, min(e, lim))
        starts.append(r)
        r = e
    starts.append(n)
    st = np.asarray(starts, dtype=np.int64)
    work = (pre[st[1:]] - pre[st[:-1]]) + np.diff(st)
    live = np.add.reduceat((hdeg > 0).astype(np.int64), st[:-1])
    bown = np.zeros(len(st) - 1, dtype=np.int64)
    _deal_blocks(work, live, nparts, bown)
    own_h = np.repeat(bown, np.diff(st)).astype(np.int8)
    owner = np.empty(n, dtype=np.int8)
    owner[hub] = own_h
    return owner


def main():
    args = [int(a) for a in sys.argv[1:]]
    scale, ef, seed = (args[:3] if len(args) >= 3 else (23, 40, 85))
    ns = args[3:] or [2, 4, 8]
    t0 = time.time()
    csr = rmat(scale, ef, seed)
    n = csr.n
    rp = csr.rowptr.astype(np.int64)
    deg = np.diff(rp)
    ci = csr.colidx.astype(np.int32)
    live = deg > 0
    print(f"R-MAT scale {scale} ef {ef} seed {seed}: n {n} nnz {rp[-1]} live {int(live.sum())} "
          f"({time.time() - t0:.1f} s)", flush=True)
    for N in ns:
        owner = owners(deg, N)
        eown = np.repeat(owner, deg)
        lives = [int((live & (owner == q)).sum()) for q in range(N)]
        chunk = max(lives) + 2
        fr, need = [], []
        for r in range(N):
            mark = np.zeros(n, dtype=bool)
            mark[ci[eown == r]] = True
            fr.append(mark.sum() / n)
            ext = mark & live & (owner != r)
            need.append(int(ext.sum()))
        ag = (N - 1) * chunk
        print(f"N={N}: frac_read mean {np.mean(fr):.3f} min {min(fr):.3f} max {max(fr):.3f}; "
              f"allgather_in {ag} doubles ({8 * ag / 1e6:.1f} MB); needed_in mean {np.mean(need):.0f} "
              f"max {max(need)} ({8 * max(need) / 1e6:.1f} MB); ratio {max(need) / ag:.3f}", flush=True)


if __name__ == "__main__":
    main()
