"""Multi-GPU BFS, WCC, SSSP, CDLP and LCC: one process per GPU, the graph
replicated on every rank, ranks owning contiguous vertex ranges, one RCCL collective per
round.  (PageRank, whose exchange is the rank vector, lives in pr_partition.py.)

The drivers below run a list of *local ranks* in lock step against a `Comm`:

* TorchComm -- one local rank per process; collectives are torch.distributed (backend
  "nccl" = RCCL over xGMI on MI355X, or gloo on CPU).
* LocalComm -- all ranks in this process; a collective combines the per-rank tensors.
  Used to run the partitioned GPU path with 1..k simulated ranks on one device.

A backend supplies the per-rank device steps; GpuBackend binds the gx_*_part_* entry
points of libgx (include/gx.h).  Every state array is full length on every rank:

    BFS  : expand owned frontier rows -> next (uint8)   the discoveries as words, or
                                                          all-reduce MAX; commit levels
    WCC  : hook owned rows' edges     -> parent (int32) the changed entries as words (MIN),
                                                          or all-reduce MIN; compress
    SSSP : 1-D split (gx_sssp_split): relax the edges into owned vertices -> the improved
           owned vertices as (vertex, fp64 bits) pairs, all-gathered (sparse, per round)
    CDLP : new labels of owned rows   -> the changed labels as words, or all-gather of
                                         the owned slices

The words exchange (_exchange, gx_part_changes / gx_part_apply) moves 8 bytes per changed
entry after a count all-gather, and falls back to the dense collective when that is more.
    LCC  : triangle counts of owned orientation sources -> all-reduce SUM, finish

Results are the single-GPU results (BFS levels, canonical WCC labels, the SSSP fixed point,
the CDLP labels, exact LCC counts).  The reference has no distributed path.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from .pr_partition import partition_rows

INF_LEVEL = np.iinfo(np.int64).max


# ---------------------------------------------------------------------------- comms
class LocalComm:
    """All ranks live in this process: combine the per-rank tensors elementwise."""

    world_size = None   # = the number of local ranks

    def all_reduce(self, ts: Sequence, op: str) -> None:
        import torch
        r = ts[0].clone()
        for t in ts[1:]:
            if op == "min":
                r = torch.minimum(r, t)
            elif op == "max":
                r = torch.maximum(r, t)
            elif op == "sum":
                r = r + t
            else:
                raise ValueError(op)
        for t in ts:
            t.copy_(r)

    def all_gather(self, outs: Sequence, ins: Sequence) -> None:
        import torch
        cat = torch.cat(list(ins))
        for o in outs:
            o.copy_(cat)


class TorchComm:
    """One local rank per process; torch.distributed collectives (RCCL or gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.ops = {"min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX, "sum": dist.ReduceOp.SUM}

    def all_reduce(self, ts: Sequence, op: str) -> None:
        for t in ts:
            self.dist.all_reduce(t, op=self.ops[op], group=self.group)

    def all_gather(self, outs: Sequence, ins: Sequence) -> None:
        gloo = self.dist.get_backend(self.group) == "gloo"
        for o, i in zip(outs, ins):
            if gloo:   # gloo has no all_gather_into_tensor
                parts = list(o.chunk(self.world_size))
                self.dist.all_gather(parts, i, group=self.group)
            else:
                self.dist.all_gather_into_tensor(o, i, group=self.group)


# ------------------------------------------------------------------------- backend
class GpuBackend:
    """gx_*_part_* of libgx on one device for one rank; tensors are torch CUDA tensors.
    Steps launch on torch's current stream by default, so they are ordered with the
    tensor initialisation and the collectives torch issues on that stream."""

    def __init__(self, graph, stream_handle=None):
        from . import _native as N
        self.N = N
        self.lib = N.lib()
        self.g = graph.handle
        if stream_handle is None:
            import torch
            stream_handle = lambda: torch.cuda.current_stream().cuda_stream   # noqa: E731
        self.stream = stream_handle

    @staticmethod
    def _p(t):
        return C.c_void_p(t.data_ptr())

    def _s(self):
        return C.c_void_p(self.stream())

    def bfs_init(self, src, level):
        self.N.check(self.lib.gx_bfs_part_init(self.g, src, self._p(level), self._s()), "gx_bfs_part_init")

    def bfs_expand(self, v0, v1, level, cur, nxt):
        self.N.check(self.lib.gx_bfs_part_expand(self.g, v0, v1, self._p(level), cur, self._p(nxt), self._s()),
                     "gx_bfs_part_expand")

    def bfs_commit(self, nxt, level, cur, count):
        self.N.check(self.lib.gx_bfs_part_commit(self.g, self._p(nxt), self._p(level), cur, self._p(count),
                                                 self._s()), "gx_bfs_part_commit")

    def changes(self, a, b, v0, v1, elem, words, count):
        self.N.check(self.lib.gx_part_changes(self._p(a), self._p(b) if b is not None else None, v0, v1, elem,
                                              self._p(words), self._p(count), self._s()), "gx_part_changes")

    def apply(self, words, counts, nranks, stride, arr, elem, op):
        self.N.check(self.lib.gx_part_apply(self._p(words), self._p(counts), nranks, stride, self._p(arr), elem, op,
                                            self._s()), "gx_part_apply")

    def pack_bits(self, nxt, bits):
        self.N.check(self.lib.gx_part_pack_bits(self._p(nxt), nxt.numel(), self._p(bits), self._s()), "gx_part_pack_bits")

    def or_bits(self, gathered, nranks, nxt):
        self.N.check(self.lib.gx_part_or_bits(self._p(gathered), nranks, nxt.numel(), self._p(nxt), self._s()),
                     "gx_part_or_bits")

    def wcc_init(self, parent):
        self.N.check(self.lib.gx_wcc_part_init(self.g, self._p(parent), self._s()), "gx_wcc_part_init")

    def wcc_hook(self, v0, v1, parent, changed):
        self.N.check(self.lib.gx_wcc_part_hook(self.g, v0, v1, self._p(parent), self._p(changed), self._s()),
                     "gx_wcc_part_hook")

    def wcc_compress(self, parent):
        self.N.check(self.lib.gx_wcc_part_compress(self.g, self._p(parent), self._s()), "gx_wcc_part_compress")

    def sssp_split(self, v0, v1):
        return _GpuSsspSplit(self, v0, v1)

    def cdlp_part(self, v0, v1):
        return _GpuCdlpPart(self, v0, v1)

    def lcc_part(self):
        return _GpuLccPart(self)


class _GpuSsspSplit:
    """gx_sssp_split_* for one rank: owned targets [v0, v1)."""

    def __init__(self, be: GpuBackend, v0: int, v1: int):
        self.be = be
        self.h = C.c_void_p()
        be.N.check(be.lib.gx_sssp_split_create(be.g, v0, v1, C.byref(self.h)), "gx_sssp_split_create")

    def start(self, src):
        self.be.N.check(self.be.lib.gx_sssp_split_start(self.h, src, self.be._s()), "gx_sssp_split_start")

    def relax(self, pairs, count):
        self.be.N.check(self.be.lib.gx_sssp_split_relax(self.h, self.be._p(pairs), self.be._p(count), self.be._s()),
                        "gx_sssp_split_relax")

    def apply(self, pairs, counts, nranks, stride):
        self.be.N.check(self.be.lib.gx_sssp_split_apply(self.h, self.be._p(pairs), self.be._p(counts), nranks, stride,
                                                        self.be._s()), "gx_sssp_split_apply")

    def distances(self, out):
        self.be.N.check(self.be.lib.gx_sssp_split_distances(self.h, self.be._p(out), self.be._s()),
                        "gx_sssp_split_distances")

    def close(self):
        if self.h:
            self.be.lib.gx_sssp_split_free(self.h)
            self.h = C.c_void_p()


class _GpuCdlpPart:
    def __init__(self, be: GpuBackend, v0: int, v1: int):
        self.be = be
        self.h = C.c_void_p()
        be.N.check(be.lib.gx_cdlp_part_create(be.g, v0, v1, C.byref(self.h)), "gx_cdlp_part_create")

    def init(self, labels):
        self.be.N.check(self.be.lib.gx_cdlp_part_init(self.h, self.be._p(labels), self.be._s()), "gx_cdlp_part_init")

    def step(self, labels, nxt, changed):
        self.be.N.check(self.be.lib.gx_cdlp_part_step(self.h, self.be._p(labels), self.be._p(nxt),
                                                      self.be._p(changed), self.be._s()), "gx_cdlp_part_step")

    def close(self):
        if self.h:
            self.be.lib.gx_cdlp_part_free(self.h)
            self.h = C.c_void_p()


class _GpuLccPart:
    def __init__(self, be: GpuBackend):
        self.be = be
        self.h = C.c_void_p()
        be.N.check(be.lib.gx_lcc_part_create(be.g, C.byref(self.h)), "gx_lcc_part_create")

    def ranges(self, nranks: int) -> np.ndarray:
        r = np.zeros(nranks + 1, dtype=np.uint64)
        self.be.N.check(self.be.lib.gx_lcc_part_ranges(self.h, nranks, self.be.N.as_u64p(r)), "gx_lcc_part_ranges")
        return r

    def counts(self, v0, v1, tc):
        self.be.N.check(self.be.lib.gx_lcc_part_counts(self.h, v0, v1, self.be._p(tc), self.be._s()),
                        "gx_lcc_part_counts")

    def finish(self, tc, out):
        self.be.N.check(self.be.lib.gx_lcc_part_finish(self.h, self.be._p(tc), self.be._p(out), self.be._s()),
                        "gx_lcc_part_finish")

    def close(self):
        if self.h:
            self.be.lib.gx_lcc_part_free(self.h)
            self.h = C.c_void_p()


# -------------------------------------------------------------------------- drivers
@dataclass
class LocalRank:
    backend: object
    v0: int
    v1: int
    device: object
    rank: int = 0   # global rank (index into the ranges of all ranks)


def vertex_ranges(rowptr: np.ndarray, nranks: int) -> np.ndarray:
    """Contiguous vertex ranges with ~nnz/nranks stored entries each (uint64[nranks+1])."""
    return partition_rows(rowptr, nranks)


def _zeros(rank: LocalRank, n: int, dtype):
    import torch
    return torch.zeros(n, dtype=dtype, device=rank.device)


OP_SET, OP_MIN, OP_MAX = 0, 1, 2
# _exchange: "auto" (the smaller of words and dense), "sparse", "dense" (GX_EXCHANGE)
EXCHANGE = os.environ.get("GX_EXCHANGE", "auto")
# bytes each rank sent per exchange kind since the last reset (bench.py reports them)
STATS = {"rounds": 0, "word_rounds": 0, "word_bytes": 0, "dense_bytes": 0, "dense_only_bytes": 0}


def reset_stats():
    for k in STATS:
        STATS[k] = 0


class _Bufs:
    """Per-call scratch of the round loops: one set of exchange buffers per rank,
    allocated on first use and reused by every round of a bfs / wcc / cdlp call, so a round
    costs no allocation beyond a gathered-words buffer that grows by doubling."""

    def __init__(self):
        self.d = {}

    def get(self, key, rank: LocalRank, n: int, dtype, zero: bool = True):
        import torch
        t = self.d.get(key)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.zeros(max(n, 2 * t.numel() if t is not None else n), dtype=dtype, device=rank.device)
            self.d[key] = t
        elif zero:
            t[:n].zero_()
        return t[:n]


def _exchange(ranks: List[LocalRank], comm, arrs, olds, spans, elem: int, op: int, dense_bytes: int, dense,
              dsts=None, bufs: "_Bufs" = None) -> int:
    """Frontier-sized exchange: every rank's entries of arrs[k] over spans[k] = (v0, v1) that
    differ from olds[k] (None: from 0) leave as (v << 32 | value) words (gx_part_changes); the
    counts are all-gathered (the one host read), then the first max-count words of every rank,
    which every rank applies with `op` (gx_part_apply) to dsts[k] (default arrs[k]).  When
    those words would outweigh the dense collective (`dense_bytes` per rank, e.g. 2 n for an
    all-reduce of n bytes), `dense()` runs instead (EXCHANGE = "sparse" / "dense" forces one).
    Returns the number of changes over all ranks (0: nothing changed anywhere).  `bufs` (one
    per algorithm call) keeps the word, count and gathered buffers across rounds."""
    import torch
    nranks = getattr(comm, "world_size", None) or len(ranks)
    if bufs is None:
        bufs = _Bufs()
    # room for any rank's count: the all-gather sends the first max-count words of every rank
    # (written by gx_part_changes before they are read: no zeroing)
    words = [bufs.get(("w", k), r, max(1, a.numel()), torch.int64, zero=False)
             for k, (r, a) in enumerate(zip(ranks, arrs))]
    cnt = [bufs.get(("c", k), r, 1, torch.int64) for k, r in enumerate(ranks)]
    for r, a, b, (v0, v1), w, c in zip(ranks, arrs, olds, spans, words, cnt):
        r.backend.changes(a, b, v0, v1, elem, w, c)
    counts = [bufs.get(("n", k), r, nranks, torch.int64) for k, r in enumerate(ranks)]
    comm.all_gather(counts, cnt)
    cw = counts[0].cpu().numpy()   # identical on every rank
    m, tot = int(cw.max()), int(cw.sum())
    STATS["rounds"] += 1
    STATS["dense_only_bytes"] += dense_bytes   # what the dense collective alone would move
    if m == 0:
        return 0
    if EXCHANGE == "dense" or (EXCHANGE != "sparse" and 8 * m * nranks > dense_bytes):
        STATS["dense_bytes"] += dense_bytes
        dense()
        return tot
    STATS["word_rounds"] += 1
    STATS["word_bytes"] += 8 * m * nranks
    gathered = [bufs.get(("g", k), r, m * nranks, torch.int64, zero=False) for k, r in enumerate(ranks)]
    comm.all_gather(gathered, [w[:m] for w in words])
    for r, g, cs, a in zip(ranks, gathered, counts, dsts if dsts is not None else arrs):
        r.backend.apply(g, cs, nranks, m, a, elem, op)
    return tot


def bfs(ranks: List[LocalRank], comm, n: int, src: int):
    """Level-synchronous top-down BFS; returns rank 0's level tensor (int64, INT64_MAX =
    unreached).  A level's discoveries travel as vertex words while they are fewer than the
    dense all-reduce MAX of the n-byte `next` moves (_exchange)."""
    import torch
    level = [_zeros(r, n, torch.int64) for r in ranks]
    for r, lv in zip(ranks, level):
        r.backend.bfs_init(src, lv)
    nranks = getattr(comm, "world_size", None) or len(ranks)
    # dense form: the bitmaps all-gathered (n / 8 bytes from each rank), or, from 16 ranks on,
    # the all-reduce MAX of next (~2 n bytes)
    dense_bytes = min(2 * n, nranks * ((n + 31) // 32) * 4)
    cur = 0
    bufs = _Bufs()
    while True:
        nxt = [bufs.get(("next", k), r, n, torch.uint8) for k, r in enumerate(ranks)]
        for r, lv, nx in zip(ranks, level, nxt):
            r.backend.bfs_expand(r.v0, r.v1, lv, cur, nx)
        _exchange(ranks, comm, nxt, [None] * len(ranks), [(0, n)] * len(ranks), 1, OP_SET, dense_bytes,
                  lambda: _bfs_dense(ranks, comm, nxt, n, bufs), bufs=bufs)
        count = [bufs.get(("count", k), r, 1, torch.int64) for k, r in enumerate(ranks)]
        for r, lv, nx, c in zip(ranks, level, nxt, count):
            r.backend.bfs_commit(nx, lv, cur, c)
        if int(count[0].item()) == 0:   # identical on every rank (same inputs)
            break
        cur += 1
    return level[0]


def _bfs_dense(ranks: List[LocalRank], comm, nxt, n: int, bufs: "_Bufs" = None) -> None:
    """A level's discoveries exchanged densely: bit-packed and all-gathered (gx_part_pack_bits /
    gx_part_or_bits) while that is smaller than the all-reduce MAX of the n-byte `next`."""
    import torch
    nranks = getattr(comm, "world_size", None) or len(ranks)
    nw = (n + 31) // 32
    if nranks * nw * 4 >= 2 * n:
        comm.all_reduce(nxt, "max")
        return
    if bufs is None:
        bufs = _Bufs()
    bits = [bufs.get(("bits", k), r, nw, torch.int32, zero=False) for k, r in enumerate(ranks)]
    for r, nx, b in zip(ranks, nxt, bits):
        r.backend.pack_bits(nx, b)
    gathered = [bufs.get(("bitsg", k), r, nw * nranks, torch.int32, zero=False) for k, r in enumerate(ranks)]
    comm.all_gather(gathered, bits)
    for r, g, nx in zip(ranks, gathered, nxt):
        r.backend.or_bits(g, nranks, nx)


def wcc(ranks: List[LocalRank], comm, n: int):
    """Min-root hooking over owned rows + MIN exchange of the forest; returns parent (int32):
    the smallest vertex id of each component.  Every rank starts a round with the same forest,
    so only the entries its hooks changed travel (_exchange, applied with MIN); a round in which
    no rank changed anything is the fixed point (no separate flag collective)."""
    import torch
    parent = [_zeros(r, n, torch.int32) for r in ranks]
    for r, p in zip(ranks, parent):
        r.backend.wcc_init(p)
    bufs = _Bufs()
    while True:
        prev = [bufs.get(("prev", k), r, n, torch.int32, zero=False).copy_(p)
                for k, (r, p) in enumerate(zip(ranks, parent))]
        changed = [bufs.get(("changed", k), r, 1, torch.int32) for k, r in enumerate(ranks)]
        for r, p, c in zip(ranks, parent, changed):
            r.backend.wcc_hook(r.v0, r.v1, p, c)
        tot = _exchange(ranks, comm, parent, prev, [(0, n)] * len(ranks), 4, OP_MIN, 8 * n,
                        lambda: comm.all_reduce(parent, "min"), bufs=bufs)
        if tot == 0:
            break
        for r, p in zip(ranks, parent):
            r.backend.wcc_compress(p)
    return parent[0]


def sssp(ranks: List[LocalRank], comm, n: int, src: int):
    """Delta-stepping on the 1-D split (gx_sssp_split): each rank relaxes the edges into its
    owned vertices; per round the count words {pairs, done} are all-gathered (one host read),
    then the improved owned vertices as (vertex, fp64 bits) pairs, max-count words from every
    rank.  Returns the distances (float64, inf = unreached)."""
    import torch
    nranks = getattr(comm, "world_size", None) or len(ranks)
    parts = [r.backend.sssp_split(r.v0, r.v1) for r in ranks]
    try:
        # n pairs of room on every rank: the all-gather sends max-count pairs from each, which
        # may exceed what a small range could ever fill
        pairs = [_zeros(r, 2 * max(1, n), torch.int64) for r in ranks]
        count = [_zeros(r, 2, torch.int64) for r in ranks]
        counts = [_zeros(r, 2 * nranks, torch.int64) for r in ranks]
        for p in parts:
            p.start(src)
        while True:
            for p, pr, c in zip(parts, pairs, count):
                p.relax(pr, c)
            comm.all_gather(counts, count)
            cw = counts[0].cpu().numpy()   # identical on every rank
            done = cw[1::2]
            if done.any():
                # every rank takes the same decisions from replicated counts; a rank that stops
                # alone would leave the others' relaxations unapplied
                if not done.all():
                    raise RuntimeError(f"sssp: ranks disagree on termination (done words {done.tolist()})")
                break
            m = int(cw[0::2].max())
            if m:
                gathered = [_zeros(r, 2 * m * nranks, torch.int64) for r in ranks]
                comm.all_gather(gathered, [pr[:2 * m] for pr in pairs])
            else:
                gathered = pairs
            for p, g, cs in zip(parts, gathered, counts):
                p.apply(g, cs, nranks, m)
        out = _zeros(ranks[0], n, torch.float64)
        parts[0].distances(out)
        return out
    finally:
        for p in parts:
            p.close()


def cdlp(ranks: List[LocalRank], comm, n: int, iters: int, ranges: np.ndarray):
    """Synchronous label propagation; each rank updates its range, the owned slices are
    all-gathered.  `ranges` (uint64[nranks+1]) covers ALL ranks.  Returns labels (int32)."""
    import torch
    nranks = len(ranges) - 1
    sizes = [int(ranges[k + 1] - ranges[k]) for k in range(nranks)]
    chunk = max(1, max(sizes))
    parts = [r.backend.cdlp_part(r.v0, r.v1) for r in ranks]
    try:
        labels = [_zeros(r, n, torch.int32) for r in ranks]
        nxt = [_zeros(r, n, torch.int32) for r in ranks]
        for p, lb in zip(parts, labels):
            p.init(lb)
        bufs = _Bufs()
        for _ in range(iters):
            changed = [bufs.get(("changed", k), r, 1, torch.int32) for k, r in enumerate(ranks)]
            for p, lb, nx, c in zip(parts, labels, nxt, changed):
                p.step(lb, nx, c)

            def dense():
                send = [bufs.get(("send", k), r, chunk, torch.int32) for k, r in enumerate(ranks)]
                for r, nx, sd in zip(ranks, nxt, send):
                    sd[:r.v1 - r.v0].copy_(nx[r.v0:r.v1])
                gathered = [bufs.get(("sendg", k), r, chunk * nranks, torch.int32, zero=False)
                            for k, r in enumerate(ranks)]
                comm.all_gather(gathered, send)
                for g, lb in zip(gathered, labels):
                    lb.copy_(torch.cat([g[k * chunk:k * chunk + sizes[k]] for k in range(nranks)]))

            # the owned labels that changed, set into every rank's labels (_exchange); the
            # all-gather of the owned slices when more than half of them changed
            tot = _exchange(ranks, comm, nxt, labels, [(r.v0, r.v1) for r in ranks], 4, OP_SET, 4 * n, dense,
                            dsts=labels, bufs=bufs)
            if tot == 0:   # fixed point (LAGraph_cdlp.c:328-332)
                break
        return labels[0]
    finally:
        for p in parts:
            p.close()


def lcc(ranks: List[LocalRank], comm, n: int):
    """Triangle counts per owned orientation source + SUM exchange; returns LCC (float64).
    The ranks' vertex ranges are replaced by the work-balanced ones of gx_lcc_part_ranges."""
    import torch
    parts = [r.backend.lcc_part() for r in ranks]
    try:
        nranks = getattr(comm, "world_size", None) or len(ranks)
        rng = parts[0].ranges(nranks)   # identical on every rank (same graph, same estimate)
        tc = [_zeros(r, n, torch.int64) for r in ranks]
        for r, p, t in zip(ranks, parts, tc):
            p.counts(int(rng[r.rank]), int(rng[r.rank + 1]), t)
        comm.all_reduce(tc, "sum")
        out = [_zeros(r, n, torch.float64) for r in ranks]
        for p, t, o in zip(parts, tc, out):
            p.finish(t, o)
        return out[0]
    finally:
        for p in parts:
            p.close()
