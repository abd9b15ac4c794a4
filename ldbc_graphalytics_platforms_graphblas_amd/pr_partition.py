"""1-D row-partitioned PageRank across ranks (one process per GPU, torch.distributed/RCCL).

The pull matrix (A' for directed graphs, A itself for undirected ones) is cut into
contiguous row blocks balanced by stored entries.  Every rank keeps only its rows (with
global column ids, remapped once to the padded exchange layout by gx_pr_part_create) and a
full replica of the rank vector.  One iteration is:

    gx_pr_part_step   : pull SpMV over the local rows -> next local chunk (+ dangling slot)
    all_gather        : chunks of all ranks -> full vector        (RCCL over xGMI)

The exchange layout is `nranks` chunks of `chunk` doubles; rank k's rows sit at the start of
chunk k and its dangling-score sum in the chunk's last slot, so a single
all_gather_into_tensor carries both the vector and the dangling mass (no extra all-reduce).
Rows without out-edges are never gathered by anyone: when every rank's such rows come last
(hub-first order), only each rank's leading `live` rows go in its chunk
(gx_pr_part_create_live), and the exchanged vector shrinks by their share (29.5 % of SYN-7_5).
The reference has no distributed path ("Collective call sites: none"); this is
the exchange step the north star adds.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Union

import numpy as np

from .graphio import CSR


def relabel(csr: CSR, order: np.ndarray):
    """Relabel a CSR by `order` (new id -> old id): row order[i] becomes row i, every column
    is renamed, and every row is sorted by new column id (neighbouring lanes of a gather then
    often share an x cache line).  Returns (perm, CSR) with perm[old] = new."""
    n = csr.n
    deg = np.diff(csr.rowptr.astype(np.int64))
    perm = np.empty(n, dtype=np.int64)
    perm[order] = np.arange(n, dtype=np.int64)
    new_deg = deg[order]
    nrp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(new_deg, out=nrp[1:])
    idx = np.repeat(csr.rowptr.astype(np.int64)[order] - nrp[:-1], new_deg) + np.arange(int(nrp[-1]))
    nci = perm[csr.colidx.astype(np.int64)[idx]]
    rows = np.repeat(np.arange(n, dtype=np.int64), new_deg)
    if csr.vals is None:
        key = np.sort(rows * n + nci)
        nci = (key - rows * n).astype(np.uint64)
        vals = None
    else:
        o = np.argsort(rows * n + nci, kind="stable")
        nci = nci[o].astype(np.uint64)
        vals = np.ascontiguousarray(csr.vals[idx][o])
    return perm, CSR(n, nrp.astype(np.uint64), np.ascontiguousarray(nci), vals)


def hub_relabel(csr: CSR):
    """Hub-first vertex order (out-degree descending, ties by id) -- the layout gx_pagerank
    uses internally: the pull SpMV gathers x(u) once per out-edge of u, so the most gathered
    entries of x land in its first few MiB and stay resident in each XCD's L2.
    Returns (perm, relabelled CSR) with perm[old] = new."""
    deg = np.diff(csr.rowptr.astype(np.int64))
    return relabel(csr, np.argsort(-deg, kind="stable"))


def interleaved_relabel(csr: CSR, nparts: int):
    """The hub-first order dealt round-robin over `nparts` row blocks: part v owns hub-first
    vertices v, v + nparts, v + 2 nparts, ... as one contiguous id range, still hub-first
    inside it.  Every part gets n/nparts rows (+-1) and, dealing a degree-sorted list, about
    nnz/nparts entries (the parts differ by at most the largest degree), so the padded
    exchange layout of gx_pr_part (nparts chunks of max rows + 1) is ~n doubles long.
    Contiguous hub-first ranges balanced by entries instead give the low-degree tail part
    most of the rows: on SYN-7_5 the exchanged vector was 7.2 n at 8 parts, 13 n at 16.
    Returns (perm, relabelled CSR, bounds) with perm[old] = new and bounds[nparts + 1] the
    row boundaries of the parts."""
    n = csr.n
    deg = np.diff(csr.rowptr.astype(np.int64))
    hub = np.argsort(-deg, kind="stable")               # hub-first id -> old id
    deal = [hub[v::nparts] for v in range(nparts)]
    bounds = np.zeros(nparts + 1, dtype=np.uint64)
    bounds[1:] = np.cumsum([len(d) for d in deal])
    perm, out = relabel(csr, np.concatenate(deal) if n else hub)
    return perm, out, bounds


def _deal_blocks(work: np.ndarray, live: np.ndarray, nparts: int, owner: np.ndarray) -> None:
    """Blocks to parts, heaviest first: the upper half by work to the least loaded part (LPT);
    the lighter half (the sparse tail's row-heavy blocks) to the part with the fewest live rows
    among those it keeps within 1 % of the mean work, so the exchanged chunk (the largest live
    row count) shrinks too -- SYN-8_5 at 8 parts: 0.709 n -> 0.672 n doubles per iteration, work
    imbalance 1.001 -> 1.01 (pr_multi_blocks does the same)."""
    nb = len(work)
    if nb == 0:
        return
    order = np.argsort(-work, kind="stable")
    heavy = np.median(work)
    target = work.sum() / nparts
    load = np.zeros(nparts, dtype=np.float64)
    lv = np.zeros(nparts, dtype=np.int64)
    for b in order:
        if work[b] >= heavy:
            p = int(np.argmin(load))
        else:
            fit = [k for k in range(nparts) if load[k] + work[b] <= target * 1.01]
            p = min(fit, key=lambda k: (lv[k], k)) if fit else int(np.argmin(load))
        owner[b] = p
        load[p] += work[b]
        lv[p] += live[b]


def block_relabel(csr: CSR, nparts: int, rows_per_block: int = 16320, block_nnz: int = 32 << 20):
    """The single-GPU plan's sorted blocks dealt whole over `nparts` parts: the hub-first order
    cut greedily into blocks of at most `rows_per_block` rows and `block_nnz` entries (as
    pr_plan_sorted cuts a huge graph, gx_pr_sorted.hip), the blocks dealt heaviest first
    (_deal_blocks: work, then live rows), and each part's blocks kept in hub-first order as one
    contiguous id range.  Unlike interleaved_relabel, whose parts hold every nparts-th hub-first
    row (so a part's 16 Ki-row block spans nparts x as many hub positions and shares each x line
    with nparts x fewer entries), every part's blocks are the whole-graph plan's own: the same
    entries per gathered x line, 1/nparts of the blocks.  Rows without out-edges come last in
    each part (the hub-first tail's blocks are the last ones of every part that gets them), so
    live_rows holds.  Returns (perm, relabelled CSR, bounds) as interleaved_relabel."""
    n = csr.n
    deg = np.diff(csr.rowptr.astype(np.int64))
    hub = np.argsort(-deg, kind="stable")
    hdeg = deg[hub]
    pre = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(hdeg, out=pre[1:])
    starts = []
    r = 0
    while r < n:
        lim = min(n, r + rows_per_block)
        # the last row end within block_nnz of the block's start (at least one row)
        e = int(np.searchsorted(pre, pre[r] + block_nnz, side="right")) - 1
        e = max(r + 1, min(e, lim))
        starts.append(r)
        r = e
    starts.append(n)
    nb = len(starts) - 1
    st = np.asarray(starts, dtype=np.int64)
    # work of a block: entries + a row term (epilogue); live rows: rows with out-edges (exchanged)
    work = (pre[st[1:]] - pre[st[:-1]]) + np.diff(st)
    live = np.add.reduceat((hdeg > 0).astype(np.int64), st[:-1]) if nb else np.zeros(0, dtype=np.int64)
    owner = np.zeros(nb, dtype=np.int64)
    _deal_blocks(work, live, nparts, owner)
    parts = [[hub[starts[b]:starts[b + 1]] for b in range(nb) if owner[b] == p] for p in range(nparts)]
    deal = [np.concatenate(x) if x else np.zeros(0, dtype=np.int64) for x in parts]
    bounds = np.zeros(nparts + 1, dtype=np.uint64)
    bounds[1:] = np.cumsum([len(d) for d in deal])
    perm, out = relabel(csr, np.concatenate(deal) if n else hub)
    return perm, out, bounds


def partition_rows(rowptr: np.ndarray, nranks: int) -> np.ndarray:
    """Row boundaries [0 = b0 <= b1 <= ... <= b_nranks = n] with ~nnz/nranks entries each."""
    rp = np.asarray(rowptr, dtype=np.int64)
    n, nnz = len(rp) - 1, int(rp[-1])
    bounds = np.zeros(nranks + 1, dtype=np.uint64)
    for k in range(1, nranks):
        target = (nnz * k) // nranks
        r = int(np.searchsorted(rp, target, side="left"))
        bounds[k] = min(max(r, int(bounds[k - 1])), n)
    bounds[nranks] = n
    return bounds


def live_rows(csr: CSR, bounds: np.ndarray) -> Optional[np.ndarray]:
    """Per part k, the number of leading rows of [bounds[k], bounds[k+1]) with out-edges, if
    every part's rows without out-edges come after all its rows with them (hub-first orders:
    interleaved_relabel, hub_relabel + partition_rows); else None (every row exchanged)."""
    deg = np.diff(csr.rowptr.astype(np.int64))
    b = np.asarray(bounds, dtype=np.int64)
    out = np.zeros(len(b) - 1, dtype=np.uint64)
    for k in range(len(b) - 1):
        seg = deg[b[k]:b[k + 1]]
        live = int(np.count_nonzero(seg))
        if live and not (seg[:live] > 0).all():
            return None
        out[k] = live
    return out


@dataclass
class LocalRows:
    row_ranges: np.ndarray   # uint64[nranks+1]
    rank: int
    rowptr: np.ndarray       # uint64[rows+1], starting at 0
    colidx: np.ndarray       # uint64[nnz_local], global column ids
    outdeg: np.ndarray       # uint64[rows], out-degree of each local row's vertex
    live: Optional[np.ndarray] = None   # uint64[nranks]: live_rows() of the partition, or None

    @property
    def rows(self) -> int:
        return len(self.rowptr) - 1

    @property
    def nnz(self) -> int:
        return int(self.rowptr[-1])


def _slice_rows(csr: CSR, pull: CSR, bounds: np.ndarray, rank: int) -> LocalRows:
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    z0, z1 = int(pull.rowptr[r0]), int(pull.rowptr[r1])
    rp = (pull.rowptr[r0:r1 + 1] - np.uint64(z0)).astype(np.uint64)
    ci = np.ascontiguousarray(pull.colidx[z0:z1], dtype=np.uint64)
    outdeg = np.diff(csr.rowptr.astype(np.int64))[r0:r1].astype(np.uint64)
    return LocalRows(bounds, rank, np.ascontiguousarray(rp), ci, np.ascontiguousarray(outdeg),
                     live_rows(csr, bounds))


def slice_rows(csr: CSR, bounds: np.ndarray, part: int, pull: Optional[CSR] = None) -> LocalRows:
    """Rows [bounds[part], bounds[part + 1]) of the pull matrix (the graph itself when
    undirected), e.g. one part of interleaved_relabel."""
    return _slice_rows(csr, csr if pull is None else pull, bounds, part)


def local_rows(csr: CSR, directed: bool, nranks: int, rank: int, pull: Optional[CSR] = None) -> LocalRows:
    """Slice the pull matrix for `rank` (pull = A' for directed graphs)."""
    if pull is None:
        pull = csr.transpose() if directed else csr
    return _slice_rows(csr, pull, partition_rows(pull.rowptr, nranks), rank)


def local_pieces(csr: CSR, directed: bool, nranks: int, rank: int, pieces: int,
                 pull: Optional[CSR] = None) -> List[LocalRows]:
    """Pipelined layout: the pull matrix is cut into nranks * pieces ranges (balanced by
    entries) and rank k owns the virtual ranks p * nranks + k, p < pieces.  Piece p of every
    rank is then one contiguous slab of the exchanged vector (chunks p*nranks .. p*nranks +
    nranks - 1), so each piece is all-gathered on its own while the next one computes."""
    if pull is None:
        pull = csr.transpose() if directed else csr
    bounds = partition_rows(pull.rowptr, nranks * pieces)
    return [_slice_rows(csr, pull, bounds, p * nranks + rank) for p in range(pieces)]


class GpuStep:
    """gx_pr_part_* on one device; buffers are torch CUDA tensors (float64)."""

    def __init__(self, ctx, n_global: int, nranks: int, lr: LocalRows, damping: float):
        from . import _native as N
        self.N = N
        self.lib = N.lib()
        self.part = C.c_void_p()
        self._live = None if lr.live is None else np.ascontiguousarray(lr.live, dtype=np.uint64)
        N.check(self.lib.gx_pr_part_create_live(ctx.handle, n_global, nranks, lr.rank, N.as_u64p(lr.row_ranges),
                                                N.as_u64p(self._live) if self._live is not None else None,
                                                N.as_u64p(lr.rowptr),
                                                N.as_u64p(lr.colidx) if lr.nnz else None,
                                                N.as_u64p(lr.outdeg) if lr.rows else
                                                N.as_u64p(np.zeros(1, np.uint64)),
                                                damping, C.byref(self.part)), "gx_pr_part_create_live")
        ch = C.c_uint64(0)
        N.check(self.lib.gx_pr_part_chunk(self.part, C.byref(ch)), "gx_pr_part_chunk")
        self.chunk = ch.value

    def init(self, x_local, stream) -> None:
        self.N.check(self.lib.gx_pr_part_init(self.part, C.c_void_p(x_local.data_ptr()), C.c_void_p(stream)),
                     "gx_pr_part_init")

    def step(self, x_full, x_local, rank_out, stream) -> None:
        ro = C.c_void_p(rank_out.data_ptr()) if rank_out is not None else None
        self.N.check(self.lib.gx_pr_part_step(self.part, C.c_void_p(x_full.data_ptr()),
                                              C.c_void_p(x_local.data_ptr()), ro, C.c_void_p(stream)),
                     "gx_pr_part_step")

    def close(self) -> None:
        if self.part:
            self.lib.gx_pr_part_free(self.part)
            self.part = C.c_void_p()


class PartitionedPageRank:
    """Runs `iters` PageRank iterations with one exchange per iteration and piece.

    `stepper` (or a list of them, one per piece: see local_pieces) provides
    init(x_local, stream), step(x_full, x_local, rank_out, stream) and `chunk`;
    `all_gather(out, inp)` is torch.distributed.all_gather_into_tensor for nranks > 1 and may
    return an async work handle (async_op=True): piece p's gather then runs while piece p+1
    computes, and all handles are waited for before the next iteration reads the vector.
    The gathered vector is double-buffered so that a gather never overwrites values a later
    piece of the same iteration still reads.  With one rank and one piece the two buffers
    simply swap roles.
    """

    def __init__(self, stepper, nranks: int, rows_local: Union[int, Sequence[int]], device,
                 all_gather: Optional[Callable] = None, stream_handle: Callable[[], int] = lambda: 0):
        import torch
        self.steps = list(stepper) if isinstance(stepper, (list, tuple)) else [stepper]
        rows = list(rows_local) if isinstance(rows_local, (list, tuple)) else [rows_local]
        if len(rows) != len(self.steps):
            raise ValueError("one rows_local per piece")
        self.gathered = all_gather is not None   # else one rank, one piece: buffers swap
        if not self.gathered and (nranks != 1 or len(self.steps) != 1):
            raise ValueError("several ranks or pieces need an all_gather")
        self.nranks = nranks
        self.rows = rows
        self.all_gather = all_gather
        self.stream = stream_handle
        ch = self.steps[0].chunk
        self.chunk = ch
        npieces = len(self.steps)
        self.x_local = [torch.zeros(ch, dtype=torch.float64, device=device) for _ in range(npieces)]
        self.x_read = torch.zeros(ch * nranks * npieces, dtype=torch.float64, device=device)
        self.x_write = torch.zeros_like(self.x_read) if self.gathered else None
        self.rank_outs = [torch.zeros(max(r, 1), dtype=torch.float64, device=device) for r in rows]

    @property
    def rank_out(self):
        """Scores of the (single) piece; see rank_outs for several pieces."""
        return self.rank_outs[0]

    def _piece(self, x, p):
        span = self.chunk * self.nranks
        return x[p * span:(p + 1) * span]

    def _gather_all(self, target):
        handles = [self.all_gather(self._piece(target, p), self.x_local[p]) for p in range(len(self.steps))]
        for h in handles:
            if h is not None:
                h.wait()

    def run(self, iters: int):
        npieces = len(self.steps)
        for p in range(npieces):
            self.steps[p].init(self.x_local[p], self.stream())
        if not self.gathered:
            self.x_local[0], self.x_read = self.x_read, self.x_local[0]
        else:
            self._gather_all(self.x_read)
        for it in range(iters):
            last = it == iters - 1
            handles = []
            for p in range(npieces):
                self.steps[p].step(self.x_read, self.x_local[p], self.rank_outs[p] if last else None, self.stream())
                if not last and self.gathered:
                    handles.append(self.all_gather(self._piece(self.x_write, p), self.x_local[p]))
            if last:
                break
            if not self.gathered:
                self.x_local[0], self.x_read = self.x_read, self.x_local[0]
            else:
                for h in handles:
                    if h is not None:
                        h.wait()
                self.x_read, self.x_write = self.x_write, self.x_read
        return self.rank_outs[0][:self.rows[0]] if npieces == 1 else \
            [o[:r] for o, r in zip(self.rank_outs, self.rows)]


class Comm:
    """RCCL communicator inside libgx (gx_comm_*), bootstrapped over torch.distributed.

    Rank 0 creates the RCCL id (gx_comm_unique_id) and `share_id(bytes) -> bytes` hands it
    to every rank (bench.py: torch.distributed.broadcast_object_list); the rank numbering is
    the partition's.  ncclCommInitRank is collective: every rank constructs its Comm
    together."""

    def __init__(self, ctx, nranks: int, rank: int, share_id: Callable[[bytes], bytes]):
        from . import _native as N
        self.N = N
        lib = N.lib()
        uid = C.create_string_buffer(128)
        mine = b""
        if rank == 0 and lib.gx_comm_unique_id(uid) == 0:
            mine = uid.raw
        got = share_id(mine)   # every rank takes part, also when rank 0 has no id
        if len(got) != 128:
            raise RuntimeError("no RCCL unique id from rank 0: " + lib.gx_last_error().decode(errors="replace"))
        uid = C.create_string_buffer(got, 128)
        self.handle = C.c_void_p()
        N.check(lib.gx_comm_create(ctx.handle, nranks, rank, uid, C.byref(self.handle)), "gx_comm_create")
        self.nranks, self.rank = nranks, rank

    def close(self) -> None:
        if self.handle:
            self.N.lib().gx_comm_free(self.handle)
            self.handle = C.c_void_p()


class DevicePageRank:
    """The whole partitioned PageRank enqueued by libgx (gx_pr_dist_*): every iteration's
    SpMV per piece and every ncclAllGather in one C call, optionally captured once into a
    hipGraph and replayed (`use_graph`).  Same partition, pieces and results as
    PartitionedPageRank, without a host round trip per iteration.

    `steppers` are the GpuStep pieces of this rank (piece p = virtual rank p*nranks+rank);
    `comm` is a Comm, or None for one rank.

    `p2p = (nranks, rank, share_all)` selects the one-shot peer-to-peer exchange instead
    (gx_pr_dist_create_p2p; no RCCL, `comm` must be None): `share_all(bytes) -> list of
    bytes` hands every rank's IPC handle to every rank in rank order (bench.py:
    torch.distributed.all_gather_object); every rank constructs its runner together."""

    def __init__(self, steppers: Sequence["GpuStep"], comm: Optional[Comm], use_graph: bool = True,
                 p2p: Optional[tuple] = None):
        from . import _native as N
        self.N = N
        self.steps = list(steppers)
        lib = N.lib()
        arr = (C.c_void_p * len(self.steps))(*[s.part.value for s in self.steps])
        self.handle = C.c_void_p()
        if p2p is None:
            N.check(lib.gx_pr_dist_create(comm.handle if comm is not None else None, arr, len(self.steps),
                                          C.byref(self.handle)), "gx_pr_dist_create")
        else:
            if comm is not None:
                raise ValueError("the peer-to-peer exchange takes no RCCL communicator")
            nranks, rank, share_all = p2p
            nb = 192   # GX_P2P_HANDLE_BYTES
            mine = C.create_string_buffer(nb)
            rc = lib.gx_pr_dist_create_p2p(nranks, rank, arr, len(self.steps), mine, C.byref(self.handle))
            err = lib.gx_last_error().decode(errors="replace") if rc else ""
            got = share_all(mine.raw if rc == 0 else b"")   # every rank takes part, also after a failure
            if rc:
                raise RuntimeError(f"gx_pr_dist_create_p2p: {err}")
            if len(got) != nranks or any(len(g) != nb for g in got):
                self.close()
                raise RuntimeError("gx_pr_dist_create_p2p: a rank has no peer-to-peer handle")
            allh = C.create_string_buffer(b"".join(got), nb * nranks)
            rc = lib.gx_pr_dist_p2p_attach(self.handle, allh)
            if rc:
                msg = lib.gx_last_error().decode(errors="replace")
                self.close()
                raise RuntimeError(f"gx_pr_dist_p2p_attach: {msg}")
        self.use_graph = use_graph

    def run(self, iters: int, stream: int = 0) -> None:
        """Asynchronous on `stream` (a hipStream_t handle; 0 = the context stream)."""
        self.N.check(self.N.lib().gx_pr_dist_run(self.handle, iters, int(self.use_graph),
                                                 C.c_void_p(stream) if stream else None), "gx_pr_dist_run")

    def scores(self, rows: Sequence[int]) -> List[np.ndarray]:
        """Per piece, the scores of its rows (waits for the last run)."""
        out = []
        for p, r in enumerate(rows):
            a = np.zeros(max(r, 1), dtype=np.float64)
            self.N.check(self.N.lib().gx_pr_dist_scores(self.handle, p, self.N.as_dp(a)), "gx_pr_dist_scores")
            out.append(a[:r])
        return out

    def close(self) -> None:
        if self.handle:
            self.N.lib().gx_pr_dist_free(self.handle)
            self.handle = C.c_void_p()
