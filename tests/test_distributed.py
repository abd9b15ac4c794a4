"""Row-partitioned PageRank across ranks (the bench's N > 1 path).

CPU (gloo, world_size 2): the same orchestration bench.py runs over RCCL --
partition_rows / local_rows / hub_relabel / PartitionedPageRank with one
all_gather_into_tensor per iteration -- driven by a numpy stepper that restates the
gx_pr_part_* contract (padded chunk layout, dangling slot), checked against the oracle.
GPU: gx_pr_part_* itself with two ranks simulated on one device.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sys.path)
from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import (PartitionedPageRank, hub_relabel,
                                                                    block_relabel, interleaved_relabel, live_rows,
                                                                    local_pieces,
                                                                    local_rows, partition_rows, slice_rows)
from oracle import oracle as O


class CpuStep:
    """numpy restatement of gx_pr_part_create/init/step (test-only stand-in for the GPU)."""

    def __init__(self, n_global, nranks, lr, damping):
        rr = lr.row_ranges.astype(np.int64)
        live = (rr[1:] - rr[:-1]) if lr.live is None else lr.live.astype(np.int64)   # gx_pr_part_create_live
        self.chunk = int((live.max() + 1 + 31) // 32 * 32)
        self.live = int(live[lr.rank])
        owner = np.searchsorted(rr, lr.colidx.astype(np.int64), side="right") - 1
        li = lr.colidx.astype(np.int64) - rr[owner]
        assert (li < live[owner]).all(), "a column past its owner's live rows"
        self.cols = owner * self.chunk + li
        self.rp = lr.rowptr.astype(np.int64)
        self.deg = lr.outdeg.astype(np.int64)
        self.rows = lr.rows
        self.n = n_global
        self.nranks = nranks
        self.d = damping

    def init(self, x_local, stream):
        inv_n = 1.0 / self.n
        x = np.where(self.deg > 0, inv_n / (self.deg / self.d), inv_n)
        x_local[:self.live] = torch.from_numpy(x[:self.live])
        x_local[self.chunk - 1] = float(np.sum(np.where(self.deg == 0, inv_n, 0.0)))

    def step(self, x_full, x_local, rank_out, stream):
        xf = x_full.numpy()
        dsum = sum(xf[k * self.chunk + self.chunk - 1] for k in range(self.nranks))
        tele = (1.0 - self.d) / self.n + self.d / self.n * dsum
        s = np.add.reduceat(np.append(xf[self.cols], 0.0), self.rp[:-1]) if len(self.cols) else np.zeros(self.rows)
        s = np.where(np.diff(self.rp) > 0, s, 0.0)
        r = tele + s
        x_local[:self.live] = torch.from_numpy(np.where(self.deg > 0, r / (self.deg / self.d), r)[:self.live])
        x_local[self.chunk - 1] = float(np.sum(np.where(self.deg == 0, r, 0.0)))
        if rank_out is not None:
            rank_out[:self.rows] = torch.from_numpy(r)


def _gloo_gather(out, inp):
    parts = list(out.chunk(dist.get_world_size()))
    dist.all_gather(parts, inp)
    if parts[0].data_ptr() != out.data_ptr():
        out.copy_(torch.cat(parts))


def _gloo_gather_async(out, inp):
    """The bench's async form: the gather of piece p runs while piece p+1 computes."""
    return dist.all_gather(list(out.chunk(dist.get_world_size())), inp, async_op=True)


def _worker(rank, world, port, q, pieces=1, layout="ranges"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        csr = rmat(11, 8, 5)
        perm, hub = hub_relabel(csr)
        if layout in ("interleave", "blocks"):   # bench.py's default layout, or whole plan blocks
            perm, hub, bounds = (interleaved_relabel(csr, world * pieces) if layout == "interleave"
                                 else block_relabel(csr, world * pieces, rows_per_block=96, block_nnz=2048))
            lrs = [slice_rows(hub, bounds, p * world + rank) for p in range(pieces)]
            pr = PartitionedPageRank([CpuStep(csr.n, world * pieces, lr, 0.85) for lr in lrs], world,
                                     [lr.rows for lr in lrs], "cpu", all_gather=_gloo_gather_async)
            out = pr.run(7)
            out = out if pieces > 1 else [out]
            mine = [(lr.rank, o.numpy().copy()) for lr, o in zip(lrs, out)]
        elif pieces == 1:
            lr = local_rows(hub, directed=False, nranks=world, rank=rank)
            pr = PartitionedPageRank(CpuStep(csr.n, world, lr, 0.85), world, lr.rows, "cpu", all_gather=_gloo_gather)
            mine = [(rank, pr.run(7).numpy().copy())]
        else:
            lrs = local_pieces(hub, False, world, rank, pieces)
            pr = PartitionedPageRank([CpuStep(csr.n, world * pieces, lr, 0.85) for lr in lrs], world,
                                     [lr.rows for lr in lrs], "cpu", all_gather=_gloo_gather_async)
            mine = [(lr.rank, o.numpy().copy()) for lr, o in zip(lrs, pr.run(7))]
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        if rank == 0:
            ordered = sorted((v for part in parts for v in part), key=lambda t: t[0])
            q.put(np.concatenate([a for _, a in ordered])[perm])
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partition_rows_balanced():
    csr = rmat(12, 16, 9)
    rp = csr.rowptr.astype(np.int64)
    for k in (1, 2, 3, 8):
        b = partition_rows(rp, k).astype(np.int64)
        assert b[0] == 0 and b[-1] == csr.n and (np.diff(b) >= 0).all()
        loads = rp[b[1:]] - rp[b[:-1]]
        assert loads.sum() == csr.nnz
        assert loads.max() <= csr.nnz / k + np.diff(rp).max() + 1


def test_interleaved_relabel_balances_rows_and_entries():
    """Dealing the hub-first order round-robin: equal row counts (+-1), entries within the
    largest degree of each other, ~n exchanged doubles, and the same PageRank."""
    csr = rmat(12, 16, 9)
    maxdeg = int(np.diff(csr.rowptr.astype(np.int64)).max())
    for k in (1, 2, 3, 8, 16):
        perm, g, b = interleaved_relabel(csr, k)
        b = b.astype(np.int64)
        assert b[0] == 0 and b[-1] == csr.n
        rows = np.diff(b)
        assert rows.max() - rows.min() <= 1
        rp = g.rowptr.astype(np.int64)
        loads = rp[b[1:]] - rp[b[:-1]]
        assert loads.sum() == csr.nnz and loads.max() - loads.min() <= maxdeg
        np.testing.assert_allclose(O.pagerank(csr, False, 0.85, 5), O.pagerank(g, False, 0.85, 5)[perm], rtol=1e-12)
    # the contiguous ranges of the hub-first order pad the exchange far beyond n
    _, hub = hub_relabel(csr)
    ranges = np.diff(partition_rows(hub.rowptr, 8).astype(np.int64))
    assert 8 * (ranges.max() + 1) > 3 * csr.n


def test_block_relabel_deals_whole_blocks():
    """block_relabel: every part's rows are whole blocks of the hub-first order (at most
    rows_per_block rows and block_nnz entries each, a longer row alone), entries balanced within
    the largest block, rows without out-edges last in every part, the relabelling isomorphic."""
    for undirected, k in ((True, 2), (True, 8), (False, 3)):
        csr = rmat(12, 8, 17, undirected=undirected)
        deg = np.diff(csr.rowptr.astype(np.int64))
        perm, g, b = block_relabel(csr, k, rows_per_block=200, block_nnz=4096)
        b = b.astype(np.int64)
        assert b[0] == 0 and b[-1] == csr.n and (np.diff(b) >= 0).all()
        ent = np.array([int(g.rowptr[b[i + 1]]) - int(g.rowptr[b[i]]) for i in range(k)])
        assert ent.sum() == csr.nnz
        # the largest block bounds the imbalance (LPT over entries + rows)
        gdeg = np.diff(g.rowptr.astype(np.int64))
        assert ent.max() - ent.min() <= max(4096, int(gdeg.max())) + 200
        assert live_rows(g, b) is not None
        # isomorphic: row perm[v] of g is row v of csr with renamed columns
        for v in (0, 1, int(np.argmax(deg)), csr.n - 1):
            a = np.sort(perm[csr.colidx[csr.rowptr[v]:csr.rowptr[v + 1]].astype(np.int64)])
            r = perm[v]
            assert np.array_equal(np.sort(g.colidx[g.rowptr[r]:g.rowptr[r + 1]].astype(np.int64)), a)


def test_live_rows_prefix_and_exchange_size():
    """Hub-first layouts keep every part's rows without out-edges last, so only the leading
    live rows are exchanged: the padded exchange is ~(vertices with out-edges) doubles."""
    csr = rmat(12, 16, 9)
    deg = np.diff(csr.rowptr.astype(np.int64))
    has_out = int(np.count_nonzero(deg))
    assert has_out < csr.n                        # R-MAT leaves isolated vertices
    for k in (1, 2, 8):
        perm, g, b = interleaved_relabel(csr, k)
        live = live_rows(g, b)
        assert live is not None and int(live.sum()) == has_out
        gdeg = np.diff(g.rowptr.astype(np.int64))
        b = b.astype(np.int64)
        for j in range(k):
            seg = gdeg[b[j]:b[j + 1]]
            assert (seg[:int(live[j])] > 0).all() and (seg[int(live[j]):] == 0).all()
        chunk = (int(live.max()) + 1 + 31) // 32 * 32
        assert k * chunk <= has_out + 33 * k          # vs ~n with every row exchanged
        _, hub = hub_relabel(csr)
        assert live_rows(hub, partition_rows(hub.rowptr, k)) is not None
    # an order that interleaves dangling rows with live ones has no live prefix
    order = np.argsort(deg, kind="stable")[::-1].copy()
    order[[0, -1]] = order[[-1, 0]]
    from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import relabel
    _, bad = relabel(csr, order)
    assert live_rows(bad, np.array([0, csr.n], dtype=np.uint64)) is None


def test_hub_relabel_is_isomorphic():
    csr = rmat(10, 8, 2)
    perm, hub = hub_relabel(csr)
    deg_new = np.diff(hub.rowptr.astype(np.int64))
    assert (np.diff(deg_new) <= 0).all()                    # hub-first
    for v in range(0, csr.n, 97):
        old = np.sort(perm[csr.colidx[csr.rowptr[v]:csr.rowptr[v + 1]].astype(np.int64)])
        row = hub.colidx[hub.rowptr[perm[v]]:hub.rowptr[perm[v] + 1]].astype(np.int64)
        assert (np.diff(row) > 0).all()                     # rows sorted
        assert (old == row).all()
    # PageRank is invariant under relabelling
    a = O.pagerank(csr, False, 0.85, 5)
    b = O.pagerank(hub, False, 0.85, 5)[perm]
    np.testing.assert_allclose(a, b, rtol=1e-12)


@pytest.mark.parametrize("pieces,layout", [(1, "ranges"), (2, "ranges"), (1, "interleave"), (2, "interleave"),
                                           (1, "blocks"), (2, "blocks")])
def test_gloo_world2_matches_oracle(pieces, layout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, pieces, layout)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    csr = rmat(11, 8, 5)
    np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, 7), rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [1, 2, 3])
@pytest.mark.parametrize("live", [True, False])
def test_gpu_partition_api_simulated_ranks(nranks, live):
    """gx_pr_part_* with `nranks` parts on one device; the exchange is a device concat.
    live: only the rows with out-edges are exchanged (gx_pr_part_create_live); else all."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import GpuStep
    csr = rmat(13, 16, 11)
    perm, hub = hub_relabel(csr)
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    steps, lrs = [], []
    for r in range(nranks):
        lr = local_rows(hub, directed=False, nranks=nranks, rank=r)
        if not live:
            lr.live = None
        lrs.append(lr)
        steps.append(GpuStep(ctx, csr.n, nranks, lr, 0.85))
    chunk = steps[0].chunk
    xl = [torch.zeros(chunk, dtype=torch.float64, device=dev) for _ in range(nranks)]
    xf = torch.zeros(chunk * nranks, dtype=torch.float64, device=dev)
    ro = [torch.zeros(max(lr.rows, 1), dtype=torch.float64, device=dev) for lr in lrs]
    iters = 6
    for r in range(nranks):
        steps[r].init(xl[r], 0)
    torch.cuda.synchronize()
    xf.copy_(torch.cat(xl))
    for it in range(iters):
        for r in range(nranks):
            steps[r].step(xf, xl[r], ro[r] if it == iters - 1 else None, 0)
        torch.cuda.synchronize()
        xf.copy_(torch.cat(xl))
    got = np.concatenate([ro[r][:lrs[r].rows].cpu().numpy() for r in range(nranks)])[perm]
    for s in steps:
        s.close()
    ctx.close()
    np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, iters), rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("pieces", [2, 8])
@pytest.mark.parametrize("combine", ["0", "1"])
def test_gpu_block_partition_pieces(pieces, combine, monkeypatch):
    """The block partition (bench.py GX_PR_PARTITION=blocks): the whole-graph plan's blocks
    dealt whole over `pieces` virtual ranks, each planned as a huge graph (GX_PR_HUGE=1), run by
    the device-driven runner with device copies; against the oracle."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import DevicePageRank, GpuStep
    monkeypatch.setenv("GX_PR_HUGE", "1")
    monkeypatch.setenv("GX_PR_COMBINE", combine)
    csr = rmat(14, 16, 12)
    perm, hub, bounds = block_relabel(csr, pieces, rows_per_block=1024, block_nnz=65536)
    ctx = Context(0)
    lrs = [slice_rows(hub, bounds, p) for p in range(pieces)]
    steps = [GpuStep(ctx, csr.n, pieces, lr, 0.85) for lr in lrs]
    dpr = DevicePageRank(steps, None, use_graph=True)
    dpr.run(10, 0)
    got = np.concatenate(dpr.scores([lr.rows for lr in lrs]))[perm]
    dpr.close()
    for s in steps:
        s.close()
    ctx.close()
    np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, 10), rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("pieces", [1, 2, 3])
@pytest.mark.parametrize("use_graph", [False, True])
@pytest.mark.parametrize("with_comm", [False, True])
def test_gpu_device_driven_pagerank(pieces, use_graph, with_comm):
    """gx_pr_dist_*: the whole run enqueued by libgx (optionally one replayed hipGraph), one
    rank cut into `pieces` virtual ranks; exchanged by device copies (no comm) or by
    ncclAllGather on a size-1 RCCL communicator.  Run twice to exercise the graph replay."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import Comm, DevicePageRank, GpuStep
    csr = rmat(13, 16, 11)
    perm, hub, bounds = interleaved_relabel(csr, pieces)
    ctx = Context(0)
    lrs = [slice_rows(hub, bounds, p) for p in range(pieces)]
    steps = [GpuStep(ctx, csr.n, pieces, lr, 0.85) for lr in lrs]
    comm = Comm(ctx, 1, 0, lambda uid: uid) if with_comm else None
    dpr = DevicePageRank(steps, comm, use_graph=use_graph)
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    want = O.pagerank(csr, False, 0.85, 6)
    for _ in range(2):
        dpr.run(6, stream.cuda_stream)
        got = np.concatenate(dpr.scores([lr.rows for lr in lrs]))[perm]
        np.testing.assert_allclose(got, want, rtol=1e-12)
    dpr.run(4, stream.cuda_stream)   # a different iteration count re-captures
    got = np.concatenate(dpr.scores([lr.rows for lr in lrs]))[perm]
    np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, 4), rtol=1e-12)
    dpr.close()
    if comm is not None:
        comm.close()
    for s in steps:
        s.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pieces", [1, 3])
@pytest.mark.parametrize("use_graph", [False, True])
@pytest.mark.parametrize("blocks", [None, "1"])
def test_gpu_p2p_exchange_one_rank(pieces, use_graph, blocks, monkeypatch):
    """gx_pr_dist_create_p2p with one rank: the put / flag / wait protocol writing into this
    rank's own vector (pieces exchanged by the peer-to-peer kernels), replayed and re-captured;
    GX_P2P_BLOCKS=1: one put workgroup per peer (the copy loop and the last-ticket signal)."""
    if blocks:
        monkeypatch.setenv("GX_P2P_BLOCKS", blocks)
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import DevicePageRank, GpuStep
    csr = rmat(13, 16, 11)
    perm, hub, bounds = interleaved_relabel(csr, pieces)
    ctx = Context(0)
    lrs = [slice_rows(hub, bounds, p) for p in range(pieces)]
    steps = [GpuStep(ctx, csr.n, pieces, lr, 0.85) for lr in lrs]
    dpr = DevicePageRank(steps, None, use_graph=use_graph, p2p=(1, 0, lambda h: [h]))
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    for iters in (6, 6, 4):
        dpr.run(iters, stream.cuda_stream)
        got = np.concatenate(dpr.scores([lr.rows for lr in lrs]))[perm]
        np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, iters), rtol=1e-12)
    dpr.close()
    for s in steps:
        s.close()
    ctx.close()


def _p2p_worker(rank, world, port, q, pieces, own_device=False):
    """One rank of the peer-to-peer exchange; both ranks share GPU 0 (IPC between two
    processes on one device), or rank r runs on GPU r (own_device: puts over xGMI into the
    peer's memory); the handles travel over gloo."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
        from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import DevicePageRank, GpuStep
        dev = rank if own_device else 0
        torch.cuda.set_device(dev)
        csr = rmat(12, 16, 7)
        perm, hub, bounds = interleaved_relabel(csr, world * pieces)
        lrs = [slice_rows(hub, bounds, p * world + rank) for p in range(pieces)]
        ctx = Context(dev)
        steps = [GpuStep(ctx, csr.n, world * pieces, lr, 0.85) for lr in lrs]

        def share_all(h):
            box = [None] * world
            dist.all_gather_object(box, h)
            return box
        dpr = DevicePageRank(steps, None, use_graph=True, p2p=(world, rank, share_all))
        stream = torch.cuda.Stream(torch.device("cuda", dev))
        results = []
        for iters in (6, 6, 4):   # replayed, then re-captured
            dpr.run(iters, stream.cuda_stream)
            mine = [(lr.rank, a) for lr, a in zip(lrs, dpr.scores([lr.rows for lr in lrs]))]
            parts = [None] * world
            dist.all_gather_object(parts, mine)
            if rank == 0:
                ordered = sorted((v for part in parts for v in part), key=lambda t: t[0])
                results.append((iters, np.concatenate([a for _, a in ordered])[perm]))
        dist.barrier()   # no rank unmaps a vector a peer still writes
        dpr.close()
        for s in steps:
            s.close()
        ctx.close()
        if rank == 0:
            q.put(results)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("pieces", [1, 2])
def test_gpu_p2p_exchange_world2_one_device(pieces):
    """Two processes, the peer-to-peer exchange between them (IPC-mapped vectors and flags on
    one device), against the oracle over three runs."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_p2p_worker, args=(r, 2, port, q, pieces)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    csr = rmat(12, 16, 7)
    for iters, got in results:
        np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, iters), rtol=1e-12)


@pytest.mark.gpu
def test_gpu_p2p_exchange_world2_two_devices():
    """The peer-to-peer exchange across devices: rank r on GPU r, the puts cross
    xGMI into the peer's vectors and flags.  Skipped where fewer than two GPUs are visible."""
    from ldbc_graphalytics_platforms_graphblas_amd import device_count
    if device_count() < 2:
        pytest.skip("needs two GPUs")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_p2p_worker, args=(r, 2, port, q, 1, True)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    csr = rmat(12, 16, 7)
    for iters, got in results:
        np.testing.assert_allclose(got, O.pagerank(csr, False, 0.85, iters), rtol=1e-12)


def test_p2p_runner_rejects_bad_arguments():
    """gx_pr_dist_create_p2p / _attach argument checks, before any device work."""
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    import ctypes as C
    lib = N.lib()
    h = C.c_void_p()
    buf = C.create_string_buffer(192)
    assert lib.gx_pr_dist_create_p2p(2, 2, None, 1, buf, C.byref(h)) != 0     # rank >= nranks
    assert lib.gx_pr_dist_create_p2p(65, 0, None, 1, buf, C.byref(h)) != 0    # > 64 ranks
    assert lib.gx_pr_dist_create_p2p(2, 0, None, 1, None, C.byref(h)) != 0    # no handle buffer
    assert lib.gx_pr_dist_p2p_attach(None, buf) != 0


def test_device_runner_rejects_mismatched_pieces():
    """Piece p must be virtual rank p * nranks + rank: checked before any device work."""
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    import ctypes as C
    h = C.c_void_p()
    rc = N.lib().gx_pr_dist_create(None, None, 1, C.byref(h))
    assert rc != 0


def test_gx_pr_partition_matches_interleaved_relabel():
    """The host partition of gx_pagerank_multi (libgx, C++) deals the hub-first order exactly
    as pr_partition.interleaved_relabel does (no GPU needed): same vertex per local row, same
    row counts and live prefixes."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd.pr_partition import live_rows
    for undirected in (True, False):
        csr = rmat(11, 6, 13, undirected=undirected)
        rp = np.ascontiguousarray(csr.rowptr, dtype=np.uint64)
        for nparts in (1, 2, 3, 8):
            order = np.zeros(csr.n, dtype=np.uint32)
            rows = np.zeros(nparts, dtype=np.uint64)
            live = np.zeros(nparts, dtype=np.uint64)
            N.check(N.lib().gx_pr_partition(csr.n, N.as_u64p(rp), nparts,
                                            order.ctypes.data_as(C.POINTER(C.c_uint32)), N.as_u64p(rows),
                                            N.as_u64p(live)), "gx_pr_partition")
            perm, hub, bounds = interleaved_relabel(csr, nparts)
            np.testing.assert_array_equal(rows, np.diff(bounds.astype(np.int64)))
            np.testing.assert_array_equal(live, live_rows(hub, bounds))
            # the vertex of local row j of part k sits at position k + j * nparts
            for k in range(nparts):
                mine = order[k::nparts].astype(np.int64)
                np.testing.assert_array_equal(perm[mine], np.arange(int(bounds[k]), int(bounds[k + 1])))


@pytest.mark.gpu
@pytest.mark.parametrize("undirected", [True, False])
def test_gx_pagerank_multi_one_device(undirected):
    """gx_pagerank_multi on one device (a size-1 in-process RCCL clique) against the oracle."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    from oracle import oracle as O
    ctx = Context(0)
    try:
        for scale, ef in ((10, 8), (14, 16)):
            csr = rmat(scale, ef, 5 + scale, undirected=undirected)
            out = np.zeros(csr.n)
            arr = (C.c_void_p * 1)(ctx.handle.value)
            s = csr.as_c()
            N.check(N.lib().gx_pagerank_multi(arr, 1, C.byref(s), int(not undirected), 0.85, 10, N.as_dp(out)),
                    "gx_pagerank_multi")
            np.testing.assert_allclose(out, O.pagerank(csr, not undirected, 0.85, 10), rtol=1e-12, atol=0)
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("undirected", [True, False])
def test_gx_sssp_multi_one_device(undirected):
    """gx_sssp_multi (bin/exe/sssp's GX_NGPUS path) on one device: the full exchange protocol
    over a size-1 in-process RCCL clique, bit-exact against the oracle and gx_sssp."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
    from oracle import oracle as O
    ctx = A.Context(0)
    try:
        for scale, ef in ((10, 8), (14, 16)):
            csr = rmat(scale, ef, 7 + scale, undirected=undirected, weighted=True)
            deg = np.diff(csr.rowptr.astype(np.int64))
            for src in (int(np.argmax(deg)), int(np.flatnonzero(deg == 0)[0]) if (deg == 0).any() else 0):
                out = np.zeros(csr.n)
                arr = (C.c_void_p * 1)(ctx.handle.value)
                s = csr.as_c()
                N.check(N.lib().gx_sssp_multi(arr, 1, C.byref(s), int(not undirected), src, N.as_dp(out)),
                        "gx_sssp_multi")
                assert np.array_equal(out, O.sssp(csr, src)), (scale, src)
    finally:
        ctx.close()


def test_gx_sssp_multi_rejects_bad_arguments():
    """Argument checks run before any device work (no GPU needed): unweighted graph, null
    contexts, source out of range."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    csr = rmat(6, 4, 1, undirected=True)
    s = csr.as_c()
    out = np.zeros(csr.n)
    arr = (C.c_void_p * 1)(None)
    assert N.lib().gx_sssp_multi(arr, 1, C.byref(s), 0, 0, N.as_dp(out)) != 0
    assert N.lib().gx_sssp_multi(None, 1, C.byref(s), 0, 0, N.as_dp(out)) != 0
    assert N.lib().gx_pagerank_multi(arr, 1, C.byref(s), 0, 0.85, 10, N.as_dp(out)) != 0


def _multi_call(fn, ctxs, csr, *args):
    """gx_<alg>_multi over the contexts `ctxs` (A.Context objects) -> result array."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    out = np.zeros(csr.n)
    arr = (C.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    s = csr.as_c()
    N.check(getattr(N.lib(), fn)(arr, len(ctxs), C.byref(s), *args, N.as_dp(out)), fn)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 3, 8])
@pytest.mark.parametrize("undirected", [True, False])
def test_multi_virtual_devices(k, undirected):
    """The executables' N > 1 path on one GPU: k contexts on device 0 are k
    virtual devices, each planned and run as its own GPU would be (pr_multi_plan's interleaved
    rows and owner * chunk + local column map with the device transpose when directed; the SSSP
    range cut; the LCC probe-work ranges), the collectives restated as device copies with their
    ordering.  PageRank rtol 1e-12, SSSP and LCC bit-exact, against the oracle."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    ctxs = [Context(0) for _ in range(k)]
    try:
        for scale, ef in ((10, 8), (14, 16)):
            csr = rmat(scale, ef, 5 + scale, undirected=undirected)
            got = _multi_call("gx_pagerank_multi", ctxs, csr, int(not undirected), 0.85, 10)
            np.testing.assert_allclose(got, O.pagerank(csr, not undirected, 0.85, 10), rtol=1e-12, atol=0)
            assert np.array_equal(_multi_call("gx_lcc_multi", ctxs, csr, int(not undirected)),
                                  O.lcc(csr, not undirected)), (k, scale)
            wcsr = rmat(scale, ef, 7 + scale, undirected=undirected, weighted=True)
            deg = np.diff(wcsr.rowptr.astype(np.int64))
            for src in (int(np.argmax(deg)), int(np.flatnonzero(deg == 0)[0]) if (deg == 0).any() else 0):
                got = _multi_call("gx_sssp_multi", ctxs, wcsr, int(not undirected), src)
                assert np.array_equal(got, O.sssp(wcsr, src)), (k, scale, src)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 3, 8])
@pytest.mark.parametrize("undirected", [True, False])
@pytest.mark.parametrize("rows,nnz", [(64, 2048), (16320, 1 << 30), (1, 1 << 30)])
def test_multi_virtual_devices_blocks(k, undirected, rows, nnz, monkeypatch):
    """gx_pagerank_multi's block partition (pr_multi_blocks, the huge-graph default): the
    hub-first order cut into blocks of at most `rows` rows and `nnz` entries -- small blocks,
    one block holding the whole graph (every other device owns nothing), one row per block --
    dealt largest first; each device planned with the whole graph's cut.  rtol 1e-12."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    monkeypatch.setenv("GX_PR_MULTI_PARTITION", "blocks")
    monkeypatch.setenv("GX_PR_MULTI_BLOCK_ROWS", str(rows))
    monkeypatch.setenv("GX_PR_MULTI_BLOCK_NNZ", str(nnz))
    ctxs = [Context(0) for _ in range(k)]
    try:
        for scale, ef in ((10, 8), (13, 16)):
            csr = rmat(scale, ef, 3 + scale, undirected=undirected)
            got = _multi_call("gx_pagerank_multi", ctxs, csr, int(not undirected), 0.85, 10)
            np.testing.assert_allclose(got, O.pagerank(csr, not undirected, 0.85, 10), rtol=1e-12, atol=0)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 3])
@pytest.mark.parametrize("pieces", [1, 3, 8])
@pytest.mark.parametrize("layout", ["interleave", "blocks"])
def test_multi_virtual_devices_pieces(k, pieces, layout, monkeypatch):
    """gx_pagerank_multi's pipelined pieces (round 6): each device's rows
    cut into `pieces` plans, piece p of device d being virtual rank p * k + d; piece p's chunks
    all-gathered on the comm streams while piece p + 1 runs.  One piece (no overlap), more
    pieces than some devices have live rows (8 pieces of a 2^10-vertex graph over 3 devices),
    both partitions, directed and undirected; rtol 1e-12 against the oracle."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    monkeypatch.setenv("GX_PR_MULTI_PIECES", str(pieces))
    monkeypatch.setenv("GX_PR_MULTI_PARTITION", layout)
    monkeypatch.setenv("GX_PR_MULTI_BLOCK_ROWS", "64")
    monkeypatch.setenv("GX_PR_MULTI_BLOCK_NNZ", "4096")
    ctxs = [Context(0) for _ in range(k)]
    try:
        for undirected in (True, False):
            for scale, ef in ((10, 8), (13, 16)):
                csr = rmat(scale, ef, 11 + scale, undirected=undirected)
                got = _multi_call("gx_pagerank_multi", ctxs, csr, int(not undirected), 0.85, 10)
                np.testing.assert_allclose(got, O.pagerank(csr, not undirected, 0.85, 10), rtol=1e-12, atol=0)
    finally:
        for c in ctxs:
            c.close()


def _multi_out(fn, ctxs, csr, dtype, *args):
    """gx_<alg>_multi with an integer result array of csr.n elements."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    out = np.zeros(csr.n, dtype=dtype)
    arr = (C.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    s = csr.as_c()
    ptr = out.ctypes.data_as(C.POINTER(C.c_int64 if dtype == np.int64 else C.c_uint64))
    N.check(getattr(N.lib(), fn)(arr, len(ctxs), C.byref(s), *args, ptr), fn)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 3])
@pytest.mark.parametrize("exchange", ["auto", "sparse", "dense"])
def test_multi_virtual_devices_bfs_wcc_cdlp(k, exchange, monkeypatch):
    """bin/exe/{bfs,wcc,cdlp}'s GX_NGPUS path (round 6): gx_bfs_multi /
    gx_wcc_multi / gx_cdlp_multi on k virtual devices, the graph replicated, vertex ranges by
    entries, per round the changed entries as words (or the dense form: BFS bitmaps, CDLP owned
    slices), directed and undirected, against the oracle bit for bit."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    monkeypatch.setenv("GX_EXCHANGE", exchange)
    ctxs = [Context(0) for _ in range(k)]
    try:
        for undirected in (True, False):
            for scale, ef in ((10, 8), (13, 16)):
                csr = rmat(scale, ef, 21 + scale, undirected=undirected)
                deg = np.diff(csr.rowptr.astype(np.int64))
                for src in (int(np.argmax(deg)), int(np.flatnonzero(deg == 0)[0]) if (deg == 0).any() else 1):
                    got = _multi_out("gx_bfs_multi", ctxs, csr, np.int64, int(not undirected), src)
                    assert np.array_equal(got, O.bfs(csr, src)), (k, scale, src)
                got = _multi_out("gx_wcc_multi", ctxs, csr, np.uint64, int(not undirected))
                assert np.array_equal(got.astype(np.int64), O.wcc(csr).astype(np.int64)), (k, scale)
                got = _multi_out("gx_cdlp_multi", ctxs, csr, np.uint64, int(not undirected), 10)
                assert np.array_equal(got.astype(np.int64), O.cdlp(csr, not undirected, 10).astype(np.int64)), (k, scale)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.gpu
def test_multi_virtual_devices_edge_cases():
    """More virtual devices than rows with out-edges (some own nothing live), an edgeless graph,
    and LCC on one device (a size-1 RCCL clique and its ncclReduce)."""
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    from ldbc_graphalytics_platforms_graphblas_amd.graphio import CSR
    ctxs = [Context(0) for _ in range(8)]
    try:
        # a 5-vertex path 0-1-2 plus two isolated vertices, undirected and weighted
        rp = np.array([0, 1, 3, 4, 4, 4], dtype=np.uint64)
        ci = np.array([1, 0, 2, 1], dtype=np.uint64)
        w = np.array([0.5, 0.5, 2.0, 2.0])
        tiny = CSR(5, rp, ci, w)
        got = _multi_call("gx_pagerank_multi", ctxs, tiny, 0, 0.85, 10)
        np.testing.assert_allclose(got, O.pagerank(tiny, False, 0.85, 10), rtol=1e-12, atol=0)
        assert np.array_equal(_multi_call("gx_sssp_multi", ctxs, tiny, 0, 2), O.sssp(tiny, 2))
        assert np.array_equal(_multi_call("gx_lcc_multi", ctxs, tiny, 0), O.lcc(tiny, False))
        empty = CSR(4, np.zeros(5, dtype=np.uint64), np.zeros(0, dtype=np.uint64), np.zeros(0))
        np.testing.assert_allclose(_multi_call("gx_pagerank_multi", ctxs[:3], empty, 1, 0.85, 10),
                                   O.pagerank(empty, True, 0.85, 10), rtol=1e-12, atol=0)
        assert np.array_equal(_multi_call("gx_lcc_multi", ctxs[:3], empty, 1), np.zeros(4))
        csr = rmat(12, 8, 31, undirected=False)
        assert np.array_equal(_multi_call("gx_lcc_multi", ctxs[:1], csr, 1), O.lcc(csr, True))
    finally:
        for c in ctxs:
            c.close()


def test_multi_rejects_bad_contexts():
    """gx_lcc_multi / gx_pagerank_multi refuse null contexts and ndev < 1 before any device
    work (no GPU needed)."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    csr = rmat(6, 4, 1, undirected=True)
    s = csr.as_c()
    out = np.zeros(csr.n)
    for fn, args in (("gx_lcc_multi", (0,)), ("gx_pagerank_multi", (0, 0.85, 10))):
        arr = (C.c_void_p * 2)(None, None)
        assert getattr(N.lib(), fn)(arr, 2, C.byref(s), *args, N.as_dp(out)) == -2   # GX_NULL_POINTER
        assert getattr(N.lib(), fn)(arr, 0, C.byref(s), *args, N.as_dp(out)) == -3   # ndev < 1
    arr = (C.c_void_p * 2)(None, None)
    assert N.lib().gx_multi_prepare(arr, 2) == -2
    assert N.lib().gx_multi_prepare(arr, 0) == -3
    assert N.lib().gx_multi_prepare(None, 1) == -2


@pytest.mark.gpu
def test_multi_clique_cache():
    """gx_multi_prepare makes the clique the gx_*_multi calls on the same context list reuse; a
    call on another list (a subset) makes its own; gx_free of a member drops every clique holding
    it, and the survivors still run (results bit-exact / rtol 1e-12 every time)."""
    import ctypes as C
    from ldbc_graphalytics_platforms_graphblas_amd import _native as N
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context
    ctxs = [Context(0) for _ in range(4)]
    try:
        arr = (C.c_void_p * 4)(*[c.handle.value for c in ctxs])
        N.check(N.lib().gx_multi_prepare(arr, 4), "gx_multi_prepare")
        N.check(N.lib().gx_multi_prepare(arr, 4), "gx_multi_prepare")
        csr = rmat(11, 8, 41, undirected=False)
        want_pr = O.pagerank(csr, True, 0.85, 10)
        want_lcc = O.lcc(csr, True)
        for sub in (ctxs, ctxs, ctxs[:2], ctxs[:1]):
            np.testing.assert_allclose(_multi_call("gx_pagerank_multi", sub, csr, 1, 0.85, 10), want_pr,
                                       rtol=1e-12, atol=0)
            assert np.array_equal(_multi_call("gx_lcc_multi", sub, csr, 1), want_lcc)
        ctxs[3].close()
        ctxs = ctxs[:3]
        np.testing.assert_allclose(_multi_call("gx_pagerank_multi", ctxs, csr, 1, 0.85, 10), want_pr,
                                   rtol=1e-12, atol=0)
        ctxs[0].close()
        ctxs = ctxs[1:]
        assert np.array_equal(_multi_call("gx_lcc_multi", ctxs, csr, 1), want_lcc)
    finally:
        for c in ctxs:
            c.close()
