"""Multi-GPU BFS / WCC / SSSP / CDLP / LCC drivers (distributed.py).

CPU (gloo, world_size 2): the drivers with TorchComm over real torch.distributed
collectives, each rank stepping through a numpy restatement of the gx_*_part_* contract
(test-only stand-in), checked against the oracle.
GPU: the gx_*_part_* entry points themselves with 1, 2 and 3 ranks simulated on one device
(LocalComm), checked against the oracle bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sys.path)
from ldbc_graphalytics_platforms_graphblas_amd import distributed as D
from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
from oracle import oracle as O

INF = np.iinfo(np.int64).max


class NumpyBackend:
    """numpy restatement of the gx_*_part_* steps on torch CPU tensors (test-only)."""

    def __init__(self, csr, directed):
        self.n = csr.n
        self.rp = csr.rowptr.astype(np.int64)
        self.ci = csr.colidx.astype(np.int64)
        self.w = csr.vals
        self.directed = directed
        self.deg = np.diff(self.rp)
        self.rows = np.repeat(np.arange(self.n), self.deg)

    def _owned_edges(self, v0, v1, pick):
        e0, e1 = self.rp[v0], self.rp[v1]
        rows, cols = self.rows[e0:e1], self.ci[e0:e1]
        m = pick[rows]
        return rows[m], cols[m], np.flatnonzero(m) + e0

    # BFS
    def bfs_init(self, src, level):
        lv = level.numpy()
        lv[:] = INF
        lv[src] = 0

    def bfs_expand(self, v0, v1, level, cur, nxt):
        lv, nx = level.numpy(), nxt.numpy()
        _, cols, _ = self._owned_edges(v0, v1, lv == cur)
        nx[cols[lv[cols] == INF]] = 1

    def bfs_commit(self, nxt, level, cur, count):
        lv, nx = level.numpy(), nxt.numpy()
        m = (nx != 0) & (lv == INF)
        lv[m] = cur + 1
        count.numpy()[0] += int(m.sum())

    # sparse exchange (gx_part_changes / gx_part_apply)
    def changes(self, a, b, v0, v1, elem, words, count):
        av = a.numpy()[v0:v1].astype(np.int64)
        bv = b.numpy()[v0:v1].astype(np.int64) if b is not None else np.zeros_like(av)
        idx = np.flatnonzero(av != bv)
        w = words.numpy()
        w[:len(idx)] = ((idx + v0).astype(np.int64) << 32) | (av[idx] & 0xFFFFFFFF)
        count.numpy()[0] = len(idx)

    def apply(self, words, counts, nranks, stride, arr, elem, op):
        w, cs, a = words.numpy(), counts.numpy(), arr.numpy()
        for k in range(nranks):
            x = w[k * stride:k * stride + int(cs[k])]
            v = (x >> 32).astype(np.int64)
            val = (x & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(a.dtype)
            if op == 0:
                a[v] = val
            elif op == 1:
                np.minimum.at(a, v, val)
            else:
                np.maximum.at(a, v, val)

    def pack_bits(self, nxt, bits):
        nx = nxt.numpy() != 0
        pad = np.zeros(bits.numel() * 32, dtype=bool)
        pad[:len(nx)] = nx
        bits.numpy()[:] = np.packbits(pad.reshape(-1, 32)[:, ::-1], axis=1, bitorder="big").view(">u4").astype(np.uint32).view(np.int32).ravel()

    def or_bits(self, gathered, nranks, nxt):
        n = nxt.numel()
        w = gathered.numpy().view(np.uint32).reshape(nranks, -1)
        anyb = np.bitwise_or.reduce(w, axis=0)
        v = np.arange(n)
        nxt.numpy()[:] = ((anyb[v // 32] >> (v % 32)) & 1).astype(np.uint8)

    # WCC
    def wcc_init(self, parent):
        parent.numpy()[:] = np.arange(self.n, dtype=np.int32)

    @staticmethod
    def _root(p, v):
        while p[v] != v:
            v = p[v]
        return v

    def wcc_hook(self, v0, v1, parent, changed):
        p = parent.numpy()
        for e in range(self.rp[v0], self.rp[v1]):
            ru, rv = self._root(p, self.rows[e]), self._root(p, self.ci[e])
            if ru != rv:
                hi, lo = max(ru, rv), min(ru, rv)
                p[hi] = min(p[hi], lo)
                changed.numpy()[0] = 1
        self.wcc_compress(parent)

    def wcc_compress(self, parent):
        p = parent.numpy()
        for v in range(self.n):
            p[v] = self._root(p, v)

    # SSSP
    def sssp_split(self, v0, v1):
        return _NpSsspSplit(self, v0, v1)

    # CDLP
    def cdlp_part(self, v0, v1):
        return _NpCdlp(self, v0, v1)

    # LCC
    def lcc_part(self):
        return _NpLcc(self)


class _NpSsspSplit:
    """numpy restatement of gx_sssp_split's protocol (gx_sssp_split.hip): the edges into
    [v0, v1) by source, a replicated distance vector, the same plan (LIGHT / HEAVY / ADVANCE /
    done) from the same replicated counts, (vertex, fp64 bits) pairs of the improved owned
    vertices."""

    def __init__(self, be, v0, v1):
        self.be, self.v0, self.v1 = be, v0, v1
        w = be.w
        mean_deg = max(1.0, len(be.ci) / max(1, be.n))
        self.delta = 3.0 * float(w.mean() if len(w) else 1.0) / mean_deg
        own = (be.ci >= v0) & (be.ci < v1)
        self.light = [[] for _ in range(be.n)]
        self.heavy = [[] for _ in range(be.n)]
        for e in np.flatnonzero(own):
            (self.light if w[e] < self.delta else self.heavy)[be.rows[e]].append((int(be.ci[e]), float(w[e])))

    def _b(self, d):
        return int(min(d / self.delta, 4.0e18))

    def _queue(self, v, d):
        self.lrel[v] = d
        self.f_next.append(v)
        if self.sstamp[v] != self.epoch:
            self.sstamp[v] = self.epoch
            self.S.append(v)

    def start(self, src):
        n = self.be.n
        self.dist = np.full(n, np.inf)
        self.dist[src] = 0.0
        self.lrel = np.full(n, np.inf)
        self.sstamp = np.zeros(n, np.int64)
        self.epoch, self.cur, self.done, self.mode = 1, 0, False, 0
        self.f_next, self.S, self.s_done, self.P = [], [], 0, set()
        self._queue(src, 0.0)

    def relax(self, pairs, count):
        work, edges = [], self.light
        if self.done:
            self.mode = 0
        elif self.f_next:
            self.mode, work, self.f_next = 1, self.f_next, []
        elif len(self.S) > self.s_done:
            self.mode, work, edges = 2, self.S[self.s_done:], self.heavy
            self.s_done = len(self.S)
        elif self.P:
            self.mode = 3
            self.epoch += 1
            self.S, self.s_done = [], 0
            pend = [v for v in self.P if self.dist[v] < self.lrel[v]]
            cb = min((self._b(self.dist[v]) for v in pend), default=int(4e18))
            self.P = {v for v in pend if self._b(self.dist[v]) > cb}
            for v in sorted(v for v in pend if self._b(self.dist[v]) <= cb):
                self._queue(v, self.dist[v])
            self.cur = cb
            work, self.f_next = self.f_next, []
        else:
            self.done, self.mode = True, 0
        before = self.dist.copy()
        for u in work:
            for v, x in edges[u]:
                self.dist[v] = min(self.dist[v], self.dist[u] + x)
        imp = np.flatnonzero(self.dist[self.v0:self.v1] < before[self.v0:self.v1]) + self.v0
        pr = pairs.numpy()
        pr[0:2 * len(imp):2] = imp
        pr[1:2 * len(imp):2] = self.dist[imp].view(np.int64)
        count.numpy()[:] = [len(imp), int(self.done)]

    def apply(self, pairs, counts, nranks, stride):
        if self.mode == 0:
            return
        pr, cw = pairs.numpy(), counts.numpy()
        for r in range(nranks):
            for i in range(int(cw[2 * r])):
                v = int(pr[2 * (r * stride + i)])
                d = float(pr[2 * (r * stride + i) + 1:2 * (r * stride + i) + 2].view(np.float64)[0])
                self.dist[v] = min(self.dist[v], d)
                if self._b(d) <= self.cur:
                    self._queue(v, d)
                else:
                    self.P.add(v)

    def distances(self, out):
        out.numpy()[:] = self.dist

    def close(self):
        pass


class _NpCdlp:
    def __init__(self, be, v0, v1):
        self.be, self.v0, self.v1 = be, v0, v1
        nb = [[] for _ in range(be.n)]
        for u, v in zip(be.rows, be.ci):
            nb[u].append(v)
            if be.directed:
                nb[v].append(u)
        self.nb = nb

    def init(self, labels):
        labels.numpy()[:] = np.arange(self.be.n, dtype=np.int32)

    def step(self, labels, nxt, changed):
        lb, nx = labels.numpy(), nxt.numpy()
        for v in range(self.v0, self.v1):
            if not self.nb[v]:
                nx[v] = lb[v]
                continue
            vals, cnt = np.unique(lb[self.nb[v]], return_counts=True)
            nx[v] = vals[cnt == cnt.max()].min()
            if nx[v] != lb[v]:
                changed.numpy()[0] = 1

    def close(self):
        pass


class _NpLcc:
    def __init__(self, be):
        self.be = be
        n = be.n
        out = [set() for _ in range(n)]
        for u, v in zip(be.rows, be.ci):
            if u != v:
                out[u].add(int(v))
        self.out = out
        self.S = [set() for _ in range(n)]
        for u in range(n):
            for v in out[u]:
                self.S[u].add(v)
                self.S[v].add(u)
        self.k = np.array([len(s) for s in self.S])
        key = lambda x: (self.k[x], x)   # noqa: E731
        self.O = [sorted(u for u in self.S[v] if key(u) > key(v)) for v in range(n)]

    def _dirs(self, a, b):
        return int(b in self.out[a]) + int(a in self.out[b])

    def ranges(self, nranks):
        return np.linspace(0, self.be.n, nranks + 1).astype(np.uint64)

    def counts(self, v0, v1, tc):
        t = tc.numpy()
        for v in range(v0, v1):
            ov = set(self.O[v])
            for u in self.O[v]:
                for x in ov.intersection(self.O[u]):
                    t[v] += self._dirs(u, x)
                    t[u] += self._dirs(v, x)
                    t[x] += self._dirs(v, u)

    def finish(self, tc, out):
        k = self.k.astype(np.float64)
        o = out.numpy()
        o[:] = np.where(self.k >= 2, tc.numpy() / np.maximum(k * (k - 1), 1.0), 0.0)

    def close(self):
        pass


def _graphs():
    und = rmat(8, 6, 21, undirected=True, weighted=True)
    dirg = rmat(8, 5, 22, undirected=False, weighted=True)
    return [(und, False), (dirg, True)]


def _src(csr):
    return int(np.argmax(np.diff(csr.rowptr.astype(np.int64))))


def _run_all(ranks, comm, csr, directed, ranges):
    n = csr.n
    src = _src(csr)
    return {
        "bfs": D.bfs(ranks, comm, n, src).cpu().numpy(),
        "wcc": D.wcc(ranks, comm, n).cpu().numpy(),
        "sssp": D.sssp(ranks, comm, n, src).cpu().numpy(),
        "cdlp": D.cdlp(ranks, comm, n, 6, ranges).cpu().numpy(),
        "lcc": D.lcc(ranks, comm, n).cpu().numpy(),
    }


def _check(res, csr, directed):
    src = _src(csr)
    assert np.array_equal(res["bfs"], O.bfs(csr, src))
    assert np.array_equal(res["wcc"].astype(np.int64), O.wcc(csr).astype(np.int64))
    assert np.array_equal(res["sssp"], O.sssp(csr, src))
    assert np.array_equal(res["cdlp"].astype(np.int64), O.cdlp(csr, directed, 6).astype(np.int64))
    assert np.array_equal(res["lcc"], O.lcc(csr, directed))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for csr, directed in _graphs():
            rng = D.vertex_ranges(csr.rowptr, world)
            r = D.LocalRank(NumpyBackend(csr, directed), int(rng[rank]), int(rng[rank + 1]), "cpu", rank)
            out.append(_run_all([r], D.TorchComm(), csr, directed, rng))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_world2_all_algorithms():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for res, (csr, directed) in zip(out, _graphs()):
        _check(res, csr, directed)


@pytest.mark.parametrize("exchange", ["auto", "sparse", "dense"])
def test_local_comm_numpy_three_ranks(exchange, monkeypatch):
    """The lock-step drivers with LocalComm (what the single-GPU simulation uses), with the
    frontier-sized word exchange chosen by size, always, or never (distributed._exchange)."""
    monkeypatch.setattr(D, "EXCHANGE", exchange)
    for csr, directed in _graphs():
        rng = D.vertex_ranges(csr.rowptr, 3)
        be = NumpyBackend(csr, directed)
        ranks = [D.LocalRank(be, int(rng[k]), int(rng[k + 1]), "cpu", k) for k in range(3)]
        _check(_run_all(ranks, D.LocalComm(), csr, directed, rng), csr, directed)


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [1, 2, 3])
@pytest.mark.parametrize("exchange", ["auto", "sparse", "dense"])
def test_gpu_partitioned_simulated_ranks(nranks, exchange, monkeypatch):
    monkeypatch.setattr(D, "EXCHANGE", exchange)
    from ldbc_graphalytics_platforms_graphblas_amd.algorithms import Context, Graph
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    for csr, directed in [(rmat(12, 8, 31, undirected=True, weighted=True), False),
                          (rmat(12, 6, 32, undirected=False, weighted=True), True)]:
        g = Graph(ctx, csr, directed)
        try:
            be = D.GpuBackend(g)
            rng = D.vertex_ranges(csr.rowptr, nranks)
            ranks = [D.LocalRank(be, int(rng[k]), int(rng[k + 1]), dev, k) for k in range(nranks)]
            _check(_run_all(ranks, D.LocalComm(), csr, directed, rng), csr, directed)
        finally:
            g.close()
    ctx.close()
