// gx_bfs.hip -- level-synchronous BFS (Graphalytics BFS = hop levels over out-edges).
//
// Replaces LA_BFS -> LAGr_BreadthFirstSearch(&level, NULL, G, src) (bfs.cpp:70-83), which
// SuiteSparse runs as a masked vxm per level over the boolean semiring.  Here:
//   top-down  : one wave per frontier vertex walks its out-row; an unvisited neighbour is
//               claimed with atomicCAS(level, -1, d+1) and appended to the next queue with
//               one wave-aggregated atomic (ballot + mbcnt).
//   bottom-up : (when the in-edges are resident: undirected graphs, or a directed graph
//               whose transpose is already built) one thread per unvisited vertex scans its
//               in-row until it meets a vertex of the current level.
// Direction switching follows Beamer's heuristic (alpha = 14, beta = 24).  Levels are
// unique, so the result is bit-exact whatever the traversal order.
#include "gx_device.h"

namespace gx {
namespace {

constexpr int kBfsBlock = 256;

__device__ __forceinline__ void wave_append(bool take, int32_t v, int32_t *queue, uint32_t *qcount) {
    const uint64_t mask = __ballot(take);
    if (mask == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int leader = __ffsll((unsigned long long)mask) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(qcount, (uint32_t)__popcll(mask));
    base = __shfl(base, leader, kWave);
    if (take) {
        const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1));
        queue[base + rank] = v;
    }
}

// top-down: one wave per frontier vertex
__global__ __launch_bounds__(kBfsBlock) void k_bfs_topdown(const int64_t *__restrict__ rp,
                                                           const int32_t *__restrict__ ci,
                                                           const int32_t *__restrict__ qin,
                                                           uint32_t qsize, int32_t *level,
                                                           int32_t depth, int32_t *qout,
                                                           uint32_t *qcount,
                                                           unsigned long long *next_edges) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = (blockIdx.x * kBfsBlock + threadIdx.x) / kWave;
    const uint32_t nwaves = gridDim.x * (kBfsBlock / kWave);
    unsigned long long edges = 0;
    for (uint32_t f = wave; f < qsize; f += nwaves) {
        const int32_t u = qin[f];
        const int64_t b = rp[u], e = rp[u + 1];
        for (int64_t k0 = b; k0 < e; k0 += kWave) {
            const int64_t k = k0 + lane;
            bool take = false;
            int32_t v = 0;
            if (k < e) {
                v = ci[k];
                if (level[v] < 0 && atomicCAS(&level[v], -1, depth + 1) == -1) {
                    take = true;
                    edges += (unsigned long long)(rp[v + 1] - rp[v]);
                }
            }
            wave_append(take, v, qout, qcount);
        }
    }
    // one atomic per wave for the next frontier's edge count (direction heuristic)
    for (int off = 32; off > 0; off >>= 1) edges += __shfl_xor(edges, off, kWave);
    if (lane == 0 && edges) atomicAdd(next_edges, edges);
}

// bottom-up: one thread per vertex; in-edges in (rpi, cii)
__global__ __launch_bounds__(kBfsBlock) void k_bfs_bottomup(const int64_t *__restrict__ rpi,
                                                            const int32_t *__restrict__ cii,
                                                            const int64_t *__restrict__ rpo,
                                                            int64_t n, int32_t *level, int32_t depth,
                                                            int32_t *qout, uint32_t *qcount,
                                                            unsigned long long *next_edges) {
    unsigned long long edges = 0;
    const int64_t stride = (int64_t)gridDim.x * kBfsBlock;
    const int64_t nround = (n + stride - 1) / stride;
    for (int64_t r = 0; r < nround; r++) {
        const int64_t v = r * stride + (int64_t)blockIdx.x * kBfsBlock + threadIdx.x;
        bool take = false;
        if (v < n && level[v] < 0) {
            for (int64_t k = rpi[v]; k < rpi[v + 1]; k++) {
                if (level[cii[k]] == depth) {
                    take = true;
                    break;
                }
            }
            if (take) {
                level[v] = depth + 1;
                edges += (unsigned long long)(rpo[v + 1] - rpo[v]);
            }
        }
        wave_append(take, (int32_t)v, qout, qcount);
    }
    for (int off = 32; off > 0; off >>= 1) edges += __shfl_xor(edges, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0 && edges) atomicAdd(next_edges, edges);
}

__global__ void k_bfs_seed(int32_t *level, int32_t *queue, int32_t src) {
    level[src] = 0;
    queue[0] = src;
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_bfs(gx_graph *g, uint64_t src, int64_t *level_out) {
    if (!g || !level_out) return fail(GX_NULL_POINTER, "gx_bfs: null argument");
    if (src >= g->n) return fail(GX_INVALID_INDEX, "gx_bfs: source out of range");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    DBuf<int32_t> level, q0, q1;
    DBuf<uint32_t> qcount;
    DBuf<unsigned long long> nedges;
    GX_TRY(level.alloc(n));
    GX_TRY(q0.alloc(n));
    GX_TRY(q1.alloc(n));
    GX_TRY(qcount.alloc(1));
    GX_TRY(nedges.alloc(1));
    GX_TRY(device_begin(ctx));
    // in-edges: the graph itself when undirected, the transpose when already resident
    const DevCSR *in = g->directed ? (g->AT.built ? &g->AT : nullptr) : &g->A;
    GX_HIP_TRY(hipMemsetAsync(level.p, 0xff, n * 4, s));
    hipLaunchKernelGGL(k_bfs_seed, dim3(1), dim3(1), 0, s, level.p, q0.p, (int32_t)src);
    GX_TRY(check_launch("k_bfs_seed"));
    uint32_t qsize = 1;
    unsigned long long mf = (unsigned long long)(g->A.h_rp[src + 1] - g->A.h_rp[src]);
    unsigned long long mu = g->nnz;
    bool bottom_up = false;
    int32_t depth = 0;
    struct Counters {
        uint32_t q;
        uint32_t pad;
        unsigned long long e;
    };
    while (qsize > 0) {
        // Beamer switch: TD -> BU when the frontier's edges exceed the unexplored ones / 14;
        // BU -> TD when the frontier shrinks below n / 24.
        if (in) {
            if (!bottom_up && mf > mu / 14) bottom_up = true;
            else if (bottom_up && (int64_t)qsize < n / 24) bottom_up = false;
        }
        GX_HIP_TRY(hipMemsetAsync(qcount.p, 0, 4, s));
        GX_HIP_TRY(hipMemsetAsync(nedges.p, 0, 8, s));
        if (bottom_up) {
            KTimer kt(ctx, "bfs_bottomup", s);
            hipLaunchKernelGGL(k_bfs_bottomup, dim3(grid_for(n, kBfsBlock, 8192)), dim3(kBfsBlock), 0, s,
                               in->rp.p, in->ci.p, g->A.rp.p, n, level.p, depth, q1.p, qcount.p,
                               nedges.p);
        } else {
            KTimer kt(ctx, "bfs_topdown", s);
            const uint64_t waves = qsize;
            hipLaunchKernelGGL(k_bfs_topdown, dim3(grid_for(waves * kWave, kBfsBlock, 8192)),
                               dim3(kBfsBlock), 0, s, g->A.rp.p, g->A.ci.p, q0.p, qsize, level.p, depth,
                               q1.p, qcount.p, nedges.p);
        }
        GX_TRY(check_launch("bfs step"));
        Counters c{};
        GX_HIP_TRY(hipMemcpyAsync(&c.q, qcount.p, 4, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipMemcpyAsync(&c.e, nedges.p, 8, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        mu = mu > mf ? mu - mf : 0;
        mf = c.e;
        qsize = c.q;
        std::swap(q0.p, q1.p);
        depth++;
    }
    GX_TRY(device_end(ctx));
    std::vector<int32_t> h(n);
    GX_HIP_TRY(hipMemcpy(h.data(), level.p, n * 4, hipMemcpyDeviceToHost));
    for (int64_t v = 0; v < n; v++) level_out[v] = h[v] < 0 ? INT64_MAX : (int64_t)h[v];
    return GX_SUCCESS;
}
