// gx_bfs.hip -- level-synchronous BFS (Graphalytics BFS = hop levels over out-edges).
//
// Replaces LA_BFS -> LAGr_BreadthFirstSearch(&level, NULL, G, src) (bfs.cpp:70-83), which
// SuiteSparse runs as a masked vxm per level over the boolean semiring.  Here:
//   top-down  : one wave per frontier vertex walks its out-row; an unvisited neighbour is
//               claimed with atomicCAS(level, -1, d+1) and appended to the next queue with
//               one wave-aggregated atomic (ballot + mbcnt).
//   bottom-up : (when the in-edges are resident: undirected graphs, or a directed graph
//               whose transpose is already built) one thread per unvisited vertex scans its
//               in-row, probing a bitmap of the current level (n/8 bytes, L2-resident) four
//               neighbours at a time, until it meets a frontier vertex.
// Direction switching follows Beamer's heuristic (alpha = 14, beta = 24).  Levels are
// unique, so the result is bit-exact whatever the traversal order.
#include <cstdlib>
#include <memory>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kBfsBlock = 256;
constexpr int kChunk = 256;   // edges per top-down work item (4 per lane)

// Frontier work items: (vertex << 32) | chunk, one item per kChunk out-edges, so a hub's
// adjacency is spread over many waves.  Appends are wave-aggregated: an inclusive scan of
// the lanes' item counts, one atomicAdd per wave.
__device__ __forceinline__ void wave_append(bool take, int32_t v, uint32_t nch, uint64_t *queue,
                                            uint32_t *qcount) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t k = take ? nch : 0u;
    uint32_t x = k;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, kWave);
        if (lane >= off) x += y;
    }
    const uint32_t total = __shfl(x, kWave - 1, kWave);
    if (total == 0) return;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(qcount, total);
    base = __shfl(base, 0, kWave);
    const uint32_t excl = x - k;
    for (uint32_t j = 0; j < k; j++) queue[base + excl + j] = ((uint64_t)(uint32_t)v << 32) | j;
}

__device__ __forceinline__ uint32_t chunks_of(int64_t deg) {
    return (uint32_t)((deg + kChunk - 1) / kChunk);
}

// top-down: one wave per work item (<= kChunk edges of one frontier vertex)
__device__ __forceinline__ void bfs_topdown(const int64_t *__restrict__ rp,
                                                           const int32_t *__restrict__ ci,
                                                           const uint64_t *__restrict__ qin,
                                                           uint32_t qsize, int32_t *level,
                                                           int32_t depth, uint64_t *qout,
                                                           uint32_t *qcount,
                                                           unsigned long long *next_edges, uint32_t bid,
                                                           uint32_t nblk) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = (bid * kBfsBlock + threadIdx.x) / kWave;
    const uint32_t nwaves = nblk * (kBfsBlock / kWave);
    unsigned long long edges = 0;
    for (uint32_t f = wave; f < qsize; f += nwaves) {
        const uint64_t item = qin[f];
        const int32_t u = (int32_t)(item >> 32);
        const int64_t e = rp[u + 1];
        const int64_t b = rp[u] + (int64_t)(uint32_t)item * kChunk;
        const int64_t end = min(e, b + kChunk);
#pragma unroll
        for (int i = 0; i < kChunk / kWave; i++) {
            const int64_t k = b + lane + (int64_t)i * kWave;
            bool take = false;
            int32_t v = 0;
            int64_t dv = 0;
            if (k < end) {
                v = ci[k];
                if (level[v] < 0 && atomicCAS(&level[v], -1, depth + 1) == -1) {
                    take = true;
                    dv = rp[v + 1] - rp[v];
                    edges += (unsigned long long)dv;
                }
            }
            wave_append(take, v, chunks_of(dv), qout, qcount);
        }
    }
    // one atomic per wave for the next frontier's edge count (direction heuristic)
    for (int off = 32; off > 0; off >>= 1) edges += __shfl_xor(edges, off, kWave);
    if (lane == 0 && edges) atomicAdd(next_edges, edges);
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_topdown(const int64_t *__restrict__ rp,
                                                           const int32_t *__restrict__ ci,
                                                           const uint64_t *__restrict__ qin, uint32_t qsize,
                                                           int32_t *level, int32_t depth, uint64_t *qout,
                                                           uint32_t *qcount, unsigned long long *next_edges) {
    bfs_topdown(rp, ci, qin, qsize, level, depth, qout, qcount, next_edges, blockIdx.x, gridDim.x);
}

// bottom-up: one thread per vertex; in-edges in (rpi, cii)
// Frontier bitmap for bottom-up steps: bit u set iff level[u] == depth.  One 64-bit word per
// wave (ballot over 64 consecutive vertices); n/8 bytes, so it stays resident in every XCD's
// L2 while the bottom-up probes hit it at random (the int32 level array does not).
__device__ __forceinline__ void bfs_bitmap(const int32_t *__restrict__ level, int64_t n, int32_t depth,
                                           uint64_t *fb, uint32_t bid, uint32_t nblk) {
    const int64_t stride = (int64_t)nblk * kBfsBlock;
    const int64_t nround = (n + stride - 1) / stride;
    for (int64_t r = 0; r < nround; r++) {
        const int64_t v = r * stride + (int64_t)bid * kBfsBlock + threadIdx.x;
        const uint64_t m = __ballot(v < n && level[v] == depth);
        if ((threadIdx.x & (kWave - 1)) == 0 && v < n) fb[v >> 6] = m;
    }
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_bitmap(const int32_t *__restrict__ level, int64_t n,
                                                          int32_t depth, uint64_t *fb) {
    bfs_bitmap(level, n, depth, fb, blockIdx.x, gridDim.x);
}

__device__ __forceinline__ uint32_t in_frontier(const uint64_t *__restrict__ fb, int32_t u) {
    return (uint32_t)((fb[u >> 6] >> (u & 63)) & 1ull);
}

// bottom-up: one thread per unvisited vertex scans its in-row, 4 neighbours per step (four
// independent bitmap probes in flight), until it meets a frontier vertex.  The next frontier
// is left in `level` (no queue: a queue append per wave is one same-address atomic per wave,
// ~11 ns each serialised, which dominated); found vertices and their out-edges are summed
// per workgroup and leave as one atomic each.
__device__ __forceinline__ void bfs_bottomup(const int64_t *__restrict__ rpi,
                                                            const int32_t *__restrict__ cii,
                                                            const int64_t *__restrict__ rpo,
                                                            const uint64_t *__restrict__ fb, int64_t n,
                                                            int32_t *level, int32_t depth,
                                                            unsigned long long *counters /* found, edges */,
                                                            uint64_t *fbn, uint32_t bid, uint32_t nblk) {
    __shared__ unsigned long long red[2][kBfsBlock / kWave];
    unsigned long long edges = 0, found = 0;
    // uniform trip count: a wave covers 64 aligned consecutive vertices per round, so with fbn
    // its ballot of the vertices found is the next level's frontier word (no bitmap pass)
    const int64_t stride = (int64_t)nblk * kBfsBlock;
    const int64_t nround = (n + stride - 1) / stride;
    for (int64_t r = 0; r < nround; r++) {
        const int64_t v = r * stride + (int64_t)bid * kBfsBlock + threadIdx.x;
        bool take = false;
        if (v < n && level[v] < 0) {
            const int64_t b = rpi[v], e = rpi[v + 1];
            for (int64_t k = b; k < e && !take; k += 4) {
                const int32_t u0 = cii[k];
                const int32_t u1 = cii[min(k + 1, e - 1)];
                const int32_t u2 = cii[min(k + 2, e - 1)];
                const int32_t u3 = cii[min(k + 3, e - 1)];
                // all four probes issue (no short-circuit), then one test
                take = (in_frontier(fb, u0) | in_frontier(fb, u1) | in_frontier(fb, u2) | in_frontier(fb, u3)) != 0;
            }
            if (take) {
                level[v] = depth + 1;
                edges += (unsigned long long)(rpo[v + 1] - rpo[v]);
                found++;
            }
        }
        if (fbn) {
            const uint64_t m = __ballot(take);
            if ((threadIdx.x & (kWave - 1)) == 0 && v < n) fbn[v >> 6] = m;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        edges += __shfl_xor(edges, off, kWave);
        found += __shfl_xor(found, off, kWave);
    }
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        red[0][w] = found;
        red[1][w] = edges;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long f = 0, ed = 0;
        for (int i = 0; i < kBfsBlock / kWave; i++) {
            f += red[0][i];
            ed += red[1][i];
        }
        if (f) atomicAdd(&counters[0], f);
        if (ed) atomicAdd(&counters[1], ed);
    }
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_bottomup(const int64_t *__restrict__ rpi,
                                                            const int32_t *__restrict__ cii,
                                                            const int64_t *__restrict__ rpo,
                                                            const uint64_t *__restrict__ fb, int64_t n,
                                                            int32_t *level, int32_t depth,
                                                            unsigned long long *counters) {
    bfs_bottomup(rpi, cii, rpo, fb, n, level, depth, counters, nullptr, blockIdx.x, gridDim.x);
}

// Top-down queue of the vertices at `depth` (after bottom-up steps), built per tile of
// kQTile consecutive vertices: count the tile's items, one atomicAdd for its base, write.
constexpr int64_t kQTile = 4096;

// With fb (the frontier bitmap a bottom-up level left) the frontier test reads n/8 bytes of
// bitmap words (one line per wave) instead of the n int32 levels, twice.
__device__ __forceinline__ void bfs_level_queue(const int64_t *__restrict__ rp, const int32_t *__restrict__ level,
                                                int64_t n, int32_t depth, uint64_t *queue, uint32_t *qcount,
                                                const uint64_t *__restrict__ fb, uint32_t bid, uint32_t nblk) {
    auto at_depth = [&](int64_t v) -> bool {
        return fb ? ((fb[v >> 6] >> (v & 63)) & 1ull) != 0 : level[v] == depth;
    };
    __shared__ uint32_t wsum[kBfsBlock / kWave];
    __shared__ uint32_t tile_base;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    for (int64_t t0 = (int64_t)bid * kQTile; t0 < n; t0 += (int64_t)nblk * kQTile) {
        const int64_t t1 = min(t0 + kQTile, n);
        uint32_t mine = 0;
        for (int64_t v = t0 + threadIdx.x; v < t1; v += kBfsBlock)
            if (at_depth(v)) mine += chunks_of(rp[v + 1] - rp[v]);
        for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off, kWave);
        if (lane == 0) wsum[w] = mine;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (int i = 0; i < kBfsBlock / kWave; i++) tot += wsum[i];
            tile_base = tot ? atomicAdd(qcount, tot) : 0u;
        }
        __syncthreads();
        // second pass: ordered positions inside the tile, one 256-vertex step at a time
        uint32_t base = tile_base;
        for (int64_t v0 = t0; v0 < t1; v0 += kBfsBlock) {
            const int64_t v = v0 + threadIdx.x;
            const uint32_t k = (v < t1 && at_depth(v)) ? chunks_of(rp[v + 1] - rp[v]) : 0u;
            uint32_t x = k;   // inclusive scan over the workgroup: waves, then wave totals
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, kWave);
                if (lane >= off) x += y;
            }
            if (lane == kWave - 1) wsum[w] = x;
            __syncthreads();
            uint32_t before = 0, step = 0;
            for (int i = 0; i < kBfsBlock / kWave; i++) {
                if (i < w) before += wsum[i];
                step += wsum[i];
            }
            const uint32_t pos = base + before + x - k;
            for (uint32_t j = 0; j < k; j++) queue[pos + j] = ((uint64_t)(uint32_t)v << 32) | j;
            base += step;
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_level_queue(const int64_t *__restrict__ rp,
                                                               const int32_t *__restrict__ level, int64_t n,
                                                               int32_t depth, uint64_t *queue, uint32_t *qcount) {
    bfs_level_queue(rp, level, n, depth, queue, qcount, nullptr, blockIdx.x, gridDim.x);
}

// ---- device-driven levels ----------------------------------------------------------------
// The host-driven loop read the frontier counts back after every level to choose the
// direction: ~30-50 us of idle device per level (SYN-g500-22: ~7 levels, 0.48 ms per BFS of
// which ~0.25 ms kernels).  Here a one-thread plan kernel consumes the last level's counts,
// applies Beamer's rule and selects the level's kernels; the others exit at once.  The host
// queues levels in batches and reads the done flag one batch late.
struct BfsState {
    int32_t depth;
    int32_t mode;          // 0 done / idle, 1 top-down, 2 bottom-up
    int32_t done;
    int32_t started;
    int32_t qi;            // top-down input queue q[qi], its count qcnt[qi]
    int32_t have_queue;    // the frontier is in q[qi] (else only in `level`)
    int32_t need_queue;    // this top-down level first rebuilds q[qi] from `level`
    int32_t bottom_up;
    int32_t has_in;
    int32_t fbi;           // bottom-up reads frontier bitmap fb[fbi] and writes the next into fb[fbi ^ 1]
    int32_t fb_ready;      // fb[fbi] already holds this level's frontier (the last level was bottom-up)
    int32_t nextbits;      // bottom-up writes the next bitmap (GX_BFS_NEXTBITS, default on)
    int32_t qbits;         // a top-down queue rebuild reads that bitmap (GX_BFS_QBITS, default on)
    int32_t pad2;
    unsigned long long alpha, beta;   // Beamer's switch thresholds (GX_BFS_ALPHA / GX_BFS_BETA)
    unsigned long long mf, mu, fsize, n;
    uint32_t qcnt[2];
    unsigned long long nedges;
    unsigned long long bucnt[2];   // bottom-up: found, their out-edges
};

__global__ void k_bfs_plan(BfsState *st) {
    if (st->done) {
        st->mode = 0;
        return;
    }
    if (st->started) {   // the last level's results
        unsigned long long next_edges, next_size;
        if (st->mode == 2) {
            next_size = st->bucnt[0];
            next_edges = st->bucnt[1];
            st->have_queue = 0;
            if (st->nextbits) {
                st->fbi ^= 1;
                st->fb_ready = 1;
            }
        } else {
            st->fb_ready = 0;
            st->qi ^= 1;
            next_size = st->qcnt[st->qi];
            next_edges = st->nedges;
            st->have_queue = 1;
        }
        st->mu = st->mu > st->mf ? st->mu - st->mf : 0ull;
        st->mf = next_edges;
        st->fsize = next_size;
        st->depth++;
    }
    st->started = 1;
    if (st->fsize == 0) {
        st->done = 1;
        st->mode = 0;
        return;
    }
    // Beamer: TD -> BU when the frontier's edges exceed the unexplored ones / 14; BU -> TD when
    // the frontier shrinks below n / 24
    if (st->has_in) {
        if (!st->bottom_up && st->mf > st->mu / st->alpha) st->bottom_up = 1;
        else if (st->bottom_up && (long long)st->fsize < (long long)(st->n / st->beta)) st->bottom_up = 0;
    }
    if (st->bottom_up) {
        st->mode = 2;
        st->bucnt[0] = st->bucnt[1] = 0;
    } else {
        st->mode = 1;
        st->need_queue = !st->have_queue;
        if (st->need_queue) st->qcnt[st->qi] = 0;
        st->qcnt[st->qi ^ 1] = 0;
        st->nedges = 0;
    }
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_bitmap_dev(const int32_t *__restrict__ level, int64_t n,
                                                              const BfsState *st, uint64_t *fb0, uint64_t *fb1) {
    if (st->mode != 2 || st->fb_ready) return;
    bfs_bitmap(level, n, st->depth, st->fbi ? fb1 : fb0, blockIdx.x, gridDim.x);
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_bottomup_dev(const int64_t *__restrict__ rpi,
                                                                const int32_t *__restrict__ cii,
                                                                const int64_t *__restrict__ rpo,
                                                                uint64_t *fb0, uint64_t *fb1, int64_t n,
                                                                int32_t *level, BfsState *st) {
    if (st->mode != 2) return;
    const int i = st->fbi;
    bfs_bottomup(rpi, cii, rpo, i ? fb1 : fb0, n, level, st->depth, st->bucnt,
                 st->nextbits ? (i ? fb0 : fb1) : nullptr, blockIdx.x, gridDim.x);
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_level_queue_dev(const int64_t *__restrict__ rp,
                                                                   const int32_t *__restrict__ level, int64_t n,
                                                                   BfsState *st, uint64_t *q0, uint64_t *q1,
                                                                   const uint64_t *fb0, const uint64_t *fb1) {
    if (st->mode != 1 || !st->need_queue) return;
    const int qi = st->qi;
    bfs_level_queue(rp, level, n, st->depth, qi ? q1 : q0, &st->qcnt[qi],
                    st->fb_ready && st->qbits ? (st->fbi ? fb1 : fb0) : nullptr, blockIdx.x, gridDim.x);
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_topdown_dev(const int64_t *__restrict__ rp,
                                                               const int32_t *__restrict__ ci, int32_t *level,
                                                               BfsState *st, uint64_t *q0, uint64_t *q1) {
    if (st->mode != 1) return;
    const int qi = st->qi;
    bfs_topdown(rp, ci, qi ? q1 : q0, st->qcnt[qi], level, st->depth, qi ? q0 : q1, &st->qcnt[qi ^ 1],
                &st->nedges, blockIdx.x, gridDim.x);
}

// A level in two launches instead of four (GX_BFS_FUSED, the default): the frontier phase
// (bottom-up: the bitmap unless the last level left it; top-down: the queue rebuild when
// needed) and the expansion (bottom-up or top-down), each branching on the plan's mode, so
// the direction not taken costs no idle launch.  Blocks past a phase's own grid exit, and the
// phase runs on exactly the grid its separate kernel had.
__global__ __launch_bounds__(kBfsBlock) void k_bfs_frontier_dev(const int64_t *__restrict__ rp,
                                                                const int32_t *__restrict__ level, int64_t n,
                                                                BfsState *st, uint64_t *fb0, uint64_t *fb1,
                                                                uint64_t *q0, uint64_t *q1, uint32_t vgrid,
                                                                uint32_t qgrid) {
    const int mode = st->mode;
    if (mode == 2) {
        if (st->fb_ready || blockIdx.x >= vgrid) return;
        bfs_bitmap(level, n, st->depth, st->fbi ? fb1 : fb0, blockIdx.x, vgrid);
    } else if (mode == 1) {
        if (!st->need_queue || blockIdx.x >= qgrid) return;
        const int qi = st->qi;
        bfs_level_queue(rp, level, n, st->depth, qi ? q1 : q0, &st->qcnt[qi],
                        st->fb_ready && st->qbits ? (st->fbi ? fb1 : fb0) : nullptr, blockIdx.x, qgrid);
    }
}

__global__ __launch_bounds__(kBfsBlock) void k_bfs_expand_dev(const int64_t *__restrict__ rpi,
                                                              const int32_t *__restrict__ cii,
                                                              const int64_t *__restrict__ rp,
                                                              const int32_t *__restrict__ ci, int32_t *level,
                                                              int64_t n, BfsState *st, uint64_t *fb0, uint64_t *fb1,
                                                              uint64_t *q0, uint64_t *q1, uint32_t bu_grid,
                                                              uint32_t tgrid) {
    const int mode = st->mode;
    if (mode == 2) {
        if (blockIdx.x >= bu_grid) return;
        const int i = st->fbi;
        bfs_bottomup(rpi, cii, rp, i ? fb1 : fb0, n, level, st->depth, st->bucnt,
                     st->nextbits ? (i ? fb0 : fb1) : nullptr, blockIdx.x, bu_grid);
    } else if (mode == 1) {
        if (blockIdx.x >= tgrid) return;
        const int qi = st->qi;
        bfs_topdown(rp, ci, qi ? q1 : q0, st->qcnt[qi], level, st->depth, qi ? q0 : q1, &st->qcnt[qi ^ 1],
                    &st->nedges, blockIdx.x, tgrid);
    }
}

__global__ void k_bfs_seed(const int64_t *__restrict__ rp, int32_t *level, uint64_t *queue, uint32_t *qcount,
                           int32_t src) {
    level[src] = 0;
    const uint32_t nch = chunks_of(rp[src + 1] - rp[src]);
    for (uint32_t j = threadIdx.x; j < nch; j += blockDim.x) queue[j] = ((uint64_t)(uint32_t)src << 32) | j;
    if (threadIdx.x == 0) *qcount = nch;
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_bfs(gx_graph *g, uint64_t src, int64_t *level_out) {
    if (!g || !level_out) return fail(GX_NULL_POINTER, "gx_bfs: null argument");
    if (src >= g->n) return fail(GX_INVALID_INDEX, "gx_bfs: source out of range");
    {
        gx_graph *h = nullptr;   // hub-first copy from the second call (gx_runtime.hip hub_for)
        GX_TRY(hub_for(g, ++g->hub_bfs_calls, &h, &src));
        if (h) return gx_bfs(h, src, level_out);
    }
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    int64_t src_rp[2] = {0, 0};   // the source's out-degree (the host row pointers are lazy)
    GX_HIP_TRY(hipMemcpy(src_rp, g->A.rp.p + src, sizeof(src_rp), hipMemcpyDeviceToHost));
    const int64_t src_deg = src_rp[1] - src_rp[0];
    DBuf<int32_t> level;
    DBuf<uint64_t> q0, q1;
    DBuf<uint32_t> qcount;
    DBuf<unsigned long long> nedges;
    DBuf<uint64_t> fbits;
    DBuf<unsigned long long> bucnt;
    GX_TRY(fbits.alloc(2 * ((n + 63) / 64)));   // two bitmaps: the device-driven path alternates them
    uint64_t *const fb1 = fbits.p + (n + 63) / 64;
    GX_TRY(bucnt.alloc(2));
    const uint64_t qcap = (uint64_t)n + g->nnz / kChunk + 64;   // sum over vertices of ceil(deg / kChunk)
    GX_TRY(level.alloc(n));
    GX_TRY(q0.alloc(qcap));
    GX_TRY(q1.alloc(qcap));
    GX_TRY(qcount.alloc(1));
    GX_TRY(nedges.alloc(1));
    GX_TRY(device_begin(ctx));
    // in-edges: the graph itself when undirected; for a directed graph the transpose, built on
    // the device and cached once the graph serves a second BFS (a one-off run, like the
    // Graphalytics executable's, would not win back the build).  GX_BFS_TRANSPOSE = 0 never,
    // 1 from the second run (default), 2 from the first.
    g->bfs_calls++;
    if (g->directed && !g->AT.built) {
        const char *e = std::getenv("GX_BFS_TRANSPOSE");
        const int mode = e ? std::atoi(e) : 1;
        if (mode == 2 || (mode == 1 && g->bfs_calls >= 2)) GX_TRY(ensure_transpose(g));
    }
    const DevCSR *in = g->directed ? (g->AT.built ? &g->AT : nullptr) : &g->A;
    GX_HIP_TRY(hipMemsetAsync(level.p, 0xff, n * 4, s));
    const unsigned bu_grid = (unsigned)std::min<int64_t>(grid_for(n, kBfsBlock, 8192), 1024);
    const char *de = std::getenv("GX_BFS_DEVICE");
    if (!de || std::atoi(de) != 0) {
        // device-driven levels (k_bfs_plan), queued in batches; the done flag is read one
        // batch late
        DBuf<BfsState> st;
        GX_TRY(st.alloc(1));
        BfsState h{};
        const int64_t dsrc = src_deg;
        h.have_queue = 1;
        h.has_in = in != nullptr;
        h.n = (unsigned long long)n;
        h.mf = (unsigned long long)dsrc;
        h.mu = g->nnz;
        h.fsize = (unsigned long long)((dsrc + kChunk - 1) / kChunk);
        const char *nb = std::getenv("GX_BFS_NEXTBITS");
        h.nextbits = !nb || std::atoi(nb) != 0;
        const char *qb = std::getenv("GX_BFS_QBITS");
        h.qbits = !qb || std::atoi(qb) != 0;
        const char *ae = std::getenv("GX_BFS_ALPHA"), *be = std::getenv("GX_BFS_BETA");
        h.alpha = (unsigned long long)std::max(1, ae ? std::atoi(ae) : 14);
        // beta 48 on undirected graphs (SYN-7_5 0.203-0.209 -> 0.186-0.192 ms, SYN-g500-22 ~1 %),
        // 24 on directed ones (SYN-cit 2-6 % slower at 48): profiles/r05_bfs_beta_ab.txt
        h.beta = (unsigned long long)std::max(1, be ? std::atoi(be) : (g->directed ? 24 : 48));
        GX_HIP_TRY(hipMemcpyAsync(st.p, &h, sizeof(h), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_bfs_seed, dim3(1), dim3(256), 0, s, g->A.rp.p, level.p, q0.p, &st.p->qcnt[0],
                           (int32_t)src);
        GX_TRY(check_launch("k_bfs_seed"));
        int32_t *h_done = nullptr;
        hipEvent_t ev = nullptr;
        GX_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h_done), 4 * sizeof(int32_t), hipHostMallocDefault));
        std::unique_ptr<int32_t, void (*)(int32_t *)> done_guard(h_done, [](int32_t *p) { (void)hipHostFree(p); });
        GX_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        std::unique_ptr<ihipEvent_t, void (*)(hipEvent_t)> ev_guard(ev, [](hipEvent_t e) { (void)hipEventDestroy(e); });
        // grids of the kernels that run idle on the levels of the other direction: an idle
        // 8192-workgroup launch cost 2.6-3.0 us, a 2048 one 0.9 (r04_bfs_kernel_stats.csv);
        // every kernel is a grid-stride loop (GX_BFS_GRID overrides)
        const char *ge = std::getenv("GX_BFS_GRID");
        const unsigned gcap = ge ? (unsigned)std::max(1, std::atoi(ge)) : 2048u;
        const unsigned vgrid = grid_for(n, kBfsBlock, gcap);
        const unsigned tgrid = std::min(8192u, gcap);
        const unsigned qgrid = (unsigned)std::min<int64_t>((n + kQTile - 1) / kQTile, 2048);
        const char *fe = std::getenv("GX_BFS_FUSED");
        const bool fused = !fe || std::atoi(fe) != 0;
        auto enqueue = [&](int k) -> int {
            for (int i = 0; i < k; i++) {
                hipLaunchKernelGGL(k_bfs_plan, dim3(1), dim3(1), 0, s, st.p);
                if (fused) {
                    if (in) {
                        KTimer kt(ctx, "bfs_frontier", s);
                        hipLaunchKernelGGL(k_bfs_frontier_dev, dim3(std::max(vgrid, qgrid)), dim3(kBfsBlock), 0, s,
                                           g->A.rp.p, level.p, n, st.p, fbits.p, fb1, q0.p, q1.p, vgrid, qgrid);
                    }
                    KTimer kt(ctx, "bfs_expand", s);
                    hipLaunchKernelGGL(k_bfs_expand_dev, dim3(std::max(in ? bu_grid : 0u, tgrid)), dim3(kBfsBlock), 0,
                                       s, in ? in->rp.p : nullptr, in ? in->ci.p : nullptr, g->A.rp.p, g->A.ci.p,
                                       level.p, n, st.p, fbits.p, fb1, q0.p, q1.p, in ? bu_grid : 0u, tgrid);
                    continue;
                }
                if (in) {
                    KTimer kt(ctx, "bfs_bottomup", s);
                    hipLaunchKernelGGL(k_bfs_bitmap_dev, dim3(vgrid), dim3(kBfsBlock), 0, s, level.p, n, st.p,
                                       fbits.p, fb1);
                    hipLaunchKernelGGL(k_bfs_bottomup_dev, dim3(bu_grid), dim3(kBfsBlock), 0, s, in->rp.p, in->ci.p,
                                       g->A.rp.p, fbits.p, fb1, n, level.p, st.p);
                }
                KTimer kt(ctx, "bfs_topdown", s);
                if (in)
                    hipLaunchKernelGGL(k_bfs_level_queue_dev, dim3(qgrid), dim3(kBfsBlock), 0, s, g->A.rp.p, level.p,
                                       n, st.p, q0.p, q1.p, fbits.p, fb1);
                hipLaunchKernelGGL(k_bfs_topdown_dev, dim3(tgrid), dim3(kBfsBlock), 0, s, g->A.rp.p, g->A.ci.p,
                                   level.p, st.p, q0.p, q1.p);
            }
            return check_launch("k_bfs_topdown_dev");
        };
        // A first batch of levels, then batches of kBatch with the done flag read one batch
        // late; a level queued past the end costs ~20 us (five launches that exit at once).
        // The first batch is the number of steps the last BFS on this graph took (a repeated
        // or nearby source needs the same: SYN-g500-22 8), else kFirst; when it was enough,
        // the host waits for it and queues nothing more.
        // The hint is capped (kMaxFirst): after a deep BFS (a long chain) a shallow one would
        // otherwise queue thousands of idle levels at ~20 us each.
        constexpr int kFirst = 6, kBatch = 2, kMaxFirst = 24;
        const int first = g->bfs_steps_hint > 0 ? std::min(g->bfs_steps_hint, kMaxFirst) : kFirst;
        // h_done[0..2] = depth, mode, done of the state (one copy)
        auto read_state = [&]() -> int {
            GX_HIP_TRY(hipMemcpyAsync(h_done, &st.p->depth, 3 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipEventRecord(ev, s));
            return GX_SUCCESS;
        };
        const void *res = nullptr;
        GX_TRY(enqueue(first));
        int64_t levels = first;
        GX_TRY(read_state());
        if (g->bfs_steps_hint > 0) {
            // the results' remap is queued behind the levels it expects to be the last, so it
            // runs while the host reads the flag (queued again below if they were not)
            GX_TRY(remap_out(g, level.p, 4, s, &res));
            GX_HIP_TRY(hipEventSynchronize(ev));
        } else {
            GX_TRY(enqueue(kBatch));
            levels += kBatch;
            GX_HIP_TRY(hipEventSynchronize(ev));
        }
        const bool more = !h_done[2];
        while (!h_done[2]) {
            GX_TRY(read_state());
            GX_TRY(enqueue(kBatch));
            levels += kBatch;
            GX_HIP_TRY(hipEventSynchronize(ev));
            if (levels > n + 2 * kFirst + 8) return fail(GX_PANIC, "gx_bfs: level loop did not end");
        }
        // steps this BFS needed: its levels plus the plan step that found the frontier empty
        g->bfs_steps_hint = h_done[0] + 1;
        if (!res || more) GX_TRY(remap_out(g, level.p, 4, s, &res));
        GX_TRY(device_end(ctx));
        GX_TRY(download(ctx, level_out, res, (uint64_t)n, Xfer::Levels));
        return GX_SUCCESS;
    }
    hipLaunchKernelGGL(k_bfs_seed, dim3(1), dim3(256), 0, s, g->A.rp.p, level.p, q0.p, qcount.p, (int32_t)src);
    GX_TRY(check_launch("k_bfs_seed"));
    uint32_t qsize = 0;
    GX_HIP_TRY(hipMemcpyAsync(&qsize, qcount.p, 4, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    unsigned long long mf = (unsigned long long)src_deg;
    unsigned long long mu = g->nnz;
    bool bottom_up = false;
    int32_t depth = 0;
    struct Counters {
        uint32_t q;
        uint32_t pad;
        unsigned long long e;
    };
    // frontier: qsize vertices (top-down steps keep them as work items in q0; after a
    // bottom-up step they are only in `level` until a top-down step needs the queue)
    bool have_queue = true;
    uint64_t fsize = qsize;
    while (fsize > 0) {
        // Beamer switch: TD -> BU when the frontier's edges exceed the unexplored ones / 14;
        // BU -> TD when the frontier shrinks below n / 24.
        if (in) {
            if (!bottom_up && mf > mu / 14) bottom_up = true;
            else if (bottom_up && (int64_t)fsize < n / 24) bottom_up = false;
        }
        unsigned long long next_edges = 0;
        uint64_t next_size = 0;
        if (bottom_up) {
            KTimer kt(ctx, "bfs_bottomup", s);
            GX_HIP_TRY(hipMemsetAsync(bucnt.p, 0, 16, s));
            hipLaunchKernelGGL(k_bfs_bitmap, dim3(grid_for(n, kBfsBlock, 8192)), dim3(kBfsBlock), 0, s, level.p, n,
                               depth, fbits.p);
            hipLaunchKernelGGL(k_bfs_bottomup, dim3(bu_grid), dim3(kBfsBlock), 0, s, in->rp.p, in->ci.p, g->A.rp.p,
                               fbits.p, n, level.p, depth, bucnt.p);
            GX_TRY(check_launch("k_bfs_bottomup"));
            unsigned long long c[2] = {0, 0};
            GX_HIP_TRY(hipMemcpyAsync(c, bucnt.p, 16, hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            next_size = c[0];
            next_edges = c[1];
            have_queue = false;
        } else {
            KTimer kt(ctx, "bfs_topdown", s);
            if (!have_queue) {
                GX_HIP_TRY(hipMemsetAsync(qcount.p, 0, 4, s));
                hipLaunchKernelGGL(k_bfs_level_queue, dim3((unsigned)std::min<int64_t>((n + kQTile - 1) / kQTile, 2048)),
                                   dim3(kBfsBlock), 0, s, g->A.rp.p, level.p, n, depth, q0.p, qcount.p);
                GX_TRY(check_launch("k_bfs_level_queue"));
                GX_HIP_TRY(hipMemcpyAsync(&qsize, qcount.p, 4, hipMemcpyDeviceToHost, s));
                GX_HIP_TRY(hipStreamSynchronize(s));
                have_queue = true;
            }
            GX_HIP_TRY(hipMemsetAsync(qcount.p, 0, 4, s));
            GX_HIP_TRY(hipMemsetAsync(nedges.p, 0, 8, s));
            hipLaunchKernelGGL(k_bfs_topdown, dim3(grid_for((uint64_t)qsize * kWave, kBfsBlock, 8192)),
                               dim3(kBfsBlock), 0, s, g->A.rp.p, g->A.ci.p, q0.p, qsize, level.p, depth, q1.p,
                               qcount.p, nedges.p);
            GX_TRY(check_launch("k_bfs_topdown"));
            Counters c{};
            GX_HIP_TRY(hipMemcpyAsync(&c.q, qcount.p, 4, hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipMemcpyAsync(&c.e, nedges.p, 8, hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            qsize = c.q;
            next_size = c.q;   // work items (~ vertices; a hub counts once per 256 edges)
            next_edges = c.e;
            std::swap(q0.p, q1.p);
        }
        mu = mu > mf ? mu - mf : 0;
        mf = next_edges;
        fsize = next_size;
        depth++;
    }
    const void *res = nullptr;
    GX_TRY(remap_out(g, level.p, 4, s, &res));
    GX_TRY(device_end(ctx));
    GX_TRY(download(ctx, level_out, res, (uint64_t)n, Xfer::Levels));
    return GX_SUCCESS;
}

GX_MODULE_WARMER(bfs)
