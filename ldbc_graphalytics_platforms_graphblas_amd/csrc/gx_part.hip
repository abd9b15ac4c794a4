// gx_part.hip -- per-rank steps of the multi-GPU BFS and WCC (SSSP's 1-D split
// is gx_sssp_split.hip).
//
// The graph is replicated on every rank (it fits: 8_5-fb is ~8 GB of CSR against 288 GB of
// HBM); ranks own contiguous vertex ranges [v0, v1) balanced by stored entries and work
// on the rows they own.  State arrays are full length on every rank and the caller makes
// them agree with one RCCL collective per round (torch.distributed over xGMI):
//   BFS  : expand owned frontier rows into `next` (one byte per vertex)   -> all-reduce MAX
//          commit: level[v] = cur+1 for newly reached v (every rank, same result)
//   WCC  : hook the edges of owned rows into the parent forest             -> all-reduce MIN
//          compress (pointer jumping) on every rank
// The reference has no distributed path ("Collective call sites: none").
// Results equal the single-GPU ones: BFS levels and WCC min-root labels are unique.
#include "gx_device.h"

namespace gx {
namespace {

constexpr int kPartBlock = 256;
constexpr int64_t kInfLevel = INT64_MAX;

// Visit the owned vertices [v0, v1) 64 at a time; `pick` selects the ones whose out-edges the
// wave then walks together (lane-strided), calling `edge(u, v, k)` for each.
template <class Pick, class Edge>
__device__ __forceinline__ void for_owned_rows(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                               int64_t v0, int64_t v1, Pick pick, Edge edge) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kPartBlock + threadIdx.x) / kWave;
    const int64_t nw = (int64_t)gridDim.x * (kPartBlock / kWave);
    for (int64_t base = v0 + wave * kWave; base < v1; base += nw * kWave) {
        const int64_t u_l = base + lane;
        uint64_t m = __ballot(u_l < v1 && pick(u_l));
        while (m) {
            const int j = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const int64_t u = base + j;
            for (int64_t k = rp[u] + lane; k < rp[u + 1]; k += kWave) edge(u, (int64_t)ci[k], k);
        }
    }
}

__global__ __launch_bounds__(kPartBlock) void k_bfsp_init(int64_t *level, int64_t n, int64_t src) {
    for (int64_t v = (int64_t)blockIdx.x * kPartBlock + threadIdx.x; v < n; v += (int64_t)gridDim.x * kPartBlock)
        level[v] = v == src ? 0 : kInfLevel;
}

__global__ __launch_bounds__(kPartBlock) void k_bfsp_expand(const int64_t *__restrict__ rp,
                                                            const int32_t *__restrict__ ci, int64_t v0, int64_t v1,
                                                            const int64_t *__restrict__ level, int64_t cur,
                                                            uint8_t *next) {
    for_owned_rows(
        rp, ci, v0, v1, [&](int64_t u) { return level[u] == cur; },
        [&](int64_t, int64_t v, int64_t) {
            if (level[v] == kInfLevel) next[v] = 1;
        });
}

__global__ __launch_bounds__(kPartBlock) void k_bfsp_commit(const uint8_t *__restrict__ next, int64_t *level,
                                                            int64_t n, int64_t nxt_level, unsigned long long *count) {
    unsigned long long c = 0;
    for (int64_t v = (int64_t)blockIdx.x * kPartBlock + threadIdx.x; v < n; v += (int64_t)gridDim.x * kPartBlock) {
        if (next[v] && level[v] == kInfLevel) {
            level[v] = nxt_level;
            c++;
        }
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0 && c) atomicAdd(count, c);
}

__global__ __launch_bounds__(kPartBlock) void k_wccp_init(int32_t *parent, int64_t n) {
    for (int64_t v = (int64_t)blockIdx.x * kPartBlock + threadIdx.x; v < n; v += (int64_t)gridDim.x * kPartBlock)
        parent[v] = (int32_t)v;
}

__device__ __forceinline__ int32_t find_root_p(const int32_t *parent, int32_t v) {
    int32_t p = parent[v];
    while (p != v) {
        v = p;
        p = parent[v];
    }
    return v;
}

// Edge-balanced hooking over the entries [e0, e1) (the owned rows' edges).
__global__ __launch_bounds__(kPartBlock) void k_wccp_hook(const int64_t *__restrict__ rp,
                                                          const int32_t *__restrict__ ci, int64_t n, int64_t e0,
                                                          int64_t e1, int32_t *parent, int *changed) {
    constexpr int kPer = 16;
    const int64_t c0 = e0 + ((int64_t)blockIdx.x * kPartBlock + threadIdx.x) * kPer;
    bool any = false;
    if (c0 < e1) {
        const int64_t c1 = min(c0 + kPer, e1);
        int64_t r = row_of_edge(rp, n, c0);
        for (int64_t e = c0; e < c1; e++) {
            while (rp[r + 1] <= e) r++;
            const int32_t ru = find_root_p(parent, (int32_t)r), rv = find_root_p(parent, ci[e]);
            if (ru != rv) {
                atomicMin(&parent[max(ru, rv)], min(ru, rv));
                any = true;
            }
        }
    }
    if (__ballot(any) && (threadIdx.x & (kWave - 1)) == 0) raise_flag(changed);
}

__global__ __launch_bounds__(kPartBlock) void k_wccp_compress(int32_t *parent, int64_t n) {
    for (int64_t v = (int64_t)blockIdx.x * kPartBlock + threadIdx.x; v < n; v += (int64_t)gridDim.x * kPartBlock)
        parent[v] = find_root_p(parent, (int32_t)v);
}

// NULL is the null (default) stream -- torch's default stream -- not the context's stream.
hipStream_t pick_stream(gx_graph *, void *stream) { return (hipStream_t)stream; }

int check_range(gx_graph *g, uint64_t v0, uint64_t v1, const char *who) {
    if (v0 > v1 || v1 > g->n) return fail(GX_INVALID_INDEX, std::string(who) + ": bad vertex range");
    return GX_SUCCESS;
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_bfs_part_init(gx_graph *g, uint64_t src, int64_t *level, void *stream) {
    if (!g || !level) return fail(GX_NULL_POINTER, "gx_bfs_part_init: null argument");
    if (src >= g->n) return fail(GX_INVALID_INDEX, "gx_bfs_part_init: source out of range");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipLaunchKernelGGL(k_bfsp_init, dim3(grid_for(g->n, kPartBlock, 8192)), dim3(kPartBlock), 0,
                       pick_stream(g, stream), level, (int64_t)g->n, (int64_t)src);
    return check_launch("k_bfsp_init");
}

extern "C" int gx_bfs_part_expand(gx_graph *g, uint64_t v0, uint64_t v1, const int64_t *level, int64_t cur,
                                  uint8_t *next, void *stream) {
    if (!g || !level || !next) return fail(GX_NULL_POINTER, "gx_bfs_part_expand: null argument");
    GX_TRY(check_range(g, v0, v1, "gx_bfs_part_expand"));
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    if (v1 > v0)
        hipLaunchKernelGGL(k_bfsp_expand, dim3(grid_for(v1 - v0, kPartBlock, 8192)), dim3(kPartBlock), 0,
                           pick_stream(g, stream), g->A.rp.p, g->A.ci.p, (int64_t)v0, (int64_t)v1, level, cur, next);
    return check_launch("k_bfsp_expand");
}

extern "C" int gx_bfs_part_commit(gx_graph *g, const uint8_t *next, int64_t *level, int64_t cur, uint64_t *count,
                                  void *stream) {
    if (!g || !next || !level || !count) return fail(GX_NULL_POINTER, "gx_bfs_part_commit: null argument");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipLaunchKernelGGL(k_bfsp_commit, dim3(grid_for(g->n, kPartBlock, 8192)), dim3(kPartBlock), 0,
                       pick_stream(g, stream), next, level, (int64_t)g->n, cur + 1, (unsigned long long *)count);
    return check_launch("k_bfsp_commit");
}

extern "C" int gx_wcc_part_init(gx_graph *g, int32_t *parent, void *stream) {
    if (!g || !parent) return fail(GX_NULL_POINTER, "gx_wcc_part_init: null argument");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipLaunchKernelGGL(k_wccp_init, dim3(grid_for(g->n, kPartBlock, 8192)), dim3(kPartBlock), 0,
                       pick_stream(g, stream), parent, (int64_t)g->n);
    return check_launch("k_wccp_init");
}

extern "C" int gx_wcc_part_hook(gx_graph *g, uint64_t v0, uint64_t v1, int32_t *parent, int *changed,
                                void *stream) {
    if (!g || !parent || !changed) return fail(GX_NULL_POINTER, "gx_wcc_part_hook: null argument");
    GX_TRY(check_range(g, v0, v1, "gx_wcc_part_hook"));
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipStream_t s = pick_stream(g, stream);
    GX_TRY(ensure_host_rp(g->ctx, g->A));
    const int64_t e0 = g->A.h_rp[v0], e1 = g->A.h_rp[v1];
    if (e1 > e0)
        hipLaunchKernelGGL(k_wccp_hook, dim3(grid_for((uint64_t)((e1 - e0 + 15) / 16), kPartBlock, 1u << 30)),
                           dim3(kPartBlock), 0, s, g->A.rp.p, g->A.ci.p, (int64_t)g->n, e0, e1, parent, changed);
    GX_TRY(check_launch("k_wccp_hook"));
    hipLaunchKernelGGL(k_wccp_compress, dim3(grid_for(g->n, kPartBlock, 8192)), dim3(kPartBlock), 0, s, parent,
                       (int64_t)g->n);
    return check_launch("k_wccp_compress");
}

extern "C" int gx_wcc_part_compress(gx_graph *g, int32_t *parent, void *stream) {
    if (!g || !parent) return fail(GX_NULL_POINTER, "gx_wcc_part_compress: null argument");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipLaunchKernelGGL(k_wccp_compress, dim3(grid_for(g->n, kPartBlock, 8192)), dim3(kPartBlock), 0,
                       pick_stream(g, stream), parent, (int64_t)g->n);
    return check_launch("k_wccp_compress");
}

GX_MODULE_WARMER(part)
