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

// Sparse exchange (gx_part_changes / gx_part_apply): a tile of kChTile entries per workgroup
// pass, 16 per thread, one counter atomic per tile (a queue atomic per wave serialised at
// ~11 ns each).  A change leaves as one 64-bit word (v << 32 | value).
constexpr int kChPer = 16;
constexpr int kChTile = kPartBlock * kChPer;

template <typename T>
__global__ __launch_bounds__(kPartBlock) void k_part_changes(const T *__restrict__ a, const T *__restrict__ b,
                                                             int64_t v0, int64_t v1, uint64_t *__restrict__ out,
                                                             unsigned long long *count) {
    __shared__ uint32_t wsum[kPartBlock / kWave];
    __shared__ unsigned long long base;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    for (int64_t t0 = v0 + (int64_t)blockIdx.x * kChTile; t0 < v1; t0 += (int64_t)gridDim.x * kChTile) {
        uint32_t flags = 0, c = 0;
#pragma unroll
        for (int j = 0; j < kChPer; j++) {
            const int64_t v = t0 + tid + (int64_t)j * kPartBlock;
            if (v < v1 && a[v] != (b ? b[v] : (T)0)) {
                flags |= 1u << j;
                c++;
            }
        }
        uint32_t incl = c;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, kWave);
            if (lane >= off) incl += y;
        }
        if (lane == kWave - 1) wsum[wid] = incl;
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kPartBlock / kWave; w++) {
            before += w < wid ? wsum[w] : 0u;
            total += wsum[w];
        }
        if (tid == 0) base = total ? atomicAdd(count, (unsigned long long)total) : 0ull;
        __syncthreads();
        uint64_t at = base + before + incl - c;
        for (int j = 0; j < kChPer; j++)
            if (flags & (1u << j)) {
                const int64_t v = t0 + tid + (int64_t)j * kPartBlock;
                out[at++] = ((uint64_t)v << 32) | (uint32_t)a[v];
            }
        __syncthreads();   // wsum / base reused by the next tile
    }
}

// op 0 set, 1 min, 2 max (int32 only for 1 / 2); rank k's count[k] words at words + k * stride
template <typename T>
__global__ __launch_bounds__(kPartBlock) void k_part_apply(const uint64_t *__restrict__ words,
                                                           const int64_t *__restrict__ counts, int nranks,
                                                           int64_t stride, T *arr, int op) {
    const int64_t total = (int64_t)nranks * stride;
    for (int64_t i = (int64_t)blockIdx.x * kPartBlock + threadIdx.x; i < total; i += (int64_t)gridDim.x * kPartBlock) {
        const int64_t k = i / stride, j = i - k * stride;
        if (j >= counts[k]) continue;
        const uint64_t w = words[i];
        const int64_t v = (int64_t)(w >> 32);
        const T val = (T)(uint32_t)w;
        if constexpr (sizeof(T) == 4) {
            if (op == 1) atomicMin((int32_t *)&arr[v], (int32_t)val);
            else if (op == 2) atomicMax((int32_t *)&arr[v], (int32_t)val);
            else arr[v] = val;
        } else {
            arr[v] = val;
        }
    }
}

// BFS's dense exchange as bits: next (one byte per vertex) -> one bit per vertex, and the
// ranks' gathered bitmaps OR-ed back into next.  A thread per 32-bit word.
__global__ __launch_bounds__(kPartBlock) void k_part_pack_bits(const uint8_t *__restrict__ next, int64_t n,
                                                               uint32_t *__restrict__ bits) {
    const int64_t nw = (n + 31) / 32;
    for (int64_t w = (int64_t)blockIdx.x * kPartBlock + threadIdx.x; w < nw; w += (int64_t)gridDim.x * kPartBlock) {
        uint32_t b = 0;
        const int64_t v0 = w * 32;
        if (v0 + 32 <= n) {
            const uint4 *q = reinterpret_cast<const uint4 *>(next + v0);   // next is 16-B aligned (tensor)
            const uint4 a = q[0], c = q[1];
            const uint32_t x[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
            for (int j = 0; j < 32; j++) b |= (uint32_t)(((x[j >> 2] >> (8 * (j & 3))) & 0xffu) != 0) << j;
        } else {
            for (int64_t v = v0; v < n; v++) b |= (uint32_t)(next[v] != 0) << (v - v0);
        }
        bits[w] = b;
    }
}

__global__ __launch_bounds__(kPartBlock) void k_part_or_bits(const uint32_t *__restrict__ gathered, int nranks,
                                                             int64_t n, uint8_t *__restrict__ next) {
    const int64_t nw = (n + 31) / 32;
    for (int64_t v = (int64_t)blockIdx.x * kPartBlock + threadIdx.x; v < n; v += (int64_t)gridDim.x * kPartBlock) {
        uint32_t any = 0;
        for (int r = 0; r < nranks; r++) any |= gathered[(int64_t)r * nw + v / 32] >> (v & 31);
        next[v] = (uint8_t)(any & 1u);
    }
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

// Sparse exchange of a partitioned step's updates (distributed.py: BFS's discoveries, WCC's
// hooked roots, CDLP's new labels at N > 1, when they are fewer than a dense collective moves).
extern "C" int gx_part_changes(const void *a, const void *b, uint64_t v0, uint64_t v1, int elem_bytes,
                               uint64_t *words, int64_t *count, void *stream) {
    if (!a || !words || !count) return fail(GX_NULL_POINTER, "gx_part_changes: null argument");
    if (v0 > v1 || v1 >= (1ull << 31)) return fail(GX_INVALID_INDEX, "gx_part_changes: bad vertex range");
    if (elem_bytes != 1 && elem_bytes != 4) return fail(GX_INVALID_VALUE, "gx_part_changes: elements of 1 or 4 bytes");
    hipStream_t s = (hipStream_t)stream;
    GX_HIP_TRY(hipMemsetAsync(count, 0, sizeof(int64_t), s));
    if (v1 == v0) return GX_SUCCESS;
    const dim3 grid(grid_for((v1 - v0 + kChPer - 1) / kChPer, kPartBlock, 4096));
    if (elem_bytes == 1)
        hipLaunchKernelGGL(k_part_changes<uint8_t>, grid, dim3(kPartBlock), 0, s, (const uint8_t *)a,
                           (const uint8_t *)b, (int64_t)v0, (int64_t)v1, words, (unsigned long long *)count);
    else
        hipLaunchKernelGGL(k_part_changes<int32_t>, grid, dim3(kPartBlock), 0, s, (const int32_t *)a,
                           (const int32_t *)b, (int64_t)v0, (int64_t)v1, words, (unsigned long long *)count);
    return check_launch("k_part_changes");
}

extern "C" int gx_part_apply(const uint64_t *words, const int64_t *counts, int nranks, uint64_t stride, void *arr,
                             int elem_bytes, int op, void *stream) {
    if (!words || !counts || !arr) return fail(GX_NULL_POINTER, "gx_part_apply: null argument");
    if (nranks < 1) return fail(GX_INVALID_VALUE, "gx_part_apply: nranks < 1");
    if (elem_bytes != 1 && elem_bytes != 4) return fail(GX_INVALID_VALUE, "gx_part_apply: elements of 1 or 4 bytes");
    if (op < 0 || op > 2 || (elem_bytes == 1 && op != 0))
        return fail(GX_INVALID_VALUE, "gx_part_apply: op 0 (set), or 1 / 2 (min / max) on 4-byte elements");
    if (stride == 0) return GX_SUCCESS;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(grid_for((uint64_t)nranks * stride, kPartBlock, 8192));
    if (elem_bytes == 1)
        hipLaunchKernelGGL(k_part_apply<uint8_t>, grid, dim3(kPartBlock), 0, s, words, counts, nranks, (int64_t)stride,
                           (uint8_t *)arr, op);
    else
        hipLaunchKernelGGL(k_part_apply<int32_t>, grid, dim3(kPartBlock), 0, s, words, counts, nranks, (int64_t)stride,
                           (int32_t *)arr, op);
    return check_launch("k_part_apply");
}

extern "C" int gx_part_pack_bits(const uint8_t *next, uint64_t n, uint32_t *bits, void *stream) {
    if (!next || !bits) return fail(GX_NULL_POINTER, "gx_part_pack_bits: null argument");
    if ((reinterpret_cast<uintptr_t>(next) & 15) != 0) return fail(GX_INVALID_VALUE, "gx_part_pack_bits: next not 16-B aligned");
    if (n == 0) return GX_SUCCESS;
    hipLaunchKernelGGL(k_part_pack_bits, dim3(grid_for((n + 31) / 32, kPartBlock, 8192)), dim3(kPartBlock), 0,
                       (hipStream_t)stream, next, (int64_t)n, bits);
    return check_launch("k_part_pack_bits");
}

extern "C" int gx_part_or_bits(const uint32_t *gathered, int nranks, uint64_t n, uint8_t *next, void *stream) {
    if (!gathered || !next) return fail(GX_NULL_POINTER, "gx_part_or_bits: null argument");
    if (nranks < 1) return fail(GX_INVALID_VALUE, "gx_part_or_bits: nranks < 1");
    if (n == 0) return GX_SUCCESS;
    hipLaunchKernelGGL(k_part_or_bits, dim3(grid_for(n, kPartBlock, 8192)), dim3(kPartBlock), 0, (hipStream_t)stream,
                       gathered, nranks, (int64_t)n, next);
    return check_launch("k_part_or_bits");
}
