// gx_sssp.hip -- single-source shortest paths, frontier Bellman-Ford (min.plus relaxations).
//
// Replaces LA_SSSP -> diagonal fill + LAGraph_Cached_EMin + LAGr_SingleSourceShortestPath
// with delta = 2.5 (sssp.cpp:53-81).  The zero diagonal the reference inserts cannot change a
// distance and is not materialised.
// Distances are non-negative fp64 kept as their IEEE bit patterns, whose unsigned order is
// the numeric order, so a relaxation is one 64-bit atomicMin.  Every round relaxes the
// out-edges of the vertices improved in the previous round (one wave per frontier vertex);
// a per-round stamp puts a vertex into the next frontier once.  The fixed point is the
// minimum over paths of the left-to-right fp64 path sum -- the same value Dijkstra and
// delta-stepping produce -- so the result is bitwise equal to the oracle.
#include <cmath>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kSsspBlock = 256;

__device__ __forceinline__ unsigned long long dbits(double d) {
    return (unsigned long long)__double_as_longlong(d);
}

__global__ __launch_bounds__(kSsspBlock) void k_sssp_relax(const int64_t *__restrict__ rp,
                                                           const int32_t *__restrict__ ci,
                                                           const double *__restrict__ w,
                                                           const int32_t *__restrict__ qin,
                                                           uint32_t qsize, unsigned long long *dist,
                                                           int32_t *stamp, int32_t round,
                                                           int32_t *qout, uint32_t *qcount) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = (blockIdx.x * kSsspBlock + threadIdx.x) / kWave;
    const uint32_t nwaves = gridDim.x * (kSsspBlock / kWave);
    for (uint32_t f = wave; f < qsize; f += nwaves) {
        const int32_t u = qin[f];
        const double du = __longlong_as_double((long long)__hip_atomic_load(
            &dist[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const int64_t b = rp[u], e = rp[u + 1];
        for (int64_t k0 = b; k0 < e; k0 += kWave) {
            const int64_t k = k0 + lane;
            bool take = false;
            int32_t v = 0;
            if (k < e) {
                v = ci[k];
                const unsigned long long nd = dbits(du + w[k]);
                if (nd < __hip_atomic_load(&dist[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    const unsigned long long old = atomicMin(&dist[v], nd);
                    if (nd < old && atomicExch(&stamp[v], round) != round) take = true;
                }
            }
            const uint64_t mask = __ballot(take);
            if (mask) {
                const int leader = __ffsll((unsigned long long)mask) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(qcount, (uint32_t)__popcll(mask));
                base = __shfl(base, leader, kWave);
                if (take) qout[base + __popcll(mask & ((1ull << lane) - 1))] = v;
            }
        }
    }
}

__global__ void k_sssp_init(unsigned long long *dist, int32_t *stamp, int64_t n, int32_t src,
                            int32_t *queue) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x) {
        dist[v] = v == src ? 0ull : 0x7FF0000000000000ull;   // +infinity
        stamp[v] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) queue[0] = src;
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_sssp(gx_graph *g, uint64_t src, double *dist_out) {
    if (!g || !dist_out) return fail(GX_NULL_POINTER, "gx_sssp: null argument");
    if (!g->weighted) return fail(GX_INVALID_VALUE, "gx_sssp: graph has no edge weights");
    if (src >= g->n) return fail(GX_INVALID_INDEX, "gx_sssp: source out of range");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    DBuf<unsigned long long> dist;
    DBuf<int32_t> stamp, q0, q1;
    DBuf<uint32_t> qcount;
    GX_TRY(dist.alloc(n));
    GX_TRY(stamp.alloc(n));
    GX_TRY(q0.alloc(n));
    GX_TRY(q1.alloc(n));
    GX_TRY(qcount.alloc(1));
    GX_TRY(device_begin(ctx));
    hipLaunchKernelGGL(k_sssp_init, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, dist.p, stamp.p, n,
                       (int32_t)src, q0.p);
    GX_TRY(check_launch("k_sssp_init"));
    uint32_t qsize = 1;
    for (int32_t round = 1; qsize > 0; round++) {
        GX_HIP_TRY(hipMemsetAsync(qcount.p, 0, 4, s));
        {
            KTimer kt(ctx, "sssp_relax", s);
            hipLaunchKernelGGL(k_sssp_relax, dim3(grid_for((uint64_t)qsize * kWave, kSsspBlock, 8192)),
                               dim3(kSsspBlock), 0, s, g->A.rp.p, g->A.ci.p, g->A.w.p, q0.p, qsize, dist.p,
                               stamp.p, round, q1.p, qcount.p);
        }
        GX_TRY(check_launch("k_sssp_relax"));
        GX_HIP_TRY(hipMemcpyAsync(&qsize, qcount.p, 4, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        std::swap(q0.p, q1.p);
    }
    GX_TRY(device_end(ctx));
    GX_HIP_TRY(hipMemcpy(dist_out, dist.p, n * 8, hipMemcpyDeviceToHost));
    return GX_SUCCESS;
}
