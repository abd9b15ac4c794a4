// gx_lcc.hip -- local clustering coefficient via degree-oriented triangle enumeration.
//
// Replaces LA_LCC -> LAGraph_lcc(&d, A, symmetric = !directed) (lcc.cpp:61-71), which
// SuiteSparse runs as a masked SpGEMM (C<S> = S*S-type, PLUS_PAIR) plus reductions.
// With N(v) = in(v) U out(v) (the undirected closure S, built on the device) and
// k = |N(v)|:
//     LCC(v) = #{(u, w) in E : u, w in N(v)} / (k (k - 1)),   0 when k < 2.
// Each triangle {a, b, c} of S contributes to a the number of stored directions between b
// and c (1 or 2: the popcount of that S entry's flag byte), and likewise for b and c.
// Triangles are enumerated once each on the degree-ordered orientation of S (edge v->u
// when (deg u, u) > (deg v, v)): for every oriented edge (v, u) the sorted lists O(v) and
// O(u) are merge-intersected; counts are exact 64-bit integer atomics, so the result is
// deterministic and equal to the oracle bit for bit (one fp64 division per vertex).
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kLccBlock = 256;
constexpr int kLccEdgesPerThread = 4;

__device__ __forceinline__ bool ranks_above(int64_t du, int32_t u, int64_t dv, int32_t v) {
    return du > dv || (du == dv && u > v);
}

__global__ void k_orient_count(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, int64_t n,
                               int64_t *__restrict__ cnt) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t dv = rp[v + 1] - rp[v];
        int64_t c = 0;
        for (int64_t k = rp[v]; k < rp[v + 1]; k++) {
            const int32_t u = ci[k];
            if (ranks_above(rp[u + 1] - rp[u], u, dv, (int32_t)v)) c++;
        }
        cnt[v] = c;
    }
}

__global__ void k_orient_fill(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                              const uint8_t *__restrict__ fl, int64_t n, const int64_t *__restrict__ orp,
                              int32_t *__restrict__ oci, uint8_t *__restrict__ ofl) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t dv = rp[v + 1] - rp[v];
        int64_t o = orp[v];
        for (int64_t k = rp[v]; k < rp[v + 1]; k++) {
            const int32_t u = ci[k];
            if (ranks_above(rp[u + 1] - rp[u], u, dv, (int32_t)v)) {
                oci[o] = u;
                ofl[o] = fl[k];
                o++;
            }
        }
    }
}

__global__ __launch_bounds__(kLccBlock) void k_lcc_triangles(const int64_t *__restrict__ orp,
                                                             const int32_t *__restrict__ oci,
                                                             const uint8_t *__restrict__ ofl, int64_t n,
                                                             int64_t m, unsigned long long *tcount) {
    const int64_t t = (int64_t)blockIdx.x * kLccBlock + threadIdx.x;
    const int64_t e0 = t * kLccEdgesPerThread;
    if (e0 >= m) return;
    const int64_t e1 = min(e0 + kLccEdgesPerThread, m);
    int64_t v = row_of_edge(orp, n, e0);
    for (int64_t e = e0; e < e1; e++) {
        while (orp[v + 1] <= e) v++;
        const int32_t u = oci[e];
        const unsigned cvu = __popc(ofl[e]);
        int64_t i = orp[v], ie = orp[v + 1];
        int64_t j = orp[u], je = orp[u + 1];
        unsigned long long tv = 0, tu = 0;
        while (i < ie && j < je) {
            const int32_t x = oci[i], y = oci[j];
            if (x < y) {
                i++;
            } else if (x > y) {
                j++;
            } else {
                // triangle {v, u, x}
                tv += __popc(ofl[j]);   // directions between u and x
                tu += __popc(ofl[i]);   // directions between v and x
                atomicAdd(&tcount[x], (unsigned long long)cvu);
                i++;
                j++;
            }
        }
        if (tv) atomicAdd(&tcount[v], tv);
        if (tu) atomicAdd(&tcount[u], tu);
    }
}

__global__ void k_lcc_final(const int64_t *__restrict__ srp, const unsigned long long *__restrict__ tc,
                            int64_t n, double *__restrict__ out) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = srp[v + 1] - srp[v];
        out[v] = k < 2 ? 0.0 : (double)tc[v] / ((double)k * (double)(k - 1));
    }
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_lcc(gx_graph *g, double *lcc) {
    if (!g || !lcc) return fail(GX_NULL_POINTER, "gx_lcc: null argument");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    if (n == 0) return GX_SUCCESS;
    GX_TRY(device_begin(ctx));
    GX_TRY(ensure_closure(g));
    const DevCSR &S = g->S;
    DBuf<int64_t> cnt, orp;
    GX_TRY(cnt.alloc(n + 1));
    GX_TRY(orp.alloc(n + 1));
    GX_HIP_TRY(hipMemsetAsync(cnt.p + n, 0, 8, s));
    const unsigned vgrid = grid_for(n, 256, 8192);
    hipLaunchKernelGGL(k_orient_count, dim3(vgrid), dim3(256), 0, s, S.rp.p, S.ci.p, n, cnt.p);
    GX_TRY(check_launch("k_orient_count"));
    size_t tmp_bytes = 0;
    GX_HIP_TRY(rocprim::exclusive_scan(nullptr, tmp_bytes, cnt.p, orp.p, (int64_t)0, (size_t)(n + 1),
                                       rocprim::plus<int64_t>(), s));
    DBuf<char> tmp;
    GX_TRY(tmp.alloc(tmp_bytes));
    GX_HIP_TRY(rocprim::exclusive_scan(tmp.p, tmp_bytes, cnt.p, orp.p, (int64_t)0, (size_t)(n + 1),
                                       rocprim::plus<int64_t>(), s));
    int64_t m = 0;
    GX_HIP_TRY(hipMemcpyAsync(&m, orp.p + n, 8, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    DBuf<int32_t> oci;
    DBuf<uint8_t> ofl;
    DBuf<unsigned long long> tc;
    DBuf<double> out;
    GX_TRY(oci.alloc(m));
    GX_TRY(ofl.alloc(m));
    GX_TRY(tc.alloc(n));
    GX_TRY(out.alloc(n));
    GX_HIP_TRY(hipMemsetAsync(tc.p, 0, n * 8, s));
    hipLaunchKernelGGL(k_orient_fill, dim3(vgrid), dim3(256), 0, s, S.rp.p, S.ci.p, S.flag.p, n, orp.p,
                       oci.p, ofl.p);
    GX_TRY(check_launch("k_orient_fill"));
    if (m) {
        KTimer kt(ctx, "lcc_triangles", s);
        hipLaunchKernelGGL(k_lcc_triangles,
                           dim3(grid_for((uint64_t)((m + kLccEdgesPerThread - 1) / kLccEdgesPerThread),
                                         kLccBlock, 1u << 30)),
                           dim3(kLccBlock), 0, s, orp.p, oci.p, ofl.p, n, m, tc.p);
    }
    GX_TRY(check_launch("k_lcc_triangles"));
    hipLaunchKernelGGL(k_lcc_final, dim3(vgrid), dim3(256), 0, s, S.rp.p, tc.p, n, out.p);
    GX_TRY(check_launch("k_lcc_final"));
    GX_TRY(device_end(ctx));
    GX_HIP_TRY(hipMemcpy(lcc, out.p, n * 8, hipMemcpyDeviceToHost));
    return GX_SUCCESS;
}
