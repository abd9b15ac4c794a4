// gx_ops.hip -- the op-level GraphBLAS C-ABI: gx_mxv, gx_vxm, gx_mxm_masked (include/gx.h).
//
// The algorithm-level entry points (gx_bfs, gx_pagerank, ...) run fused kernels; these expose the
// GraphBLAS operations the reference's LAGraph calls are built from, one call each, for unit
// parity against oracle/gx_oracle.c (orc_mxv, orc_mxm_masked):
//   PLUS_SECOND_FP64   GrB_mxv(t, .., LAGraph_plus_second_fp64, AT, w)   LAGr_PageRankGX, pr.cpp:61
//   MIN_SECOND_UINT64  GrB_mxm(S, .., GrB_MIN_SECOND_SEMIRING_UINT64, ..) LAGraph_cdlp.c:272-281,
//                      FastSV's mxv (LAGr_ConnectedComponents, wcc.cpp:61)
//   ANY_PAIR_BOOL      the BFS frontier vxm                             LAGr_BreadthFirstSearch, bfs.cpp:80
//   MIN_PLUS_FP64      the SSSP relaxation vxm                          LAGr_SingleSourceShortestPath, sssp.cpp:78
//   PLUS_PAIR_INT64    masked mxm C<A> = A A' (triangle counts)         LAGraph_lcc, lcc.cpp:68
//
// mxv with PLUS_SECOND_FP64 over A' (the PageRank product) runs the headline kernel itself:
// gx_pagerank's hub-first, column-sorted plan (k_pr_pull_units, gx_pr_sorted.hip) with damping
// 1 and no dangling mass, so its epilogue leaves r(v) = sum of the gathered u.  Every other
// product is a pull over the rows of M (A, or A' built on the device): a thread per row up to
// kShortDeg entries, longer rows cut into kSegNnz-entry segments, one wave each, combined by
// monoid atomics; then one pass applies the mask, the accumulator and presence.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "gx_pr.h"

namespace gx {
namespace {

constexpr int kShortDeg = 64;
constexpr int kSegNnz = 2048;

enum Sr { kPlusSecondF64 = 0, kMinSecondU64 = 1, kAnyPairBool = 2, kMinPlusF64 = 3, kPlusPairI64 = 4 };

template <int SR>
struct Monoid;
template <>
struct Monoid<kPlusSecondF64> {
    using T = double;
    __device__ static T id() { return 0.0; }
    __device__ static T op(T a, T b) { return a + b; }
    __device__ static void atomic(T *p, T v) { atomicAdd(p, v); }
};
template <>
struct Monoid<kMinSecondU64> {
    using T = unsigned long long;
    __device__ static T id() { return ~0ull; }
    __device__ static T op(T a, T b) { return a < b ? a : b; }
    __device__ static void atomic(T *p, T v) { atomicMin(p, v); }
};
template <>
struct Monoid<kAnyPairBool> {
    using T = unsigned long long;
    __device__ static T id() { return 0ull; }
    __device__ static T op(T a, T b) { return a | b; }
    __device__ static void atomic(T *p, T v) {
        if (v) atomicOr(p, v);
    }
};
template <>
struct Monoid<kMinPlusF64> {
    using T = double;
    __device__ static T id() { return INFINITY; }
    __device__ static T op(T a, T b) { return a < b ? a : b; }
    __device__ static void atomic(T *p, T v) {
        unsigned long long *q = reinterpret_cast<unsigned long long *>(p);
        unsigned long long old = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (v < __longlong_as_double((long long)old)) {
            if (__hip_atomic_compare_exchange_strong(q, &old, (unsigned long long)__double_as_longlong(v),
                                                     __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                break;
        }
    }
};
template <>
struct Monoid<kPlusPairI64> {
    using T = unsigned long long;   // int64 counts, two's complement
    __device__ static T id() { return 0ull; }
    __device__ static T op(T a, T b) { return a + b; }
    __device__ static void atomic(T *p, T v) { atomicAdd(p, v); }
};

// The multiplicative op on (matrix value a, vector value u(j)): mxv takes mult(a, u), vxm
// mult(u, a) (the matrix operand second); SECOND picks the second operand, PAIR is 1.
// fp64 -> uint64 the way GraphBLAS typecasts (GB_cast_to_uint64_t): NaN and values <= 0 give
// 0, values >= 2^64 give UINT64_MAX, the rest truncate.
__device__ __forceinline__ unsigned long long cast_u64(double x) {
    if (!(x > 0.0)) return 0ull;   // NaN too
    if (x >= 18446744073709551616.0) return ~0ull;
    return (unsigned long long)x;
}

template <int SR, bool VXM>
__device__ __forceinline__ typename Monoid<SR>::T term(double a, const void *u, int64_t j) {
    if constexpr (SR == kPlusSecondF64) return VXM ? a : static_cast<const double *>(u)[j];
    else if constexpr (SR == kMinSecondU64)
        return VXM ? cast_u64(a) : static_cast<const unsigned long long *>(u)[j];
    else if constexpr (SR == kMinPlusF64) {
        const double x = static_cast<const double *>(u)[j];
        return VXM ? x + a : a + x;
    } else return 1ull;
}

struct OpArgs {
    const int64_t *rp;
    const int32_t *ci;
    const double *w;          // matrix values (nullptr: an unweighted graph, every value 1)
    int64_t n;
    const void *u;
    const uint8_t *u_present;
    void *t;                  // n monoid values
    uint8_t *hit;             // n: some term exists
    int64_t *items;           // (row << 20 | segment) of the long rows
    unsigned long long *nitems;
};

template <int SR, bool VXM>
__global__ __launch_bounds__(256) void k_op_rows(OpArgs a) {
    using M = Monoid<SR>;
    using T = typename M::T;
    T *t = static_cast<T *>(a.t);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * 256) {
        const int64_t b = a.rp[i], e = a.rp[i + 1];
        if (e - b > kShortDeg) {   // segments for k_op_long; the row starts at the identity
            t[i] = M::id();
            a.hit[i] = 0;
            const int64_t nseg = (e - b + kSegNnz - 1) / kSegNnz;
            const unsigned long long at = atomicAdd(a.nitems, (unsigned long long)nseg);
            for (int64_t s = 0; s < nseg; s++) a.items[at + s] = (i << 20) | s;
            continue;
        }
        T acc = M::id();
        bool h = false;
        for (int64_t k = b; k < e; k++) {
            const int64_t j = a.ci[k];
            if (a.u_present && !a.u_present[j]) continue;
            acc = M::op(acc, term<SR, VXM>(a.w ? a.w[k] : 1.0, a.u, j));
            h = true;
        }
        t[i] = acc;
        a.hit[i] = h;
    }
}

template <int SR, bool VXM>
__global__ __launch_bounds__(256) void k_op_long(OpArgs a) {
    using M = Monoid<SR>;
    using T = typename M::T;
    T *t = static_cast<T *>(a.t);
    const int lane = threadIdx.x & (kWave - 1);
    const unsigned long long m = *a.nitems;
    for (unsigned long long it = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / kWave; it < m;
         it += (uint64_t)gridDim.x * 256 / kWave) {
        const int64_t item = a.items[it];
        const int64_t i = item >> 20, s = item & ((1 << 20) - 1);
        const int64_t b = a.rp[i] + s * kSegNnz, e = min(b + kSegNnz, a.rp[i + 1]);
        T acc = M::id();
        bool h = false;
        for (int64_t k = b + lane; k < e; k += kWave) {
            const int64_t j = a.ci[k];
            if (a.u_present && !a.u_present[j]) continue;
            acc = M::op(acc, term<SR, VXM>(a.w ? a.w[k] : 1.0, a.u, j));
            h = true;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc = M::op(acc, __shfl_xor(acc, off, kWave));
        const bool any = __ballot(h) != 0;
        if (lane == 0 && any) {
            M::atomic(&t[i], acc);
            a.hit[i] = 1;
        }
    }
}

// out<mask> (+)= t with presence (GraphBLAS C API: mask structural, optionally complemented;
// REPLACE clears the masked-out entries; ACCUM combines with the present old entries).
template <int SR, typename OutT>
__global__ __launch_bounds__(256) void k_op_finish(const void *tv, const uint8_t *hit, int64_t n, const uint8_t *mask,
                                                   int desc, OutT *out, uint8_t *out_present) {
    using M = Monoid<SR>;
    using T = typename M::T;
    const T *t = static_cast<const T *>(tv);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const bool allowed = !mask || ((mask[i] != 0) != ((desc & GX_DESC_MASK_COMP) != 0));
        const bool old = out_present ? out_present[i] != 0 : true;
        bool present = hit[i] != 0;
        T v = t[i];
        if (!allowed) {
            if (!(desc & GX_DESC_REPLACE)) continue;
            present = false;
        } else if ((desc & GX_DESC_ACCUM) && old) {
            if (!present) {
                if (out_present) out_present[i] = 1;
                continue;   // w(i) kept
            }
            T o;
            if constexpr (SR == kPlusSecondF64 || SR == kMinPlusF64) o = (T)out[i];
            else o = (T)(unsigned long long)out[i];
            v = M::op(o, v);
        }
        if (out_present) out_present[i] = present;
        if (!present) v = M::id();
        if constexpr (SR == kAnyPairBool) out[i] = (OutT)(v ? 1 : 0);
        else out[i] = (OutT)v;
    }
}

// c[perm[e]] = |row(i) ∩ row(j)| for the sorted entry e = (i, j) of the sorted copy (rp, ci):
// the shorter list's columns binary-searched in the longer one.
__global__ __launch_bounds__(256) void k_op_mxm_pair(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                     const uint64_t *__restrict__ keys, const uint32_t *__restrict__ perm,
                                                     int64_t nnz, int64_t *__restrict__ c) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * 256) {
        const int64_t i = (int64_t)(keys[e] >> 32), j = (int64_t)(uint32_t)keys[e];
        int64_t sb = rp[i], se = rp[i + 1], lb = rp[j], le = rp[j + 1];
        if (se - sb > le - lb) {
            int64_t x = sb, y = se;
            sb = lb; se = le; lb = x; le = y;
        }
        int64_t cnt = 0;
        for (int64_t k = sb; k < se; k++) {
            const int32_t v = ci[k];
            int64_t lo = lb, hi = le;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (ci[mid] < v) lo = mid + 1;
                else hi = mid;
            }
            cnt += lo < le && ci[lo] == v;
        }
        c[perm[e]] = cnt;
    }
}

__global__ void k_op_sorted_cols(const uint64_t *__restrict__ keys, int64_t nnz, int32_t *__restrict__ ci) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * blockDim.x)
        ci[e] = (int32_t)(uint32_t)keys[e];
}

__global__ void k_op_mxm_keys(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, int64_t n,
                              uint64_t *__restrict__ keys, uint32_t *__restrict__ idx) {
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; i < n;
         i += (int64_t)gridDim.x * blockDim.x / kWave)
        for (int64_t k = rp[i] + lane; k < rp[i + 1]; k += kWave) {
            keys[k] = ((uint64_t)i << 32) | (uint32_t)ci[k];
            idx[k] = (uint32_t)k;
        }
}

// x for the PageRank kernel: the hub-first chunk holds u (absent entries 0, PLUS's identity)
// and a zero dangling slot; out = r of the hub-first row order[v]... gathered back by perm.
__global__ void k_op_pr_in(const double *__restrict__ u, const uint8_t *__restrict__ up, const int32_t *__restrict__ perm,
                           int64_t n, double *__restrict__ x, int64_t slot) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        x[perm[v]] = (!up || up[v]) ? u[v] : 0.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) x[slot] = 0.0;
}

__global__ void k_op_pr_out(const double *__restrict__ r, const int32_t *__restrict__ perm, int64_t n,
                            double *__restrict__ t) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        t[v] = r[perm[v]];
}

size_t elem_size(int sr) { return sr == kAnyPairBool ? 1 : 8; }

// Upload n elements (host -> device) if p is set.
template <typename T>
int up(DBuf<T> &d, const void *p, size_t bytes, hipStream_t s) {
    if (!p) return GX_SUCCESS;
    GX_TRY(d.alloc(std::max<size_t>(bytes / sizeof(T), 1)));
    GX_HIP_TRY(hipMemcpyAsync(d.p, p, bytes, hipMemcpyHostToDevice, s));
    return GX_SUCCESS;
}

template <int SR, bool VXM>
void launch_rows(const OpArgs &a, hipStream_t s) {
    hipLaunchKernelGGL((k_op_rows<SR, VXM>), dim3(grid_for(a.n, 256, 8192)), dim3(256), 0, s, a);
    hipLaunchKernelGGL((k_op_long<SR, VXM>), dim3(1024), dim3(256), 0, s, a);
}

template <int SR>
void launch_finish(const void *t, const uint8_t *hit, int64_t n, const uint8_t *mask, int desc, void *out,
                   uint8_t *out_present, hipStream_t s) {
    const unsigned g = grid_for(n, 256, 8192);
    if constexpr (SR == kAnyPairBool)
        hipLaunchKernelGGL((k_op_finish<SR, uint8_t>), dim3(g), dim3(256), 0, s, t, hit, n, mask, desc,
                           static_cast<uint8_t *>(out), out_present);
    else if constexpr (SR == kPlusSecondF64 || SR == kMinPlusF64)
        hipLaunchKernelGGL((k_op_finish<SR, double>), dim3(g), dim3(256), 0, s, t, hit, n, mask, desc,
                           static_cast<double *>(out), out_present);
    else
        hipLaunchKernelGGL((k_op_finish<SR, unsigned long long>), dim3(g), dim3(256), 0, s, t, hit, n, mask, desc,
                           static_cast<unsigned long long *>(out), out_present);
}

int op_vector(gx_graph *g, int sr, int vxm, int desc, const uint8_t *mask, const void *u, const uint8_t *u_present,
              void *out, uint8_t *out_present) {
    if (!g || !out) return fail(GX_NULL_POINTER, "gx_mxv/gx_vxm: null argument");
    if (sr < 0 || sr > 4) return fail(GX_INVALID_VALUE, "gx_mxv/gx_vxm: unknown semiring");
    const bool needs_u = sr == kPlusSecondF64 ? !vxm : sr == kMinSecondU64 ? !vxm : sr == kMinPlusF64;
    if (needs_u && !u) return fail(GX_NULL_POINTER, "gx_mxv/gx_vxm: this semiring reads u");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    if (n == 0) return GX_SUCCESS;
    GX_TRY(device_begin(ctx));
    // M = A, or A' (vxm pulls over A' unless T0 asks for A itself); an undirected graph is
    // symmetric, so A' = A
    const bool use_t = (vxm != 0) != ((desc & GX_DESC_T0) != 0);
    if (use_t && g->directed) GX_TRY(ensure_transpose(g));
    const DevCSR &M = use_t && g->directed ? g->AT : g->A;
    const size_t es = elem_size(sr);
    DBuf<char> du, dout;
    DBuf<uint8_t> dup, dmask, dop, hit;
    DBuf<unsigned long long> t;
    GX_TRY(up(du, needs_u ? u : nullptr, (size_t)n * 8, s));
    GX_TRY(up(dup, u_present, (size_t)n, s));
    GX_TRY(up(dmask, mask, (size_t)n, s));
    GX_TRY(dout.alloc((size_t)n * es));
    // the old w is read where the mask keeps it or ACCUM combines with it
    GX_HIP_TRY(hipMemcpyAsync(dout.p, out, (size_t)n * es, hipMemcpyHostToDevice, s));
    GX_TRY(up(dop, out_present, (size_t)n, s));
    GX_TRY(t.alloc((size_t)n));
    GX_TRY(hit.alloc((size_t)n));
    const bool pr_path = sr == kPlusSecondF64 && !vxm && use_t;   // t = A' u: the PageRank product
    if (pr_path) {
        if (!g->pr) GX_TRY(pr_single_plan(g, &g->pr));
        PrPart *p = g->pr;
        const double damping = p->damping;
        p->damping = 1.0;   // teleport (1-d)/n = 0, no dangling mass: r = the gathered sum
        const unsigned gr = grid_for(n, 256, 8192);
        hipLaunchKernelGGL(k_op_pr_in, dim3(gr), dim3(256), 0, s, reinterpret_cast<const double *>(du.p), dup.p,
                           p->perm.p, n, p->xa.p, (int64_t)p->chunk - 1);
        int rc = check_launch("k_op_pr_in");
        if (rc == GX_SUCCESS) rc = pr_step(p, p->xa.p, p->xb.p, p->rank_out.p, s);
        p->damping = damping;
        GX_TRY(rc);
        hipLaunchKernelGGL(k_op_pr_out, dim3(gr), dim3(256), 0, s, p->rank_out.p, p->perm.p, n,
                           reinterpret_cast<double *>(t.p));
        GX_TRY(check_launch("k_op_pr_out"));
    }
    // presence of every t(i) (and, off the PageRank path, the values): the row pull
    DBuf<int64_t> items;
    DBuf<unsigned long long> nitems;
    GX_TRY(items.alloc((size_t)(M.nnz / kSegNnz + M.nnz / kShortDeg + 2)));   // rows past kShortDeg: < nnz / kShortDeg
    GX_TRY(nitems.alloc(1));
    GX_HIP_TRY(hipMemsetAsync(nitems.p, 0, 8, s));
    DBuf<unsigned long long> tscratch;
    OpArgs a{M.rp.p, M.ci.p, M.w.p, n, du.p, dup.p, t.p, hit.p, items.p, nitems.p};
    if (pr_path) {   // the pull below only marks presence (ANY_PAIR into a scratch)
        GX_TRY(tscratch.alloc((size_t)n));
        a.t = tscratch.p;
        launch_rows<kAnyPairBool, false>(a, s);
    } else {
        switch (sr * 2 + (vxm ? 1 : 0)) {
            case 0: launch_rows<kPlusSecondF64, false>(a, s); break;
            case 1: launch_rows<kPlusSecondF64, true>(a, s); break;
            case 2: launch_rows<kMinSecondU64, false>(a, s); break;
            case 3: launch_rows<kMinSecondU64, true>(a, s); break;
            case 4: case 5: launch_rows<kAnyPairBool, false>(a, s); break;
            case 6: launch_rows<kMinPlusF64, false>(a, s); break;
            case 7: launch_rows<kMinPlusF64, true>(a, s); break;
            default: launch_rows<kPlusPairI64, false>(a, s); break;
        }
    }
    GX_TRY(check_launch("k_op_rows"));
    switch (sr) {
        case kPlusSecondF64: launch_finish<kPlusSecondF64>(t.p, hit.p, n, dmask.p, desc, dout.p, dop.p, s); break;
        case kMinSecondU64: launch_finish<kMinSecondU64>(t.p, hit.p, n, dmask.p, desc, dout.p, dop.p, s); break;
        case kAnyPairBool: launch_finish<kAnyPairBool>(t.p, hit.p, n, dmask.p, desc, dout.p, dop.p, s); break;
        case kMinPlusF64: launch_finish<kMinPlusF64>(t.p, hit.p, n, dmask.p, desc, dout.p, dop.p, s); break;
        default: launch_finish<kPlusPairI64>(t.p, hit.p, n, dmask.p, desc, dout.p, dop.p, s); break;
    }
    GX_TRY(check_launch("k_op_finish"));
    GX_TRY(device_end(ctx));
    GX_HIP_TRY(hipMemcpyAsync(out, dout.p, (size_t)n * es, hipMemcpyDeviceToHost, s));
    if (out_present) GX_HIP_TRY(hipMemcpyAsync(out_present, dop.p, (size_t)n, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    return GX_SUCCESS;
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_mxv(gx_graph *g, int semiring, int desc, const uint8_t *mask, const void *u,
                      const uint8_t *u_present, void *w, uint8_t *w_present) {
    return op_vector(g, semiring, 0, desc, mask, u, u_present, w, w_present);
}

extern "C" int gx_vxm(gx_graph *g, int semiring, int desc, const uint8_t *mask, const void *u,
                      const uint8_t *u_present, void *w, uint8_t *w_present) {
    return op_vector(g, semiring, 1, desc, mask, u, u_present, w, w_present);
}

extern "C" int gx_mxm_masked(gx_graph *g, int semiring, int desc, int64_t *c) {
    if (!g || (!c && g->nnz)) return fail(GX_NULL_POINTER, "gx_mxm_masked: null argument");
    if (semiring != kPlusPairI64 || desc != 0)
        return fail(GX_NOT_IMPLEMENTED, "gx_mxm_masked: only C<A> = A*A' with GX_PLUS_PAIR_INT64");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n, nnz = (int64_t)g->nnz;
    if (nnz == 0) return GX_SUCCESS;
    if (nnz >= (1ll << 32)) return fail(GX_NOT_IMPLEMENTED, "gx_mxm_masked: 2^32 entries or more");
    GX_TRY(device_begin(ctx));
    // a row-sorted copy of A (rows may come unsorted), with every entry's original position
    DBuf<uint64_t> k0, k1;
    DBuf<uint32_t> i0, i1;
    DBuf<int64_t> rp;
    DBuf<int32_t> ci;
    DBuf<int64_t> dc;
    GX_TRY(k0.alloc(nnz));
    GX_TRY(k1.alloc(nnz));
    GX_TRY(i0.alloc(nnz));
    GX_TRY(i1.alloc(nnz));
    GX_TRY(ci.alloc(nnz, 16));
    GX_TRY(dc.alloc(nnz));
    hipLaunchKernelGGL(k_op_mxm_keys, dim3(grid_for(n * kWave, 256, 8192)), dim3(256), 0, s, g->A.rp.p, g->A.ci.p, n,
                       k0.p, i0.p);
    GX_TRY(check_launch("k_op_mxm_keys"));
    int bits = 1;
    while ((1ull << bits) < (uint64_t)n) bits++;
    GX_TRY(sort_pairs_u64_u32(k0.p, k1.p, i0.p, i1.p, (size_t)nnz, 32 + bits, s));
    // the sorted copy keeps A's row pointers (same rows, same lengths)
    hipLaunchKernelGGL(k_op_sorted_cols, dim3(grid_for(nnz, 256, 8192)), dim3(256), 0, s, k1.p, nnz, ci.p);
    GX_TRY(check_launch("k_op_sorted_cols"));
    hipLaunchKernelGGL(k_op_mxm_pair, dim3(grid_for(nnz, 256, 8192)), dim3(256), 0, s, g->A.rp.p, ci.p, k1.p, i1.p,
                       nnz, dc.p);
    GX_TRY(check_launch("k_op_mxm_pair"));
    GX_TRY(device_end(ctx));
    GX_HIP_TRY(hipMemcpyAsync(c, dc.p, (size_t)nnz * 8, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    return GX_SUCCESS;
}

GX_MODULE_WARMER(ops)
