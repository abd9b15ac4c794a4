// gx_sssp_split.hip -- SSSP on a 1-D split of the vertices (config 4: datagen-8_5-fb,
// 8 GPUs, 1-D partition + RCCL all-gather).  Replaces LA_SSSP's delta-stepping
// (sssp.cpp:53-81) for a rank that owns the targets [v0, v1).
//
// Layout per rank: the edges u -> v of the whole graph whose target v is owned, by source
// (CSR over all n sources), light edges (w < delta) first.  The distance vector is replicated:
// every rank holds dist[n] and applies every improvement, so every rank takes the same
// scheduling decisions from the same counts.
//
// Round (bulk synchronous, delta-stepping after Meyer & Sanders):
//   plan   one thread: LIGHT (relax the frontier queued last round), HEAVY (relax the heavy
//          edges of the vertices settled in the current bucket since the last HEAVY), ADVANCE
//          (open the smallest pending bucket: minb + take move its vertices to the frontier),
//          or done -- decided from the replicated vertex counts only;
//   relax  one wave per (vertex, 256-edge chunk) item of this rank's slice; a target whose
//          distance drops is claimed once per round onto the improved list;
//   pairs  (vertex, distance bits) of the improved owned vertices + {count, done};
//   -- the caller all-gathers the pairs of every rank (gx_sssp_split_run: one rank, none) --
//   apply  every rank's pairs: dist = min, then the vertex goes to the next frontier when its
//          bucket is <= cur (and to the current bucket's settled set), else to the pending set.
// Distances are the relaxation fixed point, bitwise the oracle's and gx_sssp's whatever the
// split or delta (gx_sssp.hip header).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include <rocprim/rocprim.hpp>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kSB = 256;        // threads per block
constexpr int kSChunk = 256;    // edges per relax item
constexpr unsigned long long kInf = 0x7FF0000000000000ull;   // +inf bits

enum : int32_t { kNone = 0, kLight = 1, kHeavy = 2, kAdvance = 3 };

// Replicated decision state (identical on every rank after every apply) + this rank's item
// counters (which differ by rank and never enter a decision).
struct SplitState {
    int64_t cur;                  // bucket being settled
    unsigned long long pminb;     // ADVANCE: smallest bucket on the pending list
    int32_t mode, round, epoch, done;
    int32_t fc;                   // frontier list relaxed this round (LIGHT / ADVANCE)
    int32_t pin;                  // pending list appended to
    uint32_t fv[2], fi[2];        // frontier vertices (replicated) / items (rank-local)
    uint32_t sv, sv_done;         // settled vertices of this epoch / heavy-relaxed so far
    uint32_t si, si_done;         // their heavy items (rank-local) / relaxed so far
    uint32_t hs0, hs1;            // HEAVY: items [hs0, hs1) of the settled list
    uint32_t pcnt[2];             // pending vertices
    uint32_t nimp;                // improved owned vertices this round (rank-local)
};

struct SplitBufs {
    const int64_t *srp;           // slice rows: [srp[u], slend[u]) light, [slend[u], srp[u+1]) heavy
    const int64_t *slend;
    const int32_t *sci;           // owned target - v0
    const double *sw;
    unsigned long long *dist;     // replicated distances (fp64 bits)
    unsigned long long *lrel;     // distance u's light edges were queued for relaxing with
    int32_t *sstamp, *pstamp, *istamp;   // settled epoch / pending flag / improved round
    uint64_t *fitems[2];          // (u << 32 | chunk)
    uint64_t *sitems;             // heavy items of the settled vertices
    int32_t *plist[2];
    int32_t *imp;                 // improved owned vertices (global ids)
    int64_t n, v0, v1;
    double inv_delta;
    SplitState *st;
};

__device__ __forceinline__ int64_t sbucket(unsigned long long bits, double inv_delta) {
    const double q = __longlong_as_double((long long)bits) * inv_delta;
    return q < 4.0e18 ? (int64_t)q : (int64_t)4000000000000000000ll;
}

// Wave-aggregated reservation: lane with c items gets its first slot; one atomic per wave.
// Every lane of the wave must call it.
__device__ __forceinline__ uint32_t wave_reserve(uint32_t *counter, uint32_t c) {
    const int lane = threadIdx.x & (kWave - 1);
    uint32_t x = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, kWave);
        if (lane >= off) x += y;
    }
    const uint32_t tot = __shfl(x, kWave - 1, kWave);
    uint32_t base = 0;
    if (lane == kWave - 1 && tot) base = atomicAdd(counter, tot);
    base = __shfl(base, kWave - 1, kWave);
    return base + x - c;
}

__device__ __forceinline__ uint32_t nchunks(int64_t len) { return (uint32_t)max<int64_t>(1, (len + kSChunk - 1) / kSChunk); }

// Queue v (distance d) for the next light relaxation of `list` and into the epoch's settled
// set; `take` lanes only (every lane calls).
__device__ __forceinline__ void queue_frontier(const SplitBufs &B, bool take, int64_t v, unsigned long long d, int list,
                                               int32_t epoch) {
    SplitState *st = B.st;
    uint32_t nl = 0, nh = 0, isv = 0;
    if (take) {
        B.lrel[v] = d;
        nl = nchunks(B.slend[v] - B.srp[v]);
        if (B.sstamp[v] != epoch) {
            B.sstamp[v] = epoch;   // the vertex is claimed by this lane alone (unique per round)
            isv = 1;
            nh = nchunks(B.srp[v + 1] - B.slend[v]);
        }
    }
    const uint32_t fvb = wave_reserve(&st->fv[list], take ? 1u : 0u);
    (void)fvb;
    const uint32_t fib = wave_reserve(&st->fi[list], nl);
    wave_reserve(&st->sv, isv);
    const uint32_t sib = wave_reserve(&st->si, nh);
    for (uint32_t j = 0; j < nl; j++) B.fitems[list][fib + j] = ((uint64_t)(uint32_t)v << 32) | j;
    for (uint32_t j = 0; j < nh; j++) B.sitems[sib + j] = ((uint64_t)(uint32_t)v << 32) | j;
}

__global__ void k_split_start(SplitBufs B, int64_t src) {
    const int64_t i = (int64_t)blockIdx.x * kSB + threadIdx.x;
    for (int64_t v = i; v < B.n; v += (int64_t)gridDim.x * kSB) {
        B.dist[v] = v == src ? 0ull : kInf;
        B.lrel[v] = kInf;
        B.sstamp[v] = 0;
        B.pstamp[v] = 0;
    }
    for (int64_t v = i; v < B.v1 - B.v0; v += (int64_t)gridDim.x * kSB) B.istamp[v] = 0;
}

__global__ void k_split_seed(SplitBufs B, int64_t src) {
    SplitState *st = B.st;
    if (threadIdx.x == 0) {
        memset(st, 0, sizeof(SplitState));
        st->epoch = 1;
        st->fc = 0;
    }
    __syncthreads();
    // first wave queues the source into list 1 (the next frontier)
    if (threadIdx.x < kWave) queue_frontier(B, threadIdx.x == 0, src, 0ull, 1, 1);
}

__global__ void k_split_plan(SplitState *st) {
    st->nimp = 0;
    if (st->done) {
        st->mode = kNone;
        return;
    }
    st->round++;
    const int nx = st->fc ^ 1;
    if (st->fv[nx] > 0) {
        st->mode = kLight;
        st->fc = nx;
        st->fv[nx ^ 1] = 0;
        st->fi[nx ^ 1] = 0;
        return;
    }
    if (st->sv > st->sv_done) {
        st->mode = kHeavy;
        st->hs0 = st->si_done;
        st->hs1 = st->si;
        st->si_done = st->si;
        st->sv_done = st->sv;
        return;
    }
    if (st->pcnt[st->pin] > 0) {
        st->mode = kAdvance;
        st->epoch++;
        st->sv = st->sv_done = st->si = st->si_done = 0;
        st->pin ^= 1;
        st->pcnt[st->pin] = 0;
        st->pminb = ~0ull;
        st->fc ^= 1;   // take fills list fc, apply the other
        st->fv[0] = st->fv[1] = st->fi[0] = st->fi[1] = 0;
        return;
    }
    st->done = 1;
    st->mode = kNone;
}

// ADVANCE: the smallest bucket among the still pending vertices of the old pending list.
__global__ __launch_bounds__(kSB) void k_split_minb(SplitBufs B) {
    SplitState *st = B.st;
    if (st->mode != kAdvance) return;
    const int32_t *pl = B.plist[st->pin ^ 1];
    const uint32_t cnt = st->pcnt[st->pin ^ 1];
    unsigned long long m = ~0ull;
    for (uint32_t i = blockIdx.x * kSB + threadIdx.x; i < cnt; i += gridDim.x * kSB) {
        const int32_t v = pl[i];
        const unsigned long long d = B.dist[v];
        if (d < B.lrel[v]) m = min(m, (unsigned long long)sbucket(d, B.inv_delta));
    }
    for (int off = 32; off > 0; off >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, off, kWave));
    if ((threadIdx.x & (kWave - 1)) == 0 && m != ~0ull) atomicMin(&st->pminb, m);
}

// ADVANCE: the pending vertices of bucket <= pminb go to the frontier relaxed this round,
// the other still pending ones to the new pending list; relaxed ones are dropped.
__global__ __launch_bounds__(kSB) void k_split_take(SplitBufs B) {
    SplitState *st = B.st;
    if (st->mode != kAdvance) return;
    const int32_t *pl = B.plist[st->pin ^ 1];
    const uint32_t cnt = st->pcnt[st->pin ^ 1];
    const unsigned long long cb = st->pminb;
    const int32_t epoch = st->epoch, fc = st->fc, pin = st->pin;
    const uint32_t span = (cnt + kSB - 1) / kSB * kSB;   // whole waves iterate together
    for (uint32_t i = blockIdx.x * kSB + threadIdx.x; i < span; i += gridDim.x * kSB) {
        const bool valid = i < cnt;
        const int32_t v = valid ? pl[i] : 0;
        const unsigned long long d = valid ? B.dist[v] : kInf;
        const bool pend = valid && d < B.lrel[v];
        const bool now = pend && (unsigned long long)sbucket(d, B.inv_delta) <= cb;
        const bool keep = pend && !now;
        if (valid && !keep) B.pstamp[v] = 0;
        const uint32_t at = wave_reserve(&st->pcnt[pin], keep ? 1u : 0u);
        if (keep) B.plist[pin][at] = v;
        queue_frontier(B, now, v, d, fc, epoch);
    }
}

// One wave per item of the list this round relaxes.
__global__ __launch_bounds__(kSB) void k_split_relax(SplitBufs B) {
    SplitState *st = B.st;
    const int32_t mode = st->mode;
    if (mode == kNone) return;
    if (mode == kAdvance && blockIdx.x == 0 && threadIdx.x == 0) st->cur = (int64_t)min(st->pminb, 4000000000000000000ull);
    const bool heavy = mode == kHeavy;
    const uint64_t *items = heavy ? B.sitems : B.fitems[st->fc];
    const uint32_t i0 = heavy ? st->hs0 : 0u, i1 = heavy ? st->hs1 : st->fi[st->fc];
    const int32_t round = st->round;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = (blockIdx.x * kSB + threadIdx.x) / kWave, nw = gridDim.x * (kSB / kWave);
    for (uint32_t it = i0 + wid; it < i1; it += nw) {
        const uint64_t x = items[it];
        const int64_t u = (int64_t)(x >> 32);
        const int64_t j = (int64_t)(x & 0xffffffffu);
        const int64_t a = heavy ? B.slend[u] : B.srp[u], b = heavy ? B.srp[u + 1] : B.slend[u];
        const int64_t e0 = a + j * kSChunk, e1 = min(b, e0 + kSChunk);
        const double du = __longlong_as_double((long long)B.dist[u]);
        for (int64_t eb = e0; eb < e1; eb += kWave) {
            const int64_t e = eb + lane;
            bool won = false;
            int32_t t = 0;
            if (e < e1) {
                t = B.sci[e];
                const unsigned long long nd = (unsigned long long)__double_as_longlong(du + B.sw[e]);
                unsigned long long *dv = &B.dist[B.v0 + t];
                if (nd < __hip_atomic_load(dv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    const unsigned long long old =
                        __hip_atomic_fetch_min(dv, nd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    won = nd < old && B.istamp[t] != round && atomicExch(&B.istamp[t], round) != round;
                }
            }
            const uint32_t at = wave_reserve(&st->nimp, won ? 1u : 0u);
            if (won) B.imp[at] = (int32_t)(B.v0 + t);
        }
    }
}

// (vertex, distance bits) of the improved owned vertices, then {count, done}.
__global__ __launch_bounds__(kSB) void k_split_pairs(SplitBufs B, uint64_t *pairs, uint64_t *count) {
    const SplitState *st = B.st;
    const uint32_t k = st->nimp;
    for (uint32_t i = blockIdx.x * kSB + threadIdx.x; i < k; i += gridDim.x * kSB) {
        const int32_t v = B.imp[i];
        pairs[2 * (uint64_t)i] = (uint64_t)v;
        pairs[2 * (uint64_t)i + 1] = B.dist[v];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        count[0] = k;
        count[1] = (uint64_t)st->done;
    }
}

// Every rank's pairs (rank r's at pairs + 2 r stride, their number at counts[2 r]).
__global__ __launch_bounds__(kSB) void k_split_apply(SplitBufs B, const uint64_t *pairs, const uint64_t *counts,
                                                     int nranks, uint64_t stride) {
    SplitState *st = B.st;
    if (st->mode == kNone) return;
    const int64_t cur = st->cur;
    const int32_t epoch = st->epoch, nx = st->fc ^ 1, pin = st->pin;
    for (int r = 0; r < nranks; r++) {
        const uint64_t cnt = counts[2 * r];
        const uint64_t *pr = pairs + 2 * (uint64_t)r * stride;
        const uint64_t span = (cnt + kSB - 1) / kSB * kSB;
        for (uint64_t i = (uint64_t)blockIdx.x * kSB + threadIdx.x; i < span; i += (uint64_t)gridDim.x * kSB) {
            const bool valid = i < cnt;
            const int64_t v = valid ? (int64_t)pr[2 * i] : 0;
            const unsigned long long d = valid ? pr[2 * i + 1] : kInf;
            if (valid && d < B.dist[v]) B.dist[v] = d;   // one pair per vertex and round
            const bool near = valid && sbucket(d, B.inv_delta) <= cur;
            const bool far = valid && !near && B.pstamp[v] == 0;
            if (far) B.pstamp[v] = 1;
            const uint32_t at = wave_reserve(&st->pcnt[pin], far ? 1u : 0u);
            if (far) B.plist[pin][at] = (int32_t)v;
            queue_frontier(B, near, v, d, nx, epoch);
        }
    }
}

// ---- slice layout: the entries of A whose target is owned, light first ----
__global__ __launch_bounds__(kSB) void k_slice_count(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                     const double *__restrict__ w, int64_t n, int64_t v0, int64_t v1,
                                                     double delta, int64_t *lc, int64_t *tc) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (kSB / kWave);
    for (int64_t u = ((int64_t)blockIdx.x * kSB + threadIdx.x) / kWave; u < n; u += nw) {
        uint32_t l = 0, t = 0;
        for (int64_t e = rp[u] + lane; e < rp[u + 1]; e += kWave) {
            const int32_t v = ci[e];
            if (v >= v0 && v < v1) {
                t++;
                l += w[e] < delta;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            l += __shfl_xor(l, off, kWave);
            t += __shfl_xor(t, off, kWave);
        }
        if (lane == 0) {
            lc[u] = l;
            tc[u] = t;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) tc[n] = 0;
}

__global__ __launch_bounds__(kSB) void k_slice_scatter(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                       const double *__restrict__ w, int64_t n, int64_t v0, int64_t v1,
                                                       double delta, const int64_t *__restrict__ srp,
                                                       const int64_t *__restrict__ lc, int64_t *slend, int32_t *sci,
                                                       double *sw) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (kSB / kWave);
    const uint64_t below = (1ull << lane) - 1ull;
    for (int64_t u = ((int64_t)blockIdx.x * kSB + threadIdx.x) / kWave; u < n; u += nw) {
        int64_t pl = srp[u], ph = srp[u] + lc[u];
        if (lane == 0) slend[u] = ph;
        for (int64_t eb = rp[u]; eb < rp[u + 1]; eb += kWave) {
            const int64_t e = eb + lane;
            const bool valid = e < rp[u + 1];
            const int32_t v = valid ? ci[e] : -1;
            const double x = valid ? w[e] : 0.0;
            const bool own = valid && v >= v0 && v < v1;
            const bool light = own && x < delta, heavy = own && !(x < delta);
            const uint64_t ml = __ballot(light), mh = __ballot(heavy);
            if (light) {
                const int64_t p = pl + __popcll(ml & below);
                sci[p] = (int32_t)(v - v0);
                sw[p] = x;
            }
            if (heavy) {
                const int64_t p = ph + __popcll(mh & below);
                sci[p] = (int32_t)(v - v0);
                sw[p] = x;
            }
            pl += __popcll(ml);
            ph += __popcll(mh);
        }
    }
}

__global__ __launch_bounds__(256) void k_split_sum_w(const double *__restrict__ w, int64_t m, double *sum) {
    double acc = 0.0;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < m; k += (int64_t)gridDim.x * 256) acc += w[k];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) atomicAdd(sum, acc);
}

}  // namespace
}  // namespace gx

using namespace gx;

struct gx_sssp_split {
    gx_graph *g = nullptr;
    int64_t n = 0, v0 = 0, v1 = 0, snnz = 0;
    double delta = 1.0;
    DBuf<int64_t> srp, slend;
    DBuf<int32_t> sci;
    DBuf<double> sw;
    DBuf<unsigned long long> dist, lrel;
    DBuf<int32_t> sstamp, pstamp, istamp, plist0, plist1, imp;
    DBuf<uint64_t> fitems0, fitems1, sitems, own_pairs, own_count;
    DBuf<SplitState> st;
    int32_t *h_done = nullptr;
    unsigned grid = 0;
    ~gx_sssp_split() {
        if (h_done) (void)hipHostFree(h_done);
    }
    SplitBufs bufs() {
        SplitBufs B;
        B.srp = srp.p;
        B.slend = slend.p;
        B.sci = sci.p;
        B.sw = sw.p;
        B.dist = dist.p;
        B.lrel = lrel.p;
        B.sstamp = sstamp.p;
        B.pstamp = pstamp.p;
        B.istamp = istamp.p;
        B.fitems[0] = fitems0.p;
        B.fitems[1] = fitems1.p;
        B.sitems = sitems.p;
        B.plist[0] = plist0.p;
        B.plist[1] = plist1.p;
        B.imp = imp.p;
        B.n = n;
        B.v0 = v0;
        B.v1 = v1;
        B.inv_delta = 1.0 / delta;
        B.st = st.p;
        return B;
    }
};

// as the other *_part_* steps (gx.h): NULL is the null (default) stream -- torch's -- so the
// steps order with the tensors and collectives issued there
static hipStream_t split_stream(gx_sssp_split *, void *stream) { return (hipStream_t)stream; }

// plan -> minb -> take -> relax -> pairs (this rank's improved owned vertices)
static int split_relax(gx_sssp_split *p, uint64_t *pairs, uint64_t *count, hipStream_t s) {
    const SplitBufs B = p->bufs();
    hipLaunchKernelGGL(k_split_plan, dim3(1), dim3(1), 0, s, B.st);
    hipLaunchKernelGGL(k_split_minb, dim3(p->grid), dim3(kSB), 0, s, B);
    hipLaunchKernelGGL(k_split_take, dim3(p->grid), dim3(kSB), 0, s, B);
    hipLaunchKernelGGL(k_split_relax, dim3(p->grid), dim3(kSB), 0, s, B);
    hipLaunchKernelGGL(k_split_pairs, dim3(p->grid), dim3(kSB), 0, s, B, pairs, count);
    return check_launch("k_split_relax");
}

static int split_apply(gx_sssp_split *p, const uint64_t *pairs, const uint64_t *counts, int nranks, uint64_t stride,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_split_apply, dim3(p->grid), dim3(kSB), 0, s, p->bufs(), pairs, counts, nranks, stride);
    return check_launch("k_split_apply");
}

extern "C" int gx_sssp_split_create(gx_graph *g, uint64_t v0, uint64_t v1, gx_sssp_split **out) {
    if (!g || !out) return fail(GX_NULL_POINTER, "gx_sssp_split_create: null argument");
    if (!g->weighted) return fail(GX_INVALID_VALUE, "gx_sssp_split_create: graph has no edge weights");
    if (v0 > v1 || v1 > g->n) return fail(GX_INVALID_INDEX, "gx_sssp_split_create: bad vertex range");
    if (g->n >= (1ull << 31)) return fail(GX_NOT_IMPLEMENTED, "gx_sssp_split_create: more than 2^31 vertices");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipStream_t s = g->ctx->stream;
    std::unique_ptr<gx_sssp_split> p(new gx_sssp_split());
    p->g = g;
    p->n = (int64_t)g->n;
    p->v0 = (int64_t)v0;
    p->v1 = (int64_t)v1;
    const int64_t n = p->n, own = p->v1 - p->v0;
    // bucket width: gx_sssp's rule (scale x mean weight / mean degree; GX_SSSP_DELTA and
    // GX_SSSP_DSCALE override) -- any positive value gives the same distances
    double mean = 1.0;
    if (g->nnz) {
        DBuf<double> sum;
        GX_TRY(sum.alloc(1));
        GX_HIP_TRY(hipMemsetAsync(sum.p, 0, sizeof(double), s));
        hipLaunchKernelGGL(k_split_sum_w, dim3(grid_for(g->nnz, 256, 4096)), dim3(256), 0, s, g->A.w.p,
                           (int64_t)g->nnz, sum.p);
        GX_TRY(check_launch("k_split_sum_w"));
        double h = 0.0;
        GX_HIP_TRY(hipMemcpyAsync(&h, sum.p, sizeof(double), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        mean = h / (double)g->nnz;
    }
    double scale = g->directed ? 0.5 : 4.0, delta = 0.0;
    if (const char *e = std::getenv("GX_SSSP_DSCALE")) scale = std::atof(e);
    if (const char *e = std::getenv("GX_SSSP_DELTA")) delta = std::atof(e);
    if (!(delta > 0.0)) delta = scale * mean / std::max(1.0, (double)g->nnz / std::max<double>(1.0, (double)n));
    if (!(delta > 0.0) || !std::isfinite(delta)) delta = 1.0;
    p->delta = delta;
    // slice: count, scan, scatter
    GX_TRY(p->srp.alloc(n + 1));
    GX_TRY(p->slend.alloc(std::max<int64_t>(n, 1)));
    {
        DBuf<int64_t> lc, tc;
        GX_TRY(lc.alloc(std::max<int64_t>(n, 1)));
        GX_TRY(tc.alloc(n + 1));
        const unsigned wg = grid_for((uint64_t)n * kWave, kSB, 16384);
        if (n) {
            hipLaunchKernelGGL(k_slice_count, dim3(wg), dim3(kSB), 0, s, g->A.rp.p, g->A.ci.p, g->A.w.p, n, p->v0, p->v1,
                               delta, lc.p, tc.p);
            GX_TRY(check_launch("k_slice_count"));
        } else {
            GX_HIP_TRY(hipMemsetAsync(tc.p, 0, sizeof(int64_t), s));
        }
        GX_TRY(scan_exclusive_i64(tc.p, p->srp.p, (size_t)(n + 1), s));
        GX_HIP_TRY(hipMemcpyAsync(&p->snnz, p->srp.p + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        GX_TRY(p->sci.alloc(std::max<int64_t>(p->snnz, 1)));
        GX_TRY(p->sw.alloc(std::max<int64_t>(p->snnz, 1)));
        if (n) {
            hipLaunchKernelGGL(k_slice_scatter, dim3(wg), dim3(kSB), 0, s, g->A.rp.p, g->A.ci.p, g->A.w.p, n, p->v0,
                               p->v1, delta, p->srp.p, lc.p, p->slend.p, p->sci.p, p->sw.p);
            GX_TRY(check_launch("k_slice_scatter"));
        }
        GX_HIP_TRY(hipStreamSynchronize(s));   // lc / tc die here
    }
    // state: item lists hold at most one item per vertex plus one per 256 slice entries
    const uint64_t icap = (uint64_t)n + (uint64_t)p->snnz / kSChunk + 64;
    GX_TRY(p->dist.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(p->lrel.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(p->sstamp.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(p->pstamp.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(p->istamp.alloc(std::max<int64_t>(own, 1)));
    GX_TRY(p->plist0.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(p->plist1.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(p->imp.alloc(std::max<int64_t>(own, 1)));
    GX_TRY(p->fitems0.alloc(icap));
    GX_TRY(p->fitems1.alloc(icap));
    GX_TRY(p->sitems.alloc(icap));
    GX_TRY(p->own_pairs.alloc(2 * (uint64_t)std::max<int64_t>(own, 1)));
    GX_TRY(p->own_count.alloc(2));
    GX_TRY(p->st.alloc(1));
    GX_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&p->h_done), 2 * sizeof(int32_t), hipHostMallocDefault));
    p->grid = (unsigned)std::max(1, g->ctx->num_cus) * 8;
    *out = p.release();
    return GX_SUCCESS;
}

extern "C" int gx_sssp_split_free(gx_sssp_split *p) {
    if (p) {
        (void)hipSetDevice(p->g->ctx->device);
        delete p;
    }
    return GX_SUCCESS;
}

extern "C" int gx_sssp_split_delta(gx_sssp_split *p, double *delta) {
    if (!p || !delta) return fail(GX_NULL_POINTER, "gx_sssp_split_delta: null argument");
    *delta = p->delta;
    return GX_SUCCESS;
}

extern "C" int gx_sssp_split_start(gx_sssp_split *p, uint64_t src, void *stream) {
    if (!p) return fail(GX_NULL_POINTER, "gx_sssp_split_start: null argument");
    if (src >= (uint64_t)p->n) return fail(GX_INVALID_INDEX, "gx_sssp_split_start: source out of range");
    GX_HIP_TRY(hipSetDevice(p->g->ctx->device));
    hipStream_t s = split_stream(p, stream);
    const SplitBufs B = p->bufs();
    hipLaunchKernelGGL(k_split_start, dim3(grid_for(std::max<int64_t>(p->n, 1), kSB, 8192)), dim3(kSB), 0, s, B,
                       (int64_t)src);
    hipLaunchKernelGGL(k_split_seed, dim3(1), dim3(kSB), 0, s, B, (int64_t)src);
    return check_launch("k_split_seed");
}

extern "C" int gx_sssp_split_relax(gx_sssp_split *p, uint64_t *pairs, uint64_t *count, void *stream) {
    if (!p || !pairs || !count) return fail(GX_NULL_POINTER, "gx_sssp_split_relax: null argument");
    GX_HIP_TRY(hipSetDevice(p->g->ctx->device));
    return split_relax(p, pairs, count, split_stream(p, stream));
}

extern "C" int gx_sssp_split_apply(gx_sssp_split *p, const uint64_t *pairs, const uint64_t *counts, int nranks,
                                   uint64_t stride, void *stream) {
    if (!p || !counts || (nranks > 0 && !pairs && stride)) return fail(GX_NULL_POINTER, "gx_sssp_split_apply: null argument");
    if (nranks < 1) return fail(GX_INVALID_VALUE, "gx_sssp_split_apply: nranks < 1");
    GX_HIP_TRY(hipSetDevice(p->g->ctx->device));
    return split_apply(p, pairs, counts, nranks, stride, split_stream(p, stream));
}

extern "C" int gx_sssp_split_distances(gx_sssp_split *p, double *dist, void *stream) {
    if (!p || !dist) return fail(GX_NULL_POINTER, "gx_sssp_split_distances: null argument");
    GX_HIP_TRY(hipSetDevice(p->g->ctx->device));
    GX_HIP_TRY(hipMemcpyAsync(dist, p->dist.p, (size_t)p->n * 8, hipMemcpyDeviceToDevice, split_stream(p, stream)));
    return GX_SUCCESS;
}

// One rank owning every vertex: the rounds run back to back on the device (the apply reads
// this rank's own pairs), the host polls the done flag once per batch of rounds.
extern "C" int gx_sssp_split_run(gx_sssp_split *p, uint64_t src, double *dist_host) {
    if (!p || !dist_host) return fail(GX_NULL_POINTER, "gx_sssp_split_run: null argument");
    if (p->v0 != 0 || p->v1 != p->n) return fail(GX_INVALID_VALUE, "gx_sssp_split_run: the rank must own every vertex");
    gx_ctx *ctx = p->g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    GX_TRY(device_begin(ctx));
    GX_TRY(gx_sssp_split_start(p, src, s));
    constexpr int kBatch = 16;
    for (int64_t guard = 0;; guard++) {
        for (int k = 0; k < kBatch; k++) {
            GX_TRY(split_relax(p, p->own_pairs.p, p->own_count.p, s));
            GX_TRY(split_apply(p, p->own_pairs.p, p->own_count.p, 1, (uint64_t)std::max<int64_t>(p->n, 1), s));
        }
        GX_HIP_TRY(hipMemcpyAsync(p->h_done, &p->st.p->done, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        if (*p->h_done) break;
        if (guard > 4 * (p->n + 16)) return fail(GX_DEVICE_ERROR, "gx_sssp_split_run: no fixed point");
    }
    GX_TRY(device_end(ctx));
    GX_HIP_TRY(hipMemcpy(dist_host, p->dist.p, (size_t)p->n * 8, hipMemcpyDeviceToHost));
    return GX_SUCCESS;
}

GX_MODULE_WARMER(sssp_split)
