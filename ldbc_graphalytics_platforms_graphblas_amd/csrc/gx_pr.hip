// gx_pr.hip -- PageRank (Graphalytics definition) as one fused pull-SpMV per iteration.
//
// Replaces LA_PR -> LAGraph_Cached_OutDegree + LAGraph_Cached_AT + LAGr_PageRankGX
// (pr.cpp:47-66), whose hot loop is one GrB_mxv PLUS_SECOND over A' per iteration.
//
// Per iteration, for every vertex v of the rank's rows:
//     teleport = (1-d)/n + d/n * sum_k dangling_k           (k over ranks, fixed order)
//     r(v)     = teleport + sum_{u in in(v)} x(u)
//     x'(v)    = outdeg(v) > 0 ? r(v) / (outdeg(v)/d) : r(v)
// where x(u) = r(u)/(outdeg(u)/d) is what the previous iteration stored, and a dangling
// vertex stores r itself (it has no out-edges, so nobody gathers its slot).  That is the
// GX arithmetic of the oracle (oracle/gx_oracle.c orc_pagerank) with the division by the
// out-degree fused into the producer of x instead of a separate GrB_eWiseMult pass.
//
// HBM traffic per iteration (algorithmic): 4 B per stored entry (int32 column index),
// 8 B row pointer + 4 B out-degree + 8 B x write per row, the x gathers (L2 / MALL
// resident for the graphs we run), and 8 B per row for the scores in the last iteration.
//
// k_pr_pull is CSR-Adaptive (Greathouse & Daga): rows are packed into workgroups of at
// most kStreamNnz entries; a workgroup streams its contiguous column-index range with
// 16-B loads, gathers x into LDS, then reduces each row with a power-of-two lane group.
// Rows longer than kStreamNnz get whole workgroups (split into kSegNnz segments, combined
// by the last-arriving segment through an agent-scope release/acquire ticket), and are
// dispatched first so they overlap the stream blocks.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <thread>

#include "gx_pr.h"

namespace gx {
namespace {

struct PullArgs {
    const RowBlock *blocks;
    const int64_t *rp;
    const int32_t *ci;
    const int32_t *outdeg;
    const double *x_in;
    double *x_out;
    int64_t block_offset;
    double *rank_out;
    int64_t chunk;
    int nranks;
    int zero_slot;
    double teleport0, damping_over_n, damping;
    const int32_t *long_first;
    const int32_t *long_nseg;
    double *long_part;
    uint32_t *long_ticket;
    double *xd;
    int64_t live;
};

__device__ __forceinline__ void pr_epilogue(const PullArgs &a, int32_t row, double s,
                                            double teleport) {
    const double r = teleport + s;
    if (a.rank_out) a.rank_out[row] = r;
    const int32_t deg = a.outdeg[row];
    store_x(a.x_out, a.xd, a.live, row, deg > 0 ? r / ((double)deg / a.damping) : r);
}

template <int NB, bool STRIDE1>
__global__ __launch_bounds__(kPullBlock) void k_pr_pull(PullArgs a) {
    __shared__ __attribute__((aligned(16))) double vals[NB + 4];
    __shared__ int32_t rofs[kStreamRows + 1];
    __shared__ double wred[kPullBlock / kWave];

    const RowBlock b = a.blocks[a.block_offset + blockIdx.x];
    const int tid = threadIdx.x;

    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    if (a.zero_slot && blockIdx.x == 0 && tid == 0) a.x_out[a.chunk - 1] = 0.0;

    if (b.split < 0) {
        // ---------------- STREAM: short rows staged through LDS ----------------
        const int64_t z0 = b.nz_begin, z1 = b.nz_end;
        const int32_t r0 = b.row_begin;
        const int nrows = b.row_end - b.row_begin;
        // LDS is indexed from the 16-B aligned `base`, so every lane stores its four values
        // as two aligned 16-B words; the reduction only reads [rofs[r], rofs[r+1]).
        const int64_t base = z0 & ~(int64_t)3;
        for (int i = tid; i <= nrows; i += kPullBlock) rofs[i] = (int32_t)(a.rp[r0 + i] - base);
        const int nq = (int)((z1 - base + 3) >> 2);
        const int4 *ci4 = reinterpret_cast<const int4 *>(a.ci) + (base >> 2);
        // lane group per row, fixed for the block; the epilogue's out-degree is fetched early
        int L = kWave;
        while (L > 1 && L * nrows > kPullBlock) L >>= 1;
        const int row = tid / L, lane = tid & (L - 1);
        const bool writer = row < nrows && lane == 0;
        const int32_t deg = writer ? a.outdeg[r0 + row] : 0;
        if (STRIDE1) {
            // Lane-consecutive entries: gather instruction j of a wave covers 64 consecutive
            // entries, so with every row sorted by (hub-first) column id neighbouring lanes
            // often hit the same x cache line -- one L1 miss serves several gathers.  The
            // L1-miss count is what bounds this kernel (~70 misses in flight per CU).
            constexpr int NE = (NB + 3 + kPullBlock - 1) / kPullBlock;
            const int64_t last = z1 > base ? z1 - 1 : base;   // clamp: index loads stay valid
            int32_t c[NE];
#pragma unroll
            for (int j = 0; j < NE; j++)
                c[j] = __builtin_nontemporal_load(a.ci + min(base + tid + (int64_t)j * kPullBlock, last));
            double v[NE];
#pragma unroll
            for (int j = 0; j < NE; j++) v[j] = a.x_in[c[j]];
#pragma unroll
            for (int j = 0; j < NE; j++) {
                const int e = tid + j * kPullBlock;
                if (base + e < z1) vals[e] = v[j];
            }
        } else {
        constexpr int NQ = (NB / 4 + kPullBlock) / kPullBlock;
        // Column indices: 16 B per lane, non-temporal (read once; keep L2 for x).  Every
        // index read here is a valid x offset (neighbouring rows' entries, or the zeroed
        // slack past the end), so all gathers below are issued unconditionally.
        int4 c[NQ];
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + j * kPullBlock;
            c[j] = q < nq ? load_nt(ci4 + q) : make_int4(0, 0, 0, 0);
        }
        double v[NQ][4];
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            v[j][0] = a.x_in[c[j].x];
            v[j][1] = a.x_in[c[j].y];
            v[j][2] = a.x_in[c[j].z];
            v[j][3] = a.x_in[c[j].w];
        }
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + j * kPullBlock;
            if (q < nq) {
                double2 *d = reinterpret_cast<double2 *>(&vals[4 * q]);
                d[0] = make_double2(v[j][0], v[j][1]);
                d[1] = make_double2(v[j][2], v[j][3]);
            }
        }
        }
        __syncthreads();
        double s = 0.0;
        if (row < nrows) {
            const int kb = rofs[row], ke = rofs[row + 1];
            for (int k = kb + lane; k < ke; k += L) s += vals[k];
        }
        for (int off = L >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
        if (writer) {
            const double r = teleport + s;
            if (a.rank_out) a.rank_out[r0 + row] = r;
            store_x(a.x_out, a.xd, a.live, r0 + row, deg > 0 ? r / ((double)deg / a.damping) : r);
        }
        return;
    }

    // ---------------- LONG: one segment of one long row ----------------
    const int64_t zb = b.nz_begin, ze = b.nz_end;
    double s0 = 0.0, s1 = 0.0;
    if (STRIDE1) {
        // lane-consecutive entries, 8 loads in flight per lane, clamped (always valid)
        constexpr int U = 8;
        for (int64_t k0 = zb + tid; k0 < ze; k0 += (int64_t)U * kPullBlock) {
            int32_t c[U];
#pragma unroll
            for (int u = 0; u < U; u++)
                c[u] = __builtin_nontemporal_load(a.ci + min(k0 + (int64_t)u * kPullBlock, ze - 1));
            double g[U];
#pragma unroll
            for (int u = 0; u < U; u++) g[u] = a.x_in[c[u]];
#pragma unroll
            for (int u = 0; u < U; u++)
                if (k0 + (int64_t)u * kPullBlock < ze) ((u & 1) ? s1 : s0) += g[u];
        }
    }
    const int64_t base = zb & ~(int64_t)3;
    const int64_t nq = STRIDE1 ? 0 : (ze - base + 3) >> 2;
    const int4 *ci4 = reinterpret_cast<const int4 *>(a.ci) + (base >> 2);
    for (int64_t q = tid; q < nq; q += 2 * kPullBlock) {
        const int64_t q1 = q + kPullBlock;
        const int4 c0 = load_nt(ci4 + q);
        const int4 c1 = q1 < nq ? load_nt(ci4 + q1) : make_int4(0, 0, 0, 0);
        const int64_t e0 = base + 4 * q, e1 = base + 4 * q1;
        const int a0[4] = {c0.x, c0.y, c0.z, c0.w};
        const int a1[4] = {c1.x, c1.y, c1.z, c1.w};
        double g0[4], g1[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {   // unconditional gathers, masked adds
            g0[k] = a.x_in[a0[k]];
            g1[k] = a.x_in[a1[k]];
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (!(e0 + k >= zb && e0 + k < ze)) g0[k] = 0.0;
            if (!(e1 + k >= zb && e1 + k < ze)) g1[k] = 0.0;
        }
        s0 += (g0[0] + g0[1]) + (g0[2] + g0[3]);
        s1 += (g1[0] + g1[1]) + (g1[2] + g1[3]);
    }
    double s = wave_sum(s0 + s1);
    if ((tid & (kWave - 1)) == 0) wred[tid / kWave] = s;
    __syncthreads();
    if (tid != 0) return;
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < kPullBlock / kWave; w++) tot += wred[w];
    const int32_t sp = b.split;
    const int32_t nseg = a.long_nseg[sp];
    if (nseg == 1) {
        pr_epilogue(a, b.row_begin, tot, teleport);
        return;
    }
    const int32_t first = a.long_first[sp];
    // publish the partial (agent scope), then take a ticket; the last arriver combines
    __hip_atomic_store(&a.long_part[first + b.seg], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(&a.long_ticket[sp], 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t != (uint32_t)(nseg - 1)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    double all = 0.0;
    for (int j = 0; j < nseg; j++)
        all += __hip_atomic_load(&a.long_part[first + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.long_ticket[sp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pr_epilogue(a, b.row_begin, all, teleport);
}

// Sum of the scores of this rank's dangling vertices into the chunk's last slot.
// dlist == nullptr: the dangling rows are the contiguous range [d0, d0 + nd) (hub-first
// order puts every out-degree-0 vertex last), read coalesced.  Workgroup partials are
// combined by the last arriver's whole workgroup in a fixed order (deterministic).
__global__ __launch_bounds__(256) void k_pr_dangling(const int32_t *__restrict__ dlist, int64_t d0,
                                                     int64_t nd, int64_t per, double *x, int64_t slot,
                                                     double *part, uint32_t *ticket, const double *xd,
                                                     int64_t live) {
    __shared__ double wred[256 / kWave];
    __shared__ int last;
    const int tid = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(b0 + per, nd);
    double s = 0.0;
    if (dlist) {
        for (int64_t i = b0 + tid; i < b1; i += 256) {
            const int64_t r = dlist[i];
            s += r < live ? x[r] : xd[r - live];
        }
    } else {
        for (int64_t i = b0 + tid; i < b1; i += 256) {
            const int64_t r = d0 + i;
            s += r < live ? x[r] : xd[r - live];
        }
    }
    s = wave_sum(s);
    if ((tid & (kWave - 1)) == 0) wred[tid / kWave] = s;
    __syncthreads();
    const uint32_t G = gridDim.x;
    if (tid == 0) {
        const double tot = (wred[0] + wred[1]) + (wred[2] + wred[3]);
        if (G == 1) {
            x[slot] = tot;
            last = 0;
        } else {
            __hip_atomic_store(&part[blockIdx.x], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
        }
    }
    __syncthreads();
    if (!last) return;
    // the last arriver sums the partials with the whole workgroup (a serial loop of agent-
    // scope loads by one thread took ~20 us); thread t always takes partials t, t+256, ...
    // and the tree below is fixed, so the sum is the same in every run
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    double a = 0.0;
    for (uint32_t j = tid; j < G; j += 256) a += __hip_atomic_load(&part[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a = wave_sum(a);
    __syncthreads();
    if ((tid & (kWave - 1)) == 0) wred[tid / kWave] = a;
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x[slot] = (wred[0] + wred[1]) + (wred[2] + wred[3]);
    }
}

// x = PR_0 / (outdeg / d) (dangling rows: PR_0 itself), and the chunk's dangling slot = the
// sum of its dangling rows' PR_0 = nd / n, known at plan time (no k_pr_dangling launch per run).
__global__ void k_pr_init(const int32_t *__restrict__ outdeg, int64_t rows, double inv_n,
                          double damping, double *x, int64_t slot, double dangling0, double *xd, int64_t live) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t deg = outdeg[i];
        store_x(x, xd, live, i, deg > 0 ? inv_n / ((double)deg / damping) : inv_n);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) x[slot] = dangling0;
}

}  // namespace

int pr_plan(PrPart *p, HostView<int64_t> h_rp, const int64_t *d_rp, const int32_t *d_ci,
            const int32_t *d_outdeg, HostView<int32_t> h_outdeg) {
    const int64_t rows = (int64_t)h_rp.size() - 1;
    p->rows = (uint64_t)rows;
    if (p->live > p->rows) p->live = p->rows;   // no live prefix given: all rows
    if (p->live < p->rows) GX_TRY(p->xd.alloc(p->rows - p->live));
    p->rp = d_rp;
    p->ci = d_ci;
    p->outdeg = d_outdeg;
    // kernel choice: GX_PR_KERNEL = sorted (default) | adaptive (CSR-Adaptive k_pr_pull: row-order
    // sums, bitwise deterministic, ~3x slower)
    if (const char *e = std::getenv("GX_PR_KERNEL")) p->kernel = std::strcmp(e, "adaptive") == 0 ? 1 : 2;
    PlanClock clk("pr_plan", p->ctx->stream);
    if (p->kernel == 1) {
        const int64_t NB = kStreamNnz;
        std::vector<RowBlock> longb, streamb;
        std::vector<int32_t> lfirst, lnseg;
        int32_t nsegs = 0;
        std::vector<std::pair<int64_t, int32_t>> longrows;   // (length, row)
        int64_t r = 0;
        while (r < rows) {
            const int64_t len = h_rp[r + 1] - h_rp[r];
            if (len > NB) {
                longrows.push_back({len, (int32_t)r});
                r++;
                continue;
            }
            const int64_t start = r;
            int64_t nz = 0;
            while (r < rows && r - start < kStreamRows) {
                const int64_t l = h_rp[r + 1] - h_rp[r];
                if (l > NB || nz + l > NB) break;
                nz += l;
                r++;
            }
            streamb.push_back({h_rp[start], h_rp[r], (int32_t)start, (int32_t)r, -1, 0});
        }
        // longest rows first: they are the tail of the launch otherwise
        std::stable_sort(longrows.begin(), longrows.end(),
                         [](const auto &x, const auto &y) { return x.first > y.first; });
        for (const auto &lr : longrows) {
            const int32_t row = lr.second;
            const int64_t len = lr.first;
            const int32_t nseg = (int32_t)((len + kSegNnz - 1) / kSegNnz);
            const int32_t sp = (int32_t)lfirst.size();
            lfirst.push_back(nsegs);
            lnseg.push_back(nseg);
            for (int32_t s = 0; s < nseg; s++) {
                const int64_t zb = h_rp[row] + (int64_t)s * kSegNnz;
                const int64_t ze = std::min(zb + kSegNnz, h_rp[row + 1]);
                longb.push_back({zb, ze, row, row + 1, sp, s});
            }
            nsegs += nseg;
        }
        std::vector<RowBlock> all;
        all.reserve(longb.size() + streamb.size());
        all.insert(all.end(), longb.begin(), longb.end());
        all.insert(all.end(), streamb.begin(), streamb.end());
        p->nblocks = (uint32_t)all.size();
        p->nlong_blocks = (uint32_t)longb.size();
        p->nlong = (uint32_t)lfirst.size();
        p->nsegs = (uint32_t)nsegs;
        GX_TRY(p->blocks.alloc(std::max<size_t>(all.size(), 1)));
        GX_TRY(p->long_first.alloc(std::max<size_t>(lfirst.size(), 1)));
        GX_TRY(p->long_nseg.alloc(std::max<size_t>(lnseg.size(), 1)));
        GX_TRY(p->long_part.alloc(std::max<size_t>(nsegs, 1)));
        GX_TRY(p->long_ticket.alloc(std::max<size_t>(lfirst.size(), 1)));
        if (!all.empty())
            GX_HIP_TRY(hipMemcpy(p->blocks.p, all.data(), all.size() * sizeof(RowBlock), hipMemcpyHostToDevice));
        if (!lfirst.empty()) {
            GX_HIP_TRY(hipMemcpy(p->long_first.p, lfirst.data(), lfirst.size() * 4, hipMemcpyHostToDevice));
            GX_HIP_TRY(hipMemcpy(p->long_nseg.p, lnseg.data(), lnseg.size() * 4, hipMemcpyHostToDevice));
        }
        GX_HIP_TRY(hipMemset(p->long_ticket.p, 0, p->long_ticket.n * 4));
    }
    // dangling rows: one contiguous range (hub-first orders put them last), or a list
    int64_t nd = 0, dfirst = -1, dlast = -1;
    if (p->src_order) {
        // gx_pagerank's hub-first rows: out-degrees non-increasing, the dangling rows a suffix
        int64_t lo = 0, hi = rows;
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (h_outdeg[mid] == 0) hi = mid;
            else lo = mid + 1;
        }
        nd = rows - lo;
        if (nd > 0) {
            dfirst = lo;
            dlast = rows - 1;
        }
    } else {
        for (int64_t i = 0; i < rows; i++)
            if (h_outdeg[i] == 0) {
                nd++;
                if (dfirst < 0) dfirst = i;
                dlast = i;
            }
    }
    p->nd = (uint64_t)nd;
    p->d_range = nd > 0 && dlast - dfirst + 1 == nd;
    p->d0 = nd > 0 ? dfirst : 0;
    if (!p->d_range) {
        std::vector<int32_t> dl;
        for (int64_t i = 0; i < rows; i++)
            if (h_outdeg[i] == 0) dl.push_back((int32_t)i);
        GX_TRY(p->dlist.alloc(std::max<size_t>(dl.size(), 1)));
        if (!dl.empty())
            GX_HIP_TRY(hipMemcpy(p->dlist.p, dl.data(), dl.size() * 4, hipMemcpyHostToDevice));
    }
    p->dgrid = (uint32_t)std::min<uint64_t>(512, std::max<uint64_t>(1, (p->nd + 2047) / 2048));
    GX_TRY(p->dpart.alloc(p->dgrid));
    GX_TRY(p->dticket.alloc(1));
    GX_HIP_TRY(hipMemset(p->dticket.p, 0, 4));
    clk.mark("adaptive blocks + dangling");
    if (p->kernel == 2) GX_TRY(pr_plan_sorted(p, h_rp, h_outdeg));
    return GX_SUCCESS;
}

int pr_dangling(PrPart *p, double *x_local, hipStream_t s) {
    if (p->nd == 0) return GX_SUCCESS;
    const int64_t per = (int64_t)((p->nd + p->dgrid - 1) / p->dgrid);
    hipLaunchKernelGGL(k_pr_dangling, dim3(p->dgrid), dim3(256), 0, s, p->d_range ? nullptr : p->dlist.p,
                       (int64_t)p->d0, (int64_t)p->nd, per,
                       x_local, (int64_t)p->chunk - 1, p->dpart.p, p->dticket.p, p->xd.p, (int64_t)p->live);
    return check_launch("k_pr_dangling");
}

int pr_init(PrPart *p, double *x_local, hipStream_t s) {
    const double inv_n = 1.0 / (double)p->n_global;
    hipLaunchKernelGGL(k_pr_init, dim3(grid_for(p->rows, 256, 8192)), dim3(256), 0, s, p->outdeg,
                       (int64_t)p->rows, inv_n, p->damping, x_local, (int64_t)p->chunk - 1,
                       (double)p->nd / (double)p->n_global, p->xd.p, (int64_t)p->live);
    return check_launch("k_pr_init");
}

int pr_step(PrPart *p, const double *x_full, double *x_local, double *rank_out, hipStream_t s) {
    if (p->kernel == 2) return pr_step_sorted(p, x_full, x_local, rank_out, s);
    const double dn = (double)p->n_global;
    PullArgs a;
    a.blocks = p->blocks.p;
    a.rp = p->rp;
    a.ci = p->ci;
    a.outdeg = p->outdeg;
    a.x_in = x_full;
    a.x_out = x_local;
    a.rank_out = rank_out;
    a.chunk = (int64_t)p->chunk;
    a.nranks = p->nranks;
    a.zero_slot = p->nd == 0 ? 1 : 0;
    a.teleport0 = (1.0 - p->damping) / dn;
    a.damping_over_n = p->damping / dn;
    a.damping = p->damping;
    a.long_first = p->long_first.p;
    a.long_nseg = p->long_nseg.p;
    a.long_part = p->long_part.p;
    a.long_ticket = p->long_ticket.p;
    a.xd = p->xd.p;
    a.live = (int64_t)p->live;
    a.block_offset = 0;
    if (p->nblocks) {
        KTimer kt(p->ctx, "pr_pull", s);
        hipLaunchKernelGGL((k_pr_pull<kStreamNnz, true>), dim3(p->nblocks), dim3(kPullBlock), 0, s, a);
    }
    GX_TRY(check_launch("k_pr_pull"));
    return pr_dangling(p, x_local, s);
}

}  // namespace gx

using namespace gx;

static uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

namespace {

// Relabel a CSR by `perm` (old vertex -> new position): row perm[r] of the result holds the
// entries of row r with every column c renamed perm[c].  Edge-balanced, no sort.
// keys[e] = (perm[row] << 32) | perm[col] for every entry: sorted, they give the relabelled
// CSR with every row sorted by new column id.  Edge-balanced.
__global__ void k_permute_keys(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, int64_t n,
                               int64_t nnz, const int32_t *__restrict__ perm, uint64_t *__restrict__ keys) {
    constexpr int kPer = 16;
    const int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kPer;
    if (e0 >= nnz) return;
    const int64_t e1 = min(e0 + kPer, nnz);
    int64_t r = row_of_edge(rp, n, e0);
    for (int64_t e = e0; e < e1; e++) {
        while (rp[r + 1] <= e) r++;
        keys[e] = ((uint64_t)(uint32_t)perm[r] << 32) | (uint32_t)perm[ci[e]];
    }
}

// out[v] = in[perm[v]]: back from the hub-first order to the caller's vertex order.
__global__ void k_gather_perm(const double *__restrict__ in, const int32_t *__restrict__ perm, int64_t n,
                              double *__restrict__ out) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x)
        out[v] = in[perm[v]];
}

// Device hub-first order: keys (2^31 - 1 - outdeg) << 32 | v sort ascending into out-degree
// descending, ties by id (the host hub_order's order, which the adaptive kernel's plan keeps).
// (out-degree, vertex) pairs; a stable descending sort of the degrees gives the hub-first order
// (degree descending, ties by id)
__global__ void k_hub_keys(const int32_t *__restrict__ outdeg, int64_t n, uint32_t *__restrict__ deg,
                           int32_t *__restrict__ ids) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        deg[v] = (uint32_t)outdeg[v];
        ids[v] = (int32_t)v;
    }
}

// order[i] = v, perm[v] = i, the hub-first row's out-degree and pull length (plen[n] = 0, so an
// exclusive scan of n + 1 values gives the relabelled row pointers)
__global__ void k_hub_apply(const int32_t *__restrict__ sorted_ids, int64_t n, const int32_t *__restrict__ outdeg,
                            const int64_t *__restrict__ prp, int32_t *__restrict__ order, int32_t *__restrict__ perm,
                            int32_t *__restrict__ nout, int64_t *__restrict__ plen) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i == n) {
            plen[n] = 0;
            continue;
        }
        const int32_t v = sorted_ids[i];
        order[i] = v;
        perm[v] = (int32_t)i;
        nout[i] = outdeg[v];
        plen[i] = prp[v + 1] - prp[v];
    }
}

// Runs of equal values in the sorted (non-increasing) degrees: (position << 32 | degree) of
// every run's first element, in any order; the count may pass `cap` (then nothing past it is
// written and the caller falls back to the full arrays).
__global__ void k_degree_runs(const uint32_t *__restrict__ sdeg, int64_t n, uint64_t *__restrict__ runs,
                              uint32_t *__restrict__ count, uint32_t cap) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i > 0 && sdeg[i] == sdeg[i - 1]) continue;
        const uint32_t k = atomicAdd(count, 1u);
        if (k < cap) runs[k] = ((uint64_t)i << 32) | sdeg[i];
    }
}

// Device `d` of `ndev` (gx_pagerank_multi's interleaved partition): its local row j is hub-first
// position i = d + j ndev; the row's source vertex, out-degree and pull length (plen[rows] = 0
// for the exclusive scan).
__global__ void k_multi_pick(const int32_t *__restrict__ order, const int32_t *__restrict__ nout,
                             const int64_t *__restrict__ plen, int ndev, int d, int64_t rows,
                             int32_t *__restrict__ my_order, int32_t *__restrict__ my_out,
                             int64_t *__restrict__ my_plen) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= rows; j += (int64_t)gridDim.x * blockDim.x) {
        if (j == rows) {
            my_plen[rows] = 0;
            continue;
        }
        const int64_t i = (int64_t)d + j * ndev;
        my_order[j] = order[i];
        my_out[j] = nout[i];
        my_plen[j] = plen[i];
    }
}

// vertex -> its slot in the exchanged vector: owner (i mod ndev) * chunk + local row (i / ndev)
__global__ void k_multi_colmap(const int32_t *__restrict__ perm, int64_t n, int ndev, int64_t chunk,
                               int32_t *__restrict__ colmap) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = perm[v];
        colmap[v] = (int32_t)((i % ndev) * chunk + i / ndev);
    }
}

// Rows of device d's block partition: hub-first positions pos[j] (MultiBlocks).
__global__ void k_block_pick(const int32_t *__restrict__ order, const int32_t *__restrict__ nout,
                             const int64_t *__restrict__ plen, const int32_t *__restrict__ pos, int64_t rows,
                             int32_t *__restrict__ my_order, int32_t *__restrict__ my_out,
                             int64_t *__restrict__ my_plen) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= rows; j += (int64_t)gridDim.x * blockDim.x) {
        if (j == rows) {
            my_plen[rows] = 0;
            continue;
        }
        const int64_t i = pos[j];
        my_order[j] = order[i];
        my_out[j] = nout[i];
        my_plen[j] = plen[i];
    }
}

// vertex -> its exchange slot through its hub-first position (MultiBlocks::slot)
__global__ void k_block_colmap(const int32_t *__restrict__ perm, int64_t n, const int32_t *__restrict__ slot,
                               int32_t *__restrict__ colmap) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        colmap[v] = slot[perm[v]];
}

// Hub-first order: vertices by out-degree descending, ties by id (stable counting sort).
// The pull SpMV gathers x(u) once per out-edge of u, so this packs the most gathered
// entries of x into its first few MiB, which stay resident in each XCD's 4 MiB L2.
void hub_order(const std::vector<int32_t> &outdeg, std::vector<int32_t> &order, std::vector<int32_t> &perm) {
    const size_t n = outdeg.size();
    int32_t maxd = 0;
    for (int32_t d : outdeg) maxd = std::max(maxd, d);
    std::vector<int64_t> start((size_t)maxd + 2, 0);
    for (int32_t d : outdeg) start[(size_t)(maxd - d) + 1]++;
    for (size_t k = 1; k < start.size(); k++) start[k] += start[k - 1];
    order.assign(n, 0);
    perm.assign(n, 0);
    for (size_t v = 0; v < n; v++) {
        const int64_t pos = start[(size_t)(maxd - outdeg[v])]++;
        order[pos] = (int32_t)v;
        perm[v] = (int32_t)pos;
    }
}

}  // namespace

// The CSR-Adaptive kernel's plan (GX_PR_KERNEL=adaptive): the hub-first relabelled pull CSR
// itself, built by a radix sort of (perm[row] << 32 | perm[col]) keys.
static int pr_single_plan_adaptive(gx_graph *g, PrPart **out) {
    const uint64_t n = g->n;
    gx_ctx *ctx = g->ctx;
    hipStream_t s = ctx->stream;
    DevCSR &P = g->directed ? g->AT : g->A;
    PlanClock clk("single", s);
    GX_TRY(ensure_host_rp(ctx, g->A));
    std::vector<int32_t> h_outdeg(n), order, perm;
    for (uint64_t v = 0; v < n; v++) h_outdeg[v] = (int32_t)(g->A.h_rp[v + 1] - g->A.h_rp[v]);
    hub_order(h_outdeg, order, perm);
    clk.mark("outdeg + hub order (host)");
    std::vector<int64_t> nrp(n + 1, 0);
    std::vector<int32_t> nout(n);
    for (uint64_t i = 0; i < n; i++) {
        const int32_t v = order[i];
        nrp[i + 1] = nrp[i] + (P.h_rp[v + 1] - P.h_rp[v]);
        nout[i] = h_outdeg[v];
    }
    auto *p = new PrPart();
    p->ctx = ctx;
    p->n_global = n;
    p->nranks = 1;
    p->rank = 0;
    p->chunk = round_up(n + 2, 32);   // + a zero padding slot (chunk - 2) and the dangling slot
    int rc = p->perm.alloc(n);
    if (rc == GX_SUCCESS) rc = p->rp_own.alloc(n + 1);
    if (rc == GX_SUCCESS) rc = p->ci_own.alloc(P.nnz, 16);
    if (rc == GX_SUCCESS) rc = p->outdeg_own.alloc(n);
    if (rc == GX_SUCCESS) rc = p->xa.alloc(p->chunk);
    if (rc == GX_SUCCESS) rc = p->xb.alloc(p->chunk);
    if (rc == GX_SUCCESS) rc = p->rank_out.alloc(n);
    if (rc == GX_SUCCESS) rc = p->result.alloc(n);
    hipError_t e = hipSuccess;
    if (rc == GX_SUCCESS) e = hipMemsetAsync(p->xa.p, 0, p->chunk * sizeof(double), s);
    if (rc == GX_SUCCESS && e == hipSuccess) e = hipMemsetAsync(p->xb.p, 0, p->chunk * sizeof(double), s);
    if (rc == GX_SUCCESS && e == hipSuccess) e = hipMemcpyAsync(p->perm.p, perm.data(), n * 4, hipMemcpyHostToDevice, s);
    if (rc == GX_SUCCESS && e == hipSuccess)
        e = hipMemcpyAsync(p->rp_own.p, nrp.data(), (n + 1) * 8, hipMemcpyHostToDevice, s);
    if (rc == GX_SUCCESS && e == hipSuccess)
        e = hipMemcpyAsync(p->outdeg_own.p, nout.data(), n * 4, hipMemcpyHostToDevice, s);
    if (rc == GX_SUCCESS && e != hipSuccess) rc = fail(GX_DEVICE_ERROR, hipGetErrorString(e));
    clk.mark("row pointers + uploads");
    if (rc == GX_SUCCESS && P.nnz) {
        DBuf<uint64_t> keys, scratch;
        rc = keys.alloc(P.nnz);
        if (rc == GX_SUCCESS) rc = scratch.alloc(P.nnz);
        if (rc == GX_SUCCESS) {
            hipLaunchKernelGGL(k_permute_keys, dim3(grid_for((P.nnz + 15) / 16, 256, 1u << 30)), dim3(256), 0, s,
                               P.rp.p, P.ci.p, (int64_t)n, (int64_t)P.nnz, p->perm.p, keys.p);
            rc = check_launch("k_permute_keys");
        }
        if (rc == GX_SUCCESS) rc = sort_keys_to_csr(keys, scratch, P.nnz, (int64_t)n, p->rp_own.p, p->ci_own.p, s);
        if (rc == GX_SUCCESS) {
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = fail(GX_DEVICE_ERROR, hipGetErrorString(e));
        }
    }
    clk.mark("relabel (keys + sort)");
    if (rc == GX_SUCCESS) rc = pr_plan(p, nrp, p->rp_own.p, p->ci_own.p, p->outdeg_own.p, nout);
    clk.mark("pr_plan");
    if (rc == GX_SUCCESS) {
        e = hipStreamSynchronize(s);   // host vectors above die at return
        if (e != hipSuccess) rc = fail(GX_DEVICE_ERROR, hipGetErrorString(e));
    }
    if (rc != GX_SUCCESS) {
        delete p;
        return rc;
    }
    *out = p;
    return GX_SUCCESS;
}

// gx_pagerank's plan: the hub-first order on the device (a radix sort of n keys), the
// relabelled row pointers by a scan, then the column-sorted blocks read straight from the
// caller's pull matrix through order / perm (pr_plan_sorted's one radix sort): no relabelled
// CSR is materialised.  The host sees only the row pointers and out-degrees it plans blocks
// from.  Replaces LAGraph_Cached_OutDegree / LAGraph_Cached_AT's share of processing time
// (pr.cpp:58-60).
int gx::pr_single_plan(gx_graph *g, PrPart **out) {
    if (const char *e = std::getenv("GX_PR_KERNEL"))
        if (std::strcmp(e, "adaptive") == 0) return pr_single_plan_adaptive(g, out);
    const uint64_t n = g->n;
    gx_ctx *ctx = g->ctx;
    hipStream_t s = ctx->stream;
    DevCSR &P = g->directed ? g->AT : g->A;
    PlanClock clk("single", s);
    GX_TRY(ensure_outdeg(g));
    std::unique_ptr<PrPart> p(new PrPart());
    p->ctx = ctx;
    p->n_global = n;
    p->nranks = 1;
    p->rank = 0;
    p->chunk = round_up(n + 2, 32);   // + a zero padding slot (chunk - 2) and the dangling slot
    GX_TRY(p->perm.alloc(n));
    GX_TRY(p->order.alloc(n));
    GX_TRY(p->rp_own.alloc(n + 1));
    GX_TRY(p->outdeg_own.alloc(n));
    GX_TRY(p->xa.alloc(p->chunk));
    GX_TRY(p->xb.alloc(p->chunk));
    GX_HIP_TRY(hipMemsetAsync(p->xa.p, 0, p->chunk * sizeof(double), s));   // padding: the zero column
    GX_HIP_TRY(hipMemsetAsync(p->xb.p, 0, p->chunk * sizeof(double), s));
    GX_TRY(p->rank_out.alloc(n));
    GX_TRY(p->result.alloc(n));
    // An undirected graph pulls over A itself, so the hub-first rows' lengths are its degrees
    // sorted descending: the host gets them as runs of equal degrees (a few thousand pairs,
    // k_degree_runs over the device's sorted keys) instead of 12 n bytes of row pointers and
    // lengths (SYN-8_5: 6.6 ms of download).  A directed graph pulls over A' in out-degree order:
    // its row lengths come from the device.
    LengthRuns runs;
    bool have_runs = false;
    {
        DBuf<uint32_t> d0, d1;
        DBuf<int32_t> i0, i1;
        DBuf<int64_t> plen;
        GX_TRY(d0.alloc(n));
        GX_TRY(d1.alloc(n));
        GX_TRY(i0.alloc(n));
        GX_TRY(i1.alloc(n));
        GX_TRY(plen.alloc(n + 1));
        const unsigned grid = grid_for(n + 1, 256, 8192);
        hipLaunchKernelGGL(k_hub_keys, dim3(grid), dim3(256), 0, s, g->outdeg.p, (int64_t)n, d0.p, i0.p);
        GX_TRY(check_launch("k_hub_keys"));
        GX_TRY(sort_pairs_desc_u32_i32(d0.p, d1.p, i0.p, i1.p, n, s));
        hipLaunchKernelGGL(k_hub_apply, dim3(grid), dim3(256), 0, s, i1.p, (int64_t)n, g->outdeg.p, P.rp.p, p->order.p,
                           p->perm.p, p->outdeg_own.p, plen.p);
        GX_TRY(check_launch("k_hub_apply"));
        GX_TRY(scan_exclusive_i64(plen.p, p->rp_own.p, n + 1, s));
        if (!g->directed) {
            constexpr uint32_t kRunCap = 1u << 20;
            DBuf<uint64_t> rb;
            DBuf<uint32_t> rc;
            GX_TRY(rb.alloc(kRunCap));
            GX_TRY(rc.alloc(1));
            GX_HIP_TRY(hipMemsetAsync(rc.p, 0, 4, s));
            hipLaunchKernelGGL(k_degree_runs, dim3(grid), dim3(256), 0, s, d1.p, (int64_t)n, rb.p, rc.p, kRunCap);
            GX_TRY(check_launch("k_degree_runs"));
            uint32_t nr = 0;
            GX_HIP_TRY(hipMemcpyAsync(&nr, rc.p, 4, hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            if (nr <= kRunCap) {
                std::vector<uint64_t> h(nr);
                if (nr) GX_HIP_TRY(hipMemcpy(h.data(), rb.p, (size_t)nr * 8, hipMemcpyDeviceToHost));
                std::sort(h.begin(), h.end());   // by position
                runs.n = n;
                int64_t acc = 0;
                for (size_t k = 0; k < h.size(); k++) {
                    const int64_t pos = (int64_t)(h[k] >> 32), val = (int64_t)(uint32_t)h[k];
                    if (k) acc += (pos - runs.pos.back()) * runs.val.back();
                    runs.pos.push_back(pos);
                    runs.val.push_back(val);
                    runs.base.push_back(acc);
                }
                runs.total = (int64_t)P.nnz;
                have_runs = true;
            }
        }
        GX_HIP_TRY(hipStreamSynchronize(s));   // the temporaries are freed at the end of the block
    }
    clk.mark("hub order + row pointers (device)");
    // not value-initialised: zeroing 12 n bytes on one thread cost more than the transfer
    std::unique_ptr<int64_t[]> nrp;
    std::unique_ptr<int32_t[]> nout;
    if (!have_runs) {
        // download() stages through the context's pinned buffers and events, which the column
        // upload of gx_pagerank_csr (g->job) is using on its own thread: let it finish first
        if (g->job) GX_TRY(g->job->join());
        nrp.reset(new int64_t[n + 1]);
        nout.reset(new int32_t[n]);
        GX_TRY(download(ctx, nrp.get(), p->rp_own.p, n + 1, Xfer::Raw64));
        GX_TRY(download(ctx, nout.get(), p->outdeg_own.p, n, Xfer::Raw32));
    } else {
        p->rows_desc = true;   // row lengths non-increasing: the LONG rows are a prefix
    }
    clk.mark("row pointers to the host");
    p->src_rp = P.rp.p;
    p->src_ci = P.ci.p;
    p->src_order = p->order.p;
    p->src_perm = p->perm.p;
    // the columns still arriving (gx_pagerank_csr; undirected: the pull matrix is A itself): the
    // plan's key pass takes them chunk by chunk as they land (pr_plan_sorted)
    p->job = g->directed ? nullptr : g->job.get();
    if (have_runs)
        GX_TRY(pr_plan(p.get(), HostView<int64_t>(&runs, true), p->rp_own.p, nullptr, p->outdeg_own.p,
                       HostView<int32_t>(&runs, false)));
    else
        GX_TRY(pr_plan(p.get(), HostView<int64_t>(nrp.get(), n + 1), p->rp_own.p, nullptr, p->outdeg_own.p,
                       HostView<int32_t>(nout.get(), n)));
    GX_HIP_TRY(hipStreamSynchronize(s));   // host vectors above die at return
    p->job = nullptr;
    clk.mark("pr_plan");
    *out = p.release();
    return GX_SUCCESS;
}

// The block partition of gx_pagerank_multi (MultiBlocks), on the host from A: the hub-first
// order (hub_order, as the devices' radix sort orders it), the pull rows' lengths in it (A's
// out-degrees; A''s rows, the in-degrees, when directed), the greedy cut of pr_plan_sorted's
// huge-graph blocks (kPlanBlockRows rows, kPlanBlockNnz entries; GX_PR_MULTI_BLOCK_ROWS /
// _NNZ shrink them for tests), then largest block first to the device with the least entries +
// rows.  A device's positions stay in hub-first order, so its rows without out-edges come last
// (the live prefix).  The devices' own sorts must agree with each other, not with this order:
// a position names whichever vertex a device's order puts there, and every device's plan and
// column map read the same (device) order.
int gx::pr_multi_blocks(const gx_csr *A, int directed, int ndev, MultiBlocks *out) {
    const uint64_t n = A->n;
    // hub-first order, its degrees, all on the host's threads (the serial counting sort and its
    // random re-reads of the degrees were ~350 ms of SYN-8_5's partition)
    std::vector<int32_t> &order = out->order, &perm = out->perm;
    order.resize(n);
    perm.resize(n);
    std::vector<int64_t> hdeg(n);   // out-degree of the vertex at each hub-first position
    const bool tm = std::getenv("GX_PLAN_TIMES") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (!tm) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[plan multi_blocks] %-28s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    };
    host_hub_order_par(A->rowptr, n, order.data(), perm.data(), hdeg.data());
    mark("hub order (host)");
    std::vector<int64_t> indeg_h;
    if (directed) {   // the pull rows are A''s: their lengths are the in-degrees
        std::vector<int64_t> indeg(n, 0);
        for (uint64_t e = 0; e < A->rowptr[n]; e++) indeg[A->colidx[e]]++;
        indeg_h.resize(n);
        for (uint64_t h = 0; h < n; h++) indeg_h[h] = indeg[order[h]];
    }
    const std::vector<int64_t> &len = directed ? indeg_h : hdeg;
    auto env = [](const char *name, int64_t dflt, int64_t lo, int64_t hi) {
        const char *e = std::getenv(name);
        const int64_t v = e ? std::atoll(e) : dflt;
        return v >= lo && v <= hi ? v : dflt;
    };
    const int64_t R = env("GX_PR_MULTI_BLOCK_ROWS", kPlanBlockRows, 1, kPlanBlockRows);
    const int64_t B = env("GX_PR_MULTI_BLOCK_NNZ", kPlanBlockNnz, 1, (int64_t)1 << 30);
    std::vector<int64_t> starts;
    for (uint64_t r = 0; r < n;) {
        starts.push_back((int64_t)r);
        uint64_t e = r;
        int64_t ent = 0;
        // at least one row; then rows while both caps hold
        do ent += len[e++];
        while (e < n && (int64_t)(e - r) < R && ent + len[e] <= B);
        r = e;
    }
    starts.push_back((int64_t)n);
    mark("block cut");
    const size_t nb = starts.size() - 1;
    // work = entries + rows (the epilogue); live = rows with out-edges (the exchanged chunk)
    std::vector<int64_t> work(nb), blive(nb);
    for (size_t b = 0; b < nb; b++) {
        int64_t s = 0, l = 0;
        for (int64_t h = starts[b]; h < starts[b + 1]; h++) {
            s += len[h];
            l += hdeg[h] > 0;
        }
        work[b] = s + (starts[b + 1] - starts[b]);
        blive[b] = l;
    }
    // heaviest first: the upper half by work to the least loaded device (LPT), the lighter half
    // to the device with the fewest live rows among those it keeps within 1 % of the mean work
    // (pr_partition._deal_blocks): SYN-8_5 at 8 devices exchanges 0.672 n doubles, not 0.709 n
    std::vector<size_t> byb(nb);
    for (size_t b = 0; b < nb; b++) byb[b] = b;
    std::stable_sort(byb.begin(), byb.end(), [&](size_t x, size_t y) { return work[x] > work[y]; });
    double heavy = 0.0;
    if (nb) {
        std::vector<int64_t> w2(work);
        std::sort(w2.begin(), w2.end());
        heavy = nb % 2 ? (double)w2[nb / 2] : 0.5 * ((double)w2[nb / 2 - 1] + (double)w2[nb / 2]);
    }
    double total = 0.0;
    for (int64_t w : work) total += (double)w;
    const double target = total / ndev;
    std::vector<double> load(ndev, 0.0);
    std::vector<int64_t> lv(ndev, 0);
    std::vector<int> owner(nb, 0);
    for (size_t b : byb) {
        int d = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        if ((double)work[b] < heavy) {
            int best = -1;
            for (int k = 0; k < ndev; k++)
                if (load[k] + (double)work[b] <= target * 1.01 && (best < 0 || lv[k] < lv[best])) best = k;
            if (best >= 0) d = best;
        }
        owner[b] = d;
        load[d] += (double)work[b];
        lv[d] += blive[b];
    }
    mark("work + deal");
    out->pos.assign(ndev, {});
    std::vector<uint64_t> npos(ndev, 0), lvd(ndev, 0);
    for (size_t b = 0; b < nb; b++) {
        npos[owner[b]] += (uint64_t)(starts[b + 1] - starts[b]);
        lvd[owner[b]] += (uint64_t)blive[b];
    }
    for (int d = 0; d < ndev; d++) out->pos[d].reserve(npos[d]);
    for (size_t b = 0; b < nb; b++)
        for (int64_t h = starts[b]; h < starts[b + 1]; h++) out->pos[owner[b]].push_back((int32_t)h);
    uint64_t live = 0;
    for (int d = 0; d < ndev; d++) live = std::max(live, lvd[d]);
    out->chunk = (live + 2 + 31) / 32 * 32;
    if (out->chunk * (uint64_t)ndev >= (1ull << 31))
        return fail(GX_NOT_IMPLEMENTED, "gx_pagerank_multi: exchange too large");
    mark("positions");
    out->slot.assign(n, 0);
    for (int d = 0; d < ndev; d++)
        for (size_t j = 0; j < out->pos[d].size(); j++)
            out->slot[out->pos[d][j]] = (int32_t)((uint64_t)d * out->chunk + j);
    mark("slots");
    return GX_SUCCESS;
}

int gx::pr_multi_interleave(const gx_csr *A, int ndev, MultiBlocks *out) {
    const uint64_t n = A->n;
    const uint64_t nlive = host_count_live(A->rowptr, n);
    out->order.resize(n);
    out->perm.resize(n);
    std::vector<int64_t> hdeg(n);
    host_hub_order_par(A->rowptr, n, out->order.data(), out->perm.data(), hdeg.data());
    out->chunk = ((nlive + ndev - 1) / ndev + 2 + 31) / 32 * 32;
    if (out->chunk * (uint64_t)ndev >= (1ull << 31)) return fail(GX_NOT_IMPLEMENTED, "gx_pagerank_multi: exchange too large");
    out->pos.assign(ndev, {});
    out->slot.assign(n, 0);
    for (uint64_t h = 0; h < n; h++) {
        const int d = (int)(h % (uint64_t)ndev);
        out->slot[h] = (int32_t)((uint64_t)d * out->chunk + out->pos[d].size());
        out->pos[d].push_back((int32_t)h);
    }
    return GX_SUCCESS;
}

// gx_pagerank_multi's plan of device `d` of `ndev`, all on that device from its copy of the
// graph: the hub-first order (the same radix sort on every device, so every device derives
// the same partition), the device's rows (hub-first positions d, d + ndev, ...) as the sorted
// plan's source rows, and the column map into the exchange layout as its column renaming.
// Replaces the host transpose / row picking / column remapping of round 3.
int gx::pr_multi_plan(gx_graph *g, int ndev, int d, uint64_t chunk, double damping, const MultiBlocks *mb,
                      PrPart **out) {
    const uint64_t n = g->n;
    gx_ctx *ctx = g->ctx;
    hipStream_t s = ctx->stream;
    DevCSR &P = g->directed ? g->AT : g->A;
    PlanClock clk("multi", s);
    GX_TRY(ensure_outdeg(g));
    const uint64_t rows = mb ? mb->pos[d].size() : n > (uint64_t)d ? (n - (uint64_t)d + ndev - 1) / ndev : 0;
    std::unique_ptr<PrPart> p(new PrPart());
    p->ctx = ctx;
    p->n_global = n;
    p->nranks = ndev;
    p->rank = d;
    p->chunk = chunk;
    p->damping = damping;
    p->force_huge = mb != nullptr;   // the whole graph's block cut (pr_plan_sorted `piece`)
    GX_TRY(p->order.alloc(std::max<uint64_t>(rows, 1)));
    GX_TRY(p->perm.alloc(n));   // the column map
    GX_TRY(p->rp_own.alloc(rows + 1));
    GX_TRY(p->outdeg_own.alloc(std::max<uint64_t>(rows, 1)));
    {
        DBuf<uint32_t> d0, d1;
        DBuf<int32_t> i0, i1, ord, nout;
        DBuf<int64_t> plen, myplen;
        GX_TRY(d0.alloc(n));
        GX_TRY(d1.alloc(n));
        GX_TRY(i0.alloc(n));
        GX_TRY(i1.alloc(n));
        GX_TRY(ord.alloc(n));
        GX_TRY(nout.alloc(n));
        GX_TRY(plen.alloc(n + 1));
        GX_TRY(myplen.alloc(rows + 1));
        const unsigned grid = grid_for(n + 1, 256, 8192);
        hipLaunchKernelGGL(k_hub_keys, dim3(grid), dim3(256), 0, s, g->outdeg.p, (int64_t)n, d0.p, i0.p);
        GX_TRY(check_launch("k_hub_keys"));
        GX_TRY(sort_pairs_desc_u32_i32(d0.p, d1.p, i0.p, i1.p, n, s));
        // i0 is free after the sort: it takes the full perm
        hipLaunchKernelGGL(k_hub_apply, dim3(grid), dim3(256), 0, s, i1.p, (int64_t)n, g->outdeg.p, P.rp.p, ord.p,
                           i0.p, nout.p, plen.p);
        GX_TRY(check_launch("k_hub_apply"));
        if (mb) {
            DBuf<int32_t> pos, slot;
            GX_TRY(pos.alloc(std::max<uint64_t>(rows, 1)));
            GX_TRY(slot.alloc(n));
            if (rows) GX_HIP_TRY(hipMemcpy(pos.p, mb->pos[d].data(), rows * 4, hipMemcpyHostToDevice));
            GX_HIP_TRY(hipMemcpy(slot.p, mb->slot.data(), n * 4, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(k_block_pick, dim3(grid_for(rows + 1, 256, 8192)), dim3(256), 0, s, ord.p, nout.p, plen.p,
                               pos.p, (int64_t)rows, p->order.p, p->outdeg_own.p, myplen.p);
            GX_TRY(check_launch("k_block_pick"));
            hipLaunchKernelGGL(k_block_colmap, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, i0.p, (int64_t)n, slot.p,
                               p->perm.p);
            GX_TRY(check_launch("k_block_colmap"));
            GX_TRY(scan_exclusive_i64(myplen.p, p->rp_own.p, rows + 1, s));
            GX_HIP_TRY(hipStreamSynchronize(s));   // pos / slot die here
        } else {
            hipLaunchKernelGGL(k_multi_pick, dim3(grid_for(rows + 1, 256, 8192)), dim3(256), 0, s, ord.p, nout.p, plen.p,
                               ndev, d, (int64_t)rows, p->order.p, p->outdeg_own.p, myplen.p);
            GX_TRY(check_launch("k_multi_pick"));
            hipLaunchKernelGGL(k_multi_colmap, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, i0.p, (int64_t)n, ndev,
                               (int64_t)chunk, p->perm.p);
            GX_TRY(check_launch("k_multi_colmap"));
        }
        if (!mb) GX_TRY(scan_exclusive_i64(myplen.p, p->rp_own.p, rows + 1, s));
        GX_HIP_TRY(hipStreamSynchronize(s));   // the temporaries are freed at the end of the block
    }
    clk.mark("hub order + partition rows (device)");
    std::unique_ptr<int64_t[]> nrp(new int64_t[rows + 1]);
    std::unique_ptr<int32_t[]> nout(new int32_t[std::max<uint64_t>(rows, 1)]);
    GX_TRY(download(ctx, nrp.get(), p->rp_own.p, rows + 1, Xfer::Raw64));
    if (rows) GX_TRY(download(ctx, nout.get(), p->outdeg_own.p, rows, Xfer::Raw32));
    // the live prefix: rows with out-edges (hub-first, so a prefix of the device's rows)
    uint64_t lo = 0, hi = rows;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (nout[mid] > 0) lo = mid + 1;
        else hi = mid;
    }
    p->live = lo;
    clk.mark("row pointers to the host");
    p->src_rp = P.rp.p;
    p->src_ci = P.ci.p;
    p->src_order = p->order.p;
    p->src_perm = p->perm.p;
    GX_TRY(pr_plan(p.get(), HostView<int64_t>(nrp.get(), rows + 1), p->rp_own.p, nullptr, p->outdeg_own.p,
                   HostView<int32_t>(nout.get(), rows)));
    GX_HIP_TRY(hipStreamSynchronize(s));   // host vectors above die at return
    clk.mark("pr_plan");
    *out = p.release();
    return GX_SUCCESS;
}

extern "C" int gx_pagerank(gx_graph *g, double damping, int iters, double *rank) {
    if (!g || !rank) return fail(GX_NULL_POINTER, "gx_pagerank: null argument");
    if (iters < 0) return fail(GX_INVALID_VALUE, "gx_pagerank: negative iteration count");
    const uint64_t n = g->n;
    if (n == 0) return GX_SUCCESS;
    const auto t_entry = std::chrono::steady_clock::now();
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    GX_TRY(device_begin(ctx));
    // columns still arriving (gx_pagerank_csr): only the sorted single plan consumes them as they
    // land; every other path waits for all of them
    const char *ke = std::getenv("GX_PR_KERNEL");
    if (g->job && (g->directed || g->pr || (ke && std::strcmp(ke, "adaptive") == 0))) {
        GX_TRY(g->job->join());
        g->job.reset();
    }
    if (g->directed) GX_TRY(ensure_transpose(g));
    if (!g->pr) {
        // the plan's temporaries are freed once the upload is over (g_deferred_frees)
        std::vector<void *> deferred;
        // the upload thread narrows with half the host threads: the plan's host loops take the
        // other half (all of them on top of the upload's ran some fused calls 115 ms, not 88)
        const int saved_threads = host_threads();
        if (g->job) {
            g_deferred_frees = &deferred;
            host_set_threads(std::max(1, saved_threads - std::max(1, saved_threads / 2)));
        }
        const int rc = pr_single_plan(g, &g->pr);
        g_deferred_frees = nullptr;
        host_set_threads(saved_threads);
        if (g->job) {   // the plan has taken every chunk (or stopped early): the upload is over
            const int jrc = g->job->join();
            g->job.reset();
            for (void *q : deferred) (void)hipFree(q);
            if (rc == GX_SUCCESS && jrc != GX_SUCCESS) return jrc;
        }
        if (rc != GX_SUCCESS) return rc;
    }
    const auto t_plan = std::chrono::steady_clock::now();
    PrPart *p = g->pr;
    p->damping = damping;
    double *cur = p->xa.p, *nxt = p->xb.p;
    GX_TRY(pr_init(p, cur, s));
    for (int it = 0; it < iters; it++) {
        GX_TRY(pr_step(p, cur, nxt, it == iters - 1 ? p->rank_out.p : nullptr, s));
        std::swap(cur, nxt);
    }
    using clk = std::chrono::steady_clock;
    static const bool times = std::getenv("GX_PLAN_TIMES") && std::atoi(std::getenv("GX_PLAN_TIMES")) != 0;
    const auto t0 = clk::now();
    auto ms = [&](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    clk::time_point t1 = t0;
    if (iters > 0) {
        hipLaunchKernelGGL(k_gather_perm, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, p->rank_out.p,
                           p->perm.p, (int64_t)n, p->result.p);
        GX_TRY(check_launch("k_gather_perm"));
        host_prefault(rank, n * sizeof(double));
        t1 = clk::now();
    }
    GX_TRY(device_end(ctx));
    const auto t2 = clk::now();
    if (iters == 0) {
        for (uint64_t v = 0; v < n; v++) rank[v] = 1.0 / (double)n;
        return GX_SUCCESS;
    }
    GX_TRY(download(ctx, rank, p->result.p, n, Xfer::Raw64));
    if (times)
        std::fprintf(stderr, "[pagerank] plan %.2f ms, launches %.2f ms, prefault %.2f ms, device wait %.2f ms, "
                     "result copy %.2f ms (device %.2f ms)\n", ms(t_entry, t_plan), ms(t_plan, t0), ms(t0, t1),
                     ms(t1, t2), ms(t2, clk::now()), ctx->last_device_ms);
    return GX_SUCCESS;
}

// The executable's PageRank (bin/exe/pr: pr.cpp:77-79 brackets LAGraph_New .. LAGr_PageRankGX
// between its markers): upload + plan + iterations in one call.  For an undirected graph the
// columns are uploaded by a host thread chunk by chunk while the plan builds the hub-first order
// from the row pointers and then takes each chunk as it lands (graph_create_async,
// pr_plan_sorted's source-side key pass), and the weights, which PageRank never reads, are not
// uploaded at all.  Directed graphs (the plan needs A' whole) and GX_PR_FUSED=0 take
// gx_graph_create + gx_pagerank.
extern "C" int gx_pagerank_csr(gx_ctx *ctx, const gx_csr *A, int directed, double damping, int iters, double *rank,
                               gx_graph **keep) {
    if (!ctx || !A || !rank) return fail(GX_NULL_POINTER, "gx_pagerank_csr: null argument");
    if (iters < 0) return fail(GX_INVALID_VALUE, "gx_pagerank_csr: negative iteration count");
    if (keep) *keep = nullptr;
    const char *fe = std::getenv("GX_PR_FUSED");
    const bool fused = !directed && !(fe && std::atoi(fe) == 0);
    gx_graph *g = nullptr;
    PlanClock clk("pagerank_csr", ctx->stream);
    if (fused) GX_TRY(graph_create_async(ctx, A, directed, &g));
    else GX_TRY(gx_graph_create(ctx, A, directed, &g));
    clk.mark("graph (columns on their way)");
    const int rc = gx_pagerank(g, damping, iters, rank);
    clk.mark("gx_pagerank");
    if (rc != GX_SUCCESS) {
        const std::string msg = gx_last_error();
        (void)gx_graph_free(g);   // joins an upload the call left running (an early error)
        return fail(rc, msg);
    }
    // the graph and its plan (gigabytes of device memory) are the caller's to free, outside the
    // processing time if it likes (bin/exe/pr frees after its end marker, as before)
    if (keep) *keep = g;
    else return gx_graph_free(g);
    return GX_SUCCESS;
}

// ---------------------------------------------------------------- row partition API

extern "C" int gx_pr_part_create(gx_ctx *ctx, uint64_t n_global, int nranks, int rank,
                                 const uint64_t *row_ranges, const uint64_t *rowptr_local,
                                 const uint64_t *colidx_local, const uint64_t *outdeg_local,
                                 double damping, gx_pr_part **out) {
    return gx_pr_part_create_live(ctx, n_global, nranks, rank, row_ranges, nullptr, rowptr_local, colidx_local,
                                  outdeg_local, damping, out);
}

extern "C" int gx_pr_part_create_live(gx_ctx *ctx, uint64_t n_global, int nranks, int rank,
                                      const uint64_t *row_ranges, const uint64_t *live_rows,
                                      const uint64_t *rowptr_local, const uint64_t *colidx_local,
                                      const uint64_t *outdeg_local, double damping, gx_pr_part **out) {
    if (!ctx || !row_ranges || !rowptr_local || !outdeg_local || !out)
        return fail(GX_NULL_POINTER, "gx_pr_part_create: null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(GX_INVALID_VALUE, "bad rank/nranks");
    if (row_ranges[0] != 0 || row_ranges[nranks] != n_global)
        return fail(GX_INVALID_VALUE, "row_ranges must cover [0, n)");
    GX_HIP_TRY(hipSetDevice(ctx->device));
    // the exchanged prefix of every rank: its live rows (all of them without live_rows)
    std::vector<uint64_t> live(nranks);
    uint64_t maxlive = 0;
    for (int k = 0; k < nranks; k++) {
        if (row_ranges[k + 1] < row_ranges[k]) return fail(GX_INVALID_VALUE, "row_ranges not monotone");
        live[k] = row_ranges[k + 1] - row_ranges[k];
        if (live_rows) {
            if (live_rows[k] > live[k]) return fail(GX_INVALID_VALUE, "live_rows beyond the rank's rows");
            live[k] = live_rows[k];
        }
        maxlive = std::max(maxlive, live[k]);
    }
    const uint64_t chunk = round_up(maxlive + 2, 32);   // + the zero padding slot and the dangling slot
    if (chunk * (uint64_t)nranks >= (1ull << 31)) return fail(GX_NOT_IMPLEMENTED, "partition too large");
    const uint64_t rows = row_ranges[rank + 1] - row_ranges[rank];
    const uint64_t nnz = rowptr_local[rows];
    if (nnz && !colidx_local) return fail(GX_NULL_POINTER, "null colidx");
    for (uint64_t i = live[rank]; i < rows; i++)
        if (outdeg_local[i] != 0) return fail(GX_INVALID_VALUE, "a row past live_rows has out-edges");
    std::vector<int64_t> h_rp(rows + 1);
    for (uint64_t i = 0; i <= rows; i++) h_rp[i] = (int64_t)rowptr_local[i];
    std::vector<int32_t> ci(nnz);
    const int bad = nnz ? host_chunk_columns(colidx_local, nnz, row_ranges, nranks, live.data(), chunk, n_global, ci.data())
                        : 0;
    if (bad & 1) return fail(GX_INVALID_INDEX, "column out of range");
    if (bad & 2) return fail(GX_INVALID_VALUE, "a column is past its owner's live rows (a vertex without out-edges)");
    std::vector<int32_t> h_outdeg(rows);
    for (uint64_t i = 0; i < rows; i++) h_outdeg[i] = (int32_t)outdeg_local[i];
    PrPart *p = nullptr;
    GX_TRY(pr_part_build(ctx, n_global, nranks, rank, chunk, live[rank], h_rp, ci, h_outdeg, damping, &p));
    *out = reinterpret_cast<gx_pr_part *>(p);
    return GX_SUCCESS;
}

int gx::pr_part_build(gx_ctx *ctx, uint64_t n_global, int nranks, int rank, uint64_t chunk, uint64_t live,
                      const std::vector<int64_t> &h_rp, const std::vector<int32_t> &ci,
                      const std::vector<int32_t> &h_outdeg, double damping, PrPart **out, bool force_huge) {
    const uint64_t rows = h_rp.size() - 1, nnz = (uint64_t)h_rp[rows];
    auto *p = new PrPart();
    p->ctx = ctx;
    p->n_global = n_global;
    p->nranks = nranks;
    p->rank = rank;
    p->chunk = chunk;
    p->live = live;
    p->damping = damping;
    p->force_huge = force_huge;
    int rc = p->rp_own.alloc(rows + 1);
    if (rc == GX_SUCCESS) rc = p->ci_own.alloc(nnz, 16);
    if (rc == GX_SUCCESS) rc = p->outdeg_own.alloc(std::max<uint64_t>(rows, 1));
    hipError_t e = hipSuccess;
    if (rc == GX_SUCCESS) e = hipMemcpy(p->rp_own.p, h_rp.data(), (rows + 1) * 8, hipMemcpyHostToDevice);
    if (rc == GX_SUCCESS && e == hipSuccess && nnz)
        e = hipMemcpy(p->ci_own.p, ci.data(), nnz * 4, hipMemcpyHostToDevice);
    if (rc == GX_SUCCESS && e == hipSuccess && rows)
        e = hipMemcpy(p->outdeg_own.p, h_outdeg.data(), rows * 4, hipMemcpyHostToDevice);
    if (rc == GX_SUCCESS && e != hipSuccess)
        rc = fail(GX_DEVICE_ERROR, std::string("gx_pr_part_create upload: ") + hipGetErrorString(e));
    p->src_rp = p->rp_own.p;
    p->src_ci = p->ci_own.p;
    if (rc == GX_SUCCESS) rc = pr_plan(p, h_rp, p->rp_own.p, p->ci_own.p, p->outdeg_own.p, h_outdeg);
    if (rc != GX_SUCCESS) {
        delete p;
        return rc;
    }
    *out = p;
    return GX_SUCCESS;
}

int gx::pr_part_build_rows(gx_ctx *ctx, const gx_csr *A, int nranks, int rank, uint64_t chunk,
                           const std::vector<int32_t> &rows, const int32_t *colmap, double damping, bool force_huge,
                           PrPart **out) {
    const uint64_t nr = rows.size();
    std::vector<int64_t> h_rp(nr + 1);
    std::vector<int32_t> h_outdeg(nr);
    h_rp[0] = 0;
    uint64_t live = 0;
    for (uint64_t j = 0; j < nr; j++) {
        const int64_t len = (int64_t)(A->rowptr[rows[j] + 1] - A->rowptr[rows[j]]);
        h_rp[j + 1] = h_rp[j] + len;
        h_outdeg[j] = (int32_t)len;   // undirected: the pull row is the vertex's out-edge list
        live += len > 0;
    }
    const uint64_t nnz = (uint64_t)h_rp[nr];
    std::unique_ptr<PrPart> p(new PrPart());
    p->ctx = ctx;
    p->n_global = A->n;
    p->nranks = nranks;
    p->rank = rank;
    p->chunk = chunk;
    p->live = live;
    p->damping = damping;
    p->force_huge = force_huge;
    GX_TRY(p->rp_own.alloc(nr + 1));
    GX_TRY(p->ci_own.alloc(nnz, 16));
    GX_TRY(p->outdeg_own.alloc(std::max<uint64_t>(nr, 1)));
    bool bad = false;
    GX_TRY(upload_staged(ctx, p->rp_own.p, nr + 1, 8,
                         [&](uint64_t off, uint64_t cnt, void *buf) {
                             host_copy(buf, h_rp.data() + off, cnt * 8);
                             return true;
                         }, &bad));
    if (nr)
        GX_TRY(upload_staged(ctx, p->outdeg_own.p, nr, 4,
                             [&](uint64_t off, uint64_t cnt, void *buf) {
                                 host_copy(buf, h_outdeg.data() + off, cnt * 4);
                                 return true;
                             }, &bad));
    GX_TRY(upload_staged(ctx, p->ci_own.p, nnz, 4,
                         [&](uint64_t off, uint64_t cnt, void *buf) {
                             return host_pick_span(A->rowptr, A->colidx, rows.data(), h_rp.data(), nr, off, off + cnt,
                                                   A->n, static_cast<int32_t *>(buf));
                         }, &bad));
    if (bad) return fail(GX_INVALID_INDEX, "gx_pagerank_multi: column out of range");
    p->src_rp = p->rp_own.p;
    p->src_ci = p->ci_own.p;
    p->src_perm = colmap;
    GX_TRY(pr_plan(p.get(), HostView<int64_t>(h_rp), p->rp_own.p, p->ci_own.p, p->outdeg_own.p,
                   HostView<int32_t>(h_outdeg)));
    GX_HIP_TRY(hipStreamSynchronize(ctx->stream));
    *out = p.release();
    return GX_SUCCESS;
}

extern "C" int gx_pr_part_chunk(gx_pr_part *part, uint64_t *chunk) {
    if (!part || !chunk) return fail(GX_NULL_POINTER, "null argument");
    *chunk = reinterpret_cast<PrPart *>(part)->chunk;
    return GX_SUCCESS;
}

extern "C" int gx_pr_part_init(gx_pr_part *part, double *x_local, void *stream) {
    if (!part || !x_local) return fail(GX_NULL_POINTER, "null argument");
    PrPart *p = reinterpret_cast<PrPart *>(part);
    GX_HIP_TRY(hipSetDevice(p->ctx->device));
    return pr_init(p, x_local, stream ? (hipStream_t)stream : p->ctx->stream);
}

extern "C" int gx_pr_part_step(gx_pr_part *part, const double *x_full, double *x_local,
                               double *rank_out, void *stream) {
    if (!part || !x_full || !x_local) return fail(GX_NULL_POINTER, "null argument");
    PrPart *p = reinterpret_cast<PrPart *>(part);
    GX_HIP_TRY(hipSetDevice(p->ctx->device));
    return pr_step(p, x_full, x_local, rank_out, stream ? (hipStream_t)stream : p->ctx->stream);
}

extern "C" int gx_pr_part_free(gx_pr_part *part) {
    if (!part) return GX_SUCCESS;
    PrPart *p = reinterpret_cast<PrPart *>(part);
    (void)hipSetDevice(p->ctx->device);
    (void)hipDeviceSynchronize();
    delete p;
    return GX_SUCCESS;
}

GX_MODULE_WARMER(pr)
