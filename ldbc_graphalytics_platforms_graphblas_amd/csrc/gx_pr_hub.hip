// gx_pr_hub.hip -- hub-cached pull SpMV for PageRank (default k_pr_pull variant).
//
// Profile of the CSR-Adaptive kernel (profiles/README.md, round 1): with the hub-first
// vertex order the gathers hit L2 94% of the time, but every 8-byte gather is still one
// L1 access and one L2 request, and 64% of wave cycles are issue stalls on the vector
// memory pipe -- the kernel is bound by gather REQUESTS, not HBM bytes.  This kernel takes
// requests off that pipe:
//   * one 1024-thread workgroup per CU copies the hottest prefix of x (hub-first order, up
//     to 158 KiB = the most gathered ~20K vertices) into LDS once per launch; gathers of
//     those columns are ds_read_b64, the rest go to L2 / MALL;
//   * waves work independently on equal-size items (statically interleaved over the
//     grid), L lanes per row where all rows of an item have nearly the same length;
//     column indices stream with non-temporal loads;
//   * the dangling-score sum of the rank is reduced in the same launch (per-lane sums ->
//     per-workgroup sum -> last-arriving workgroup adds the 256 partials in order), so an
//     iteration is one launch.
// Results are deterministic: the static item assignment fixes every summation order.
#include <algorithm>

#include "gx_pr.h"

namespace gx {
namespace {

constexpr int kHubMax = 20224;   // doubles of x cached in LDS (158 KiB)

struct HubArgs {
    const WaveItem *items;
    uint32_t nitems;
    const int64_t *rp;
    const int32_t *ci;
    const int32_t *outdeg;
    const double *x_in;
    double *x_out;
    double *rank_out;
    int64_t chunk;
    int nranks;
    int64_t hub_entries;
    double teleport0, damping_over_n, damping;
    const int32_t *long_first;
    const int32_t *long_nseg;
    double *long_part;
    uint32_t *long_ticket;
    double *gpart;
    uint32_t *gticket;
};

// sum of x over entries [b, e) taken by this lane (stride L, 4 loads in flight).
// Index loads are clamped to the row (always valid, no branches); the LDS read is issued
// for every lane and the global read only for non-hub columns -- written so that the two
// cannot be folded into one flat load (which would send the hub reads down the vector
// memory pipe again).
__device__ __forceinline__ double row_sum(const HubArgs &a, const double *hub, int64_t b, int64_t e,
                                          int L, int gl) {
    double s = 0.0;
    const int32_t H = (int32_t)a.hub_entries;
    for (int64_t k0 = b + gl; k0 < e; k0 += 4 * (int64_t)L) {
        int32_t c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t k = min(k0 + (int64_t)u * L, e - 1);
            c[u] = __builtin_nontemporal_load(a.ci + k);
        }
        double hv[4], gv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) hv[u] = hub[c[u] < H ? c[u] : 0];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            gv[u] = 0.0;
            if (c[u] >= H) gv[u] = a.x_in[c[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (k0 + (int64_t)u * L < e) s += c[u] < H ? hv[u] : gv[u];
    }
    return s;
}

__device__ __forceinline__ double finish_row(const HubArgs &a, int32_t row, double s, double teleport,
                                             int32_t deg) {
    const double r = teleport + s;
    if (a.rank_out) a.rank_out[row] = r;
    a.x_out[row] = deg > 0 ? r / ((double)deg / a.damping) : r;
    return deg == 0 ? r : 0.0;   // contribution to the dangling sum
}

__global__ __launch_bounds__(kHubBlock) void k_pr_pull_hub(HubArgs a) {
    __shared__ __attribute__((aligned(16))) double hub[kHubMax];
    __shared__ double wsum[kHubBlock / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    {
        // all loads first, then all LDS stores (one round trip, not one per 16 KiB)
        constexpr int kFill = (kHubMax / 2 + kHubBlock - 1) / kHubBlock;
        const double2 *src = reinterpret_cast<const double2 *>(a.x_in);
        double2 *dst = reinterpret_cast<double2 *>(hub);
        const int npair = (int)(a.hub_entries / 2);
        double2 t[kFill];
#pragma unroll
        for (int j = 0; j < kFill; j++) {
            const int i = tid + j * kHubBlock;
            t[j] = i < npair ? src[i] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int j = 0; j < kFill; j++) {
            const int i = tid + j * kHubBlock;
            if (i < npair) dst[i] = t[j];
        }
        if ((a.hub_entries & 1) && tid == 0) hub[a.hub_entries - 1] = a.x_in[a.hub_entries - 1];
    }
    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    __syncthreads();

    double dang = 0.0;
    const uint32_t nw = gridDim.x * (kHubBlock / kWave);
    for (uint32_t i = (uint32_t)wv * gridDim.x + blockIdx.x; i < a.nitems; i += nw) {
        const WaveItem w = a.items[i];
        if (w.split >= 0) {
            // one segment of a long row: all 64 lanes
            double s = wave_sum(row_sum(a, hub, w.nz_begin, w.nz_end, kWave, lane));
            if (lane == 0) {
                const int32_t nseg = a.long_nseg[w.split];
                const int32_t row = w.row_begin;
                if (nseg == 1) {
                    dang += finish_row(a, row, s, teleport, a.outdeg[row]);
                } else {
                    const int32_t first = a.long_first[w.split];
                    __hip_atomic_store(&a.long_part[first + w.seg], s, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const uint32_t t = __hip_atomic_fetch_add(&a.long_ticket[w.split], 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
                    if (t == (uint32_t)(nseg - 1)) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        double all = 0.0;
                        for (int j = 0; j < nseg; j++)
                            all += __hip_atomic_load(&a.long_part[first + j], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&a.long_ticket[w.split], 0u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        dang += finish_row(a, row, all, teleport, a.outdeg[row]);
                    }
                }
            }
            continue;
        }
        // rows of similar length: L lanes per row, G rows per pass
        const int L = w.lanes;
        const int G = kWave / L;
        const int grp = lane / L, gl = lane & (L - 1);
        for (int32_t r0 = w.row_begin; r0 < w.row_end; r0 += G) {
            const int32_t row = r0 + grp;
            const bool valid = row < w.row_end;
            const int32_t deg = (valid && gl == 0) ? a.outdeg[row] : 0;
            double s = 0.0;
            if (valid) s = row_sum(a, hub, a.rp[row], a.rp[row + 1], L, gl);
            for (int off = L >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
            if (valid && gl == 0) dang += finish_row(a, row, s, teleport, deg);
        }
    }

    // dangling sum of the rank: lanes -> wave -> workgroup -> last-arriving workgroup
    dang = wave_sum(dang);
    if (lane == 0) wsum[wv] = dang;
    __syncthreads();
    if (tid != 0) return;
    double bs = 0.0;
#pragma unroll
    for (int w = 0; w < kHubBlock / kWave; w++) bs += wsum[w];
    __hip_atomic_store(&a.gpart[blockIdx.x], bs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(a.gticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t != gridDim.x - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    double all = 0.0;
    for (uint32_t j = 0; j < gridDim.x; j++)
        all += __hip_atomic_load(&a.gpart[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.gticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.x_out[a.chunk - 1] = all;
}

int pow2_floor(int64_t v) {
    int p = 1;
    while ((int64_t)p * 2 <= v) p *= 2;
    return p;
}

}  // namespace

int pr_plan_hub(PrPart *p, const std::vector<int64_t> &h_rp) {
    const int64_t rows = (int64_t)h_rp.size() - 1;
    std::vector<WaveItem> longi, streami;
    std::vector<int32_t> lfirst, lnseg;
    std::vector<std::pair<int64_t, int32_t>> longrows;
    int32_t nsegs = 0;
    int64_t r = 0;
    while (r < rows) {
        const int64_t len = h_rp[r + 1] - h_rp[r];
        if (len > kHubSegNnz) {
            longrows.push_back({len, (int32_t)r});
            r++;
            continue;
        }
        const int64_t start = r;
        int64_t nz = 0;
        while (r < rows && r - start < kItemRows) {
            const int64_t l = h_rp[r + 1] - h_rp[r];
            if (l > kHubSegNnz) break;
            if (r > start && nz + l > kItemNnz) break;
            nz += l;
            r++;
        }
        const int64_t nrows = r - start;
        // lanes per row: about half the mean row length, so a row takes ~2+ passes of its
        // group; rows of one item have nearly the same length in hub-first order
        int L = pow2_floor(std::max<int64_t>(1, nz / std::max<int64_t>(1, nrows) / 2));
        L = std::min(L, kWave);
        streami.push_back({h_rp[start], h_rp[r], (int32_t)start, (int32_t)r, -1, 0, L, 0});
    }
    std::stable_sort(longrows.begin(), longrows.end(),
                     [](const auto &x, const auto &y) { return x.first > y.first; });
    for (const auto &lr : longrows) {
        const int32_t row = lr.second;
        const int32_t nseg = (int32_t)((lr.first + kHubSegNnz - 1) / kHubSegNnz);
        const int32_t sp = (int32_t)lfirst.size();
        lfirst.push_back(nsegs);
        lnseg.push_back(nseg);
        for (int32_t s = 0; s < nseg; s++) {
            const int64_t zb = h_rp[row] + (int64_t)s * kHubSegNnz;
            const int64_t ze = std::min<int64_t>(zb + kHubSegNnz, h_rp[row + 1]);
            longi.push_back({zb, ze, row, row + 1, sp, s, kWave, 0});
        }
        nsegs += nseg;
    }
    std::vector<WaveItem> all;
    all.reserve(longi.size() + streami.size());
    all.insert(all.end(), longi.begin(), longi.end());
    all.insert(all.end(), streami.begin(), streami.end());
    p->nitems = (uint32_t)all.size();
    GX_TRY(p->items.alloc(std::max<size_t>(all.size(), 1)));
    GX_TRY(p->hlong_first.alloc(std::max<size_t>(lfirst.size(), 1)));
    GX_TRY(p->hlong_nseg.alloc(std::max<size_t>(lnseg.size(), 1)));
    GX_TRY(p->hlong_part.alloc(std::max<size_t>(nsegs, 1)));
    GX_TRY(p->hlong_ticket.alloc(std::max<size_t>(lfirst.size(), 1)));
    if (!all.empty())
        GX_HIP_TRY(hipMemcpy(p->items.p, all.data(), all.size() * sizeof(WaveItem), hipMemcpyHostToDevice));
    if (!lfirst.empty()) {
        GX_HIP_TRY(hipMemcpy(p->hlong_first.p, lfirst.data(), lfirst.size() * 4, hipMemcpyHostToDevice));
        GX_HIP_TRY(hipMemcpy(p->hlong_nseg.p, lnseg.data(), lnseg.size() * 4, hipMemcpyHostToDevice));
    }
    GX_HIP_TRY(hipMemset(p->hlong_ticket.p, 0, p->hlong_ticket.n * 4));
    p->hub_grid = (uint32_t)std::max(1, p->ctx->num_cus);
    p->hub_entries = std::min<int64_t>(kHubMax, (int64_t)(p->chunk * p->nranks));
    if (const char *e = std::getenv("GX_PR_HUB_ENTRIES"))
        p->hub_entries = std::max<int64_t>(0, std::min<int64_t>(p->hub_entries, std::atoll(e)));
    GX_TRY(p->gpart.alloc(p->hub_grid));
    GX_TRY(p->gticket.alloc(1));
    GX_HIP_TRY(hipMemset(p->gticket.p, 0, 4));
    return GX_SUCCESS;
}

int pr_step_hub(PrPart *p, const double *x_full, double *x_local, double *rank_out, hipStream_t s) {
    const double dn = (double)p->n_global;
    HubArgs a;
    a.items = p->items.p;
    a.nitems = p->nitems;
    a.rp = p->rp;
    a.ci = p->ci;
    a.outdeg = p->outdeg;
    a.x_in = x_full;
    a.x_out = x_local;
    a.rank_out = rank_out;
    a.chunk = (int64_t)p->chunk;
    a.nranks = p->nranks;
    a.hub_entries = p->hub_entries;
    a.teleport0 = (1.0 - p->damping) / dn;
    a.damping_over_n = p->damping / dn;
    a.damping = p->damping;
    a.long_first = p->hlong_first.p;
    a.long_nseg = p->hlong_nseg.p;
    a.long_part = p->hlong_part.p;
    a.long_ticket = p->hlong_ticket.p;
    a.gpart = p->gpart.p;
    a.gticket = p->gticket.p;
    {
        KTimer kt(p->ctx, "pr_pull", s);
        hipLaunchKernelGGL(k_pr_pull_hub, dim3(p->hub_grid), dim3(kHubBlock), 0, s, a);
    }
    return check_launch("k_pr_pull_hub");
}

}  // namespace gx
