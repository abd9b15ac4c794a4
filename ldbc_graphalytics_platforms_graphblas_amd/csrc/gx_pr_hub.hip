// gx_pr_hub.hip -- hub-cached pull SpMV for PageRank (default k_pr_pull variant).
//
// Profile of the CSR-Adaptive kernel (profiles/README.md): with the hub-first vertex
// order the gathers hit L2 94% of the time, but every 8-byte gather is one L1 access and
// one L2 request, and 64% of wave cycles are issue stalls on the vector memory pipe -- the
// kernel is bound by gather REQUESTS, not HBM bytes.  This kernel takes requests off that
// pipe and keeps many of them in flight:
//   * one 1024-thread workgroup per CU copies the hottest prefix of x (hub-first order:
//     the ~12K most gathered vertices, 95 KiB) into LDS once per launch; gathers of those
//     columns are ds_read_b64, the rest go to L2 / MALL;
//   * every wave owns a private 4 KiB LDS stage and works through equal-size items,
//     statically interleaved over the grid: a STREAM item is <= 508 consecutive entries
//     of <= 63 whole rows (two 16-B index loads + eight gathers per lane, staged, then
//     reduced by lane groups of 64 / rows); a LONG item is <= 4096 entries of one row;
//   * while the gathers of item i are in flight the wave already issues the index, row-
//     pointer and out-degree loads of item i + 1 (software pipeline, one gather round trip
//     exposed per item);
//   * the rank's dangling-score sum is reduced in the same launch (lanes -> wave ->
//     workgroup -> the last-arriving workgroup adds the per-workgroup partials in order).
// Static item assignment fixes every summation order: results are deterministic.
#include <algorithm>

#include "gx_pr.h"

namespace gx {
namespace {

constexpr int kWaves = kHubBlock / kWave;   // 16
constexpr int kStage = 512;                 // doubles per wave stage
constexpr int kStreamMax = 508;             // entries per STREAM item (2 x 64 int4 incl. alignment)
constexpr int kStreamRowsMax = 63;          // rows per STREAM item (row offsets in one lane each)
constexpr int kLongSeg = 4096;              // entries per LONG item
constexpr int kHubMax = 12224;              // doubles of x cached in LDS (95.5 KiB)

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
    int32_t hub_entries;
    uint32_t x_bytes;
    double teleport0, damping_over_n, damping;
    const int32_t *long_first;
    const int32_t *long_nseg;
    double *long_part;
    uint32_t *long_ticket;
    double *gpart;
    uint32_t *gticket;
    double *xd;
    int64_t live;
};

// Buffer resource of a global array (stride 0, raw byte offsets, range-checked).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

constexpr uint32_t kOob = 0x80000000u;   // offset past every record: the lane is dropped

// x[c]: from the LDS hub when c < H, else from global memory through a range-checked buffer
// load.  Hub lanes get an out-of-range offset, so the hardware drops them (no cache access,
// value 0) without a branch: the compiler keeps exact vmcnt counts and the next item's
// loads stay in flight.  (Exec-masking via branches forced vmcnt(0); pointing hub lanes at
// one shared line still cost one vector-L1 access per lane -- both measured.)
__device__ __forceinline__ void gather4(const double *hub, int32_t H, __amdgpu_buffer_rsrc_t xr, const int4 c,
                                        double v[4]) {
    const int cc[4] = {c.x, c.y, c.z, c.w};
    double hv[4], gv[4];
#pragma unroll
    for (int k = 0; k < 4; k++) hv[k] = hub[cc[k] < H ? cc[k] : 0];
#pragma unroll
    for (int k = 0; k < 4; k++)
        gv[k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                               xr, cc[k] < H ? kOob : (uint32_t)cc[k] * 8u, 0, 0));
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = cc[k] < H ? hv[k] : gv[k];
}

// 16 column indices (int4) at entry offset q*4 of a per-item descriptor; lanes past the
// item's records read zeros (no access).  aux 2 = non-temporal (read-once stream).
__device__ __forceinline__ int4 load_idx4(__amdgpu_buffer_rsrc_t r, int q) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)q * 16u, 0, 2);
    return make_int4((int)v[0], (int)v[1], (int)v[2], (int)v[3]);
}

// Operands of one STREAM item, loaded ahead of its gathers.  All loads are unconditional
// (addresses clamped into the item) and nothing is computed from them here, so issuing
// them never waits on the gathers already in flight.
struct StreamOps {
    int4 c0, c1;      // column indices of entries base + 4*lane .. and base + 4*(lane+64) ..
    int64_t rp;       // row pointer of row min(lane, nrows)
    int32_t deg;      // out-degree of row min(lane, nrows - 1)
};

__device__ __forceinline__ StreamOps load_stream(const HubArgs &a, const WaveItem &w, int lane) {
    StreamOps o;
    const int64_t base = w.nz_begin & ~(int64_t)3;
    const int nq = (int)((w.nz_end - base + 3) >> 2);
    const int qmax = nq > 0 ? nq - 1 : 0;
    const __amdgpu_buffer_rsrc_t cr = rsrc_of(a.ci + base, (uint32_t)nq * 16u);
    (void)qmax;
    o.c0 = load_idx4(cr, lane);
    o.c1 = load_idx4(cr, lane + kWave);
    const int nrows = w.row_end - w.row_begin;
    o.rp = a.rp[w.row_begin + min(lane, nrows)];
    o.deg = a.outdeg[w.row_begin + min(lane, nrows - 1)];
    return o;
}

__device__ __forceinline__ double finish_row(const HubArgs &a, int32_t row, double s, double teleport,
                                             int32_t deg) {
    const double r = teleport + s;
    if (a.rank_out) a.rank_out[row] = r;
    store_x(a.x_out, a.xd, a.live, row, deg > 0 ? r / ((double)deg / a.damping) : r);
    return deg == 0 ? r : 0.0;   // contribution to the dangling sum
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LONG item: entries [zb, ze) of one row; returns this lane's partial sum.
__device__ __forceinline__ double long_sum(const HubArgs &a, const double *hub, __amdgpu_buffer_rsrc_t xr,
                                           int64_t zb, int64_t ze, int lane) {
    const int64_t base = zb & ~(int64_t)3;
    const int nq = (int)((ze - base + 3) >> 2);
    const __amdgpu_buffer_rsrc_t cr = rsrc_of(a.ci + base, (uint32_t)nq * 16u);
    double s = 0.0;
    for (int q0 = 0; q0 < nq; q0 += 4 * kWave) {
        int4 c[4];
#pragma unroll
        for (int j = 0; j < 4; j++) c[j] = load_idx4(cr, q0 + lane + j * kWave);
        double v[4][4];
#pragma unroll
        for (int j = 0; j < 4; j++) gather4(hub, a.hub_entries, xr, c[j], v[j]);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e = base + 4 * (int64_t)(q0 + lane + j * kWave);
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (e + k >= zb && e + k < ze) s += v[j][k];
        }
    }
    return s;
}

__global__ __launch_bounds__(kHubBlock) void k_pr_pull_hub(HubArgs a) {
    __shared__ __attribute__((aligned(16))) double hub[kHubMax];
    __shared__ __attribute__((aligned(16))) double stage[kWaves][kStage];
    __shared__ double wsum[kWaves];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    {
        // all loads first, then all LDS stores (one round trip for the whole fill)
        constexpr int kFill = (kHubMax / 2 + kHubBlock - 1) / kHubBlock;
        const double2 *src = reinterpret_cast<const double2 *>(a.x_in);
        double2 *dst = reinterpret_cast<double2 *>(hub);
        const int npair = a.hub_entries / 2;
        if (npair > 0) {
            // clamped loads AND stores: lanes past the end rewrite the last pair with its
            // own value, so there is no branch between the loads and the LDS stores
            double2 t[kFill];
#pragma unroll
            for (int j = 0; j < kFill; j++) t[j] = src[min(tid + j * kHubBlock, npair - 1)];
#pragma unroll
            for (int j = 0; j < kFill; j++) dst[min(tid + j * kHubBlock, npair - 1)] = t[j];
        }
        if ((a.hub_entries & 1) && tid == 0) hub[a.hub_entries - 1] = a.x_in[a.hub_entries - 1];
    }
    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    __syncthreads();

    double *st = stage[wv];
    const __amdgpu_buffer_rsrc_t xr = rsrc_of(a.x_in, a.x_bytes);
    double dang = 0.0;
    const uint32_t nw = gridDim.x * kWaves;
    uint32_t i = (uint32_t)wv * gridDim.x + blockIdx.x;
    bool have = i < a.nitems;
    WaveItem cur{};
    StreamOps ops{};
    if (have) {
        cur = a.items[i];
        if (cur.split < 0) ops = load_stream(a, cur, lane);
    }
    while (have) {
        const uint32_t ni = i + nw;
        const bool nhave = ni < a.nitems;
        WaveItem nxt{};
        if (nhave) nxt = a.items[ni];
        if (cur.split >= 0) {
            // ---- LONG item: one segment of one row
            const double s = wave_sum(long_sum(a, hub, xr, cur.nz_begin, cur.nz_end, lane));
            if (lane == 0) {
                const int32_t nseg = a.long_nseg[cur.split];
                const int32_t row = cur.row_begin;
                if (nseg == 1) {
                    dang += finish_row(a, row, s, teleport, a.outdeg[row]);
                } else {
                    const int32_t first = a.long_first[cur.split];
                    __hip_atomic_store(&a.long_part[first + cur.seg], s, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const uint32_t t = __hip_atomic_fetch_add(&a.long_ticket[cur.split], 1u,
                                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (t == (uint32_t)(nseg - 1)) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        double all = 0.0;
                        for (int j = 0; j < nseg; j++)
                            all += __hip_atomic_load(&a.long_part[first + j], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&a.long_ticket[cur.split], 0u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        dang += finish_row(a, row, all, teleport, a.outdeg[row]);
                    }
                }
            }
            if (nhave && nxt.split < 0) ops = load_stream(a, nxt, lane);
        } else {
            // ---- STREAM item: gathers of this item, then the next item's operands
            double v0[4], v1[4];
            gather4(hub, a.hub_entries, xr, ops.c0, v0);
            gather4(hub, a.hub_entries, xr, ops.c1, v1);
            StreamOps nops{};
            if (nhave && nxt.split < 0) nops = load_stream(a, nxt, lane);
            const int64_t base = cur.nz_begin & ~(int64_t)3;
            const int nq = (int)((cur.nz_end - base + 3) >> 2);
            if (lane < nq) {
                double2 *d = reinterpret_cast<double2 *>(st + 4 * lane);
                d[0] = make_double2(v0[0], v0[1]);
                d[1] = make_double2(v0[2], v0[3]);
            }
            if (lane + kWave < nq) {
                double2 *d = reinterpret_cast<double2 *>(st + 4 * (lane + kWave));
                d[0] = make_double2(v1[0], v1[1]);
                d[1] = make_double2(v1[2], v1[3]);
            }
            wave_sync_lds();
            const int nrows = cur.row_end - cur.row_begin;
            int P = 1;
            while (P < nrows) P <<= 1;
            const int L = kWave / P;
            const int row = lane / L, gl = lane & (L - 1);
            const int rpv = (int)(ops.rp - base);
            const int kb = __shfl(rpv, row, kWave);
            const int ke = __shfl(rpv, row + 1 < kWave ? row + 1 : 0, kWave);
            const int32_t deg = __shfl(ops.deg, row, kWave);
            double s = 0.0;
            if (row < nrows)
                for (int k = kb + gl; k < ke; k += L) s += st[k];
            for (int off = L >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
            if (row < nrows && gl == 0) dang += finish_row(a, cur.row_begin + row, s, teleport, deg);
            wave_sync_lds();
            ops = nops;
        }
        cur = nxt;
        i = ni;
        have = nhave;
    }

    // dangling sum of the rank: lanes -> wave -> workgroup -> last-arriving workgroup
    dang = wave_sum(dang);
    if (lane == 0) wsum[wv] = dang;
    __syncthreads();
    if (tid != 0) return;
    double bs = 0.0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) bs += wsum[w];
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
        if (len > kStreamMax) {
            longrows.push_back({len, (int32_t)r});
            r++;
            continue;
        }
        const int64_t start = r;
        int64_t nz = 0;
        while (r < rows && r - start < kStreamRowsMax) {
            const int64_t l = h_rp[r + 1] - h_rp[r];
            if (l > kStreamMax || nz + l > kStreamMax) break;
            nz += l;
            r++;
        }
        streami.push_back({h_rp[start], h_rp[r], (int32_t)start, (int32_t)r, -1, 0, 0, 0});
    }
    // longest rows first: their items are the heaviest
    std::stable_sort(longrows.begin(), longrows.end(),
                     [](const auto &x, const auto &y) { return x.first > y.first; });
    for (const auto &lr : longrows) {
        const int32_t row = lr.second;
        const int32_t nseg = (int32_t)((lr.first + kLongSeg - 1) / kLongSeg);
        const int32_t sp = (int32_t)lfirst.size();
        lfirst.push_back(nsegs);
        lnseg.push_back(nseg);
        for (int32_t s = 0; s < nseg; s++) {
            const int64_t zb = h_rp[row] + (int64_t)s * kLongSeg;
            const int64_t ze = std::min<int64_t>(zb + kLongSeg, h_rp[row + 1]);
            longi.push_back({zb, ze, row, row + 1, sp, s, 0, 0});
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
    a.hub_entries = (int32_t)p->hub_entries;
    a.x_bytes = (uint32_t)(p->chunk * (uint64_t)p->nranks * 8u);
    a.teleport0 = (1.0 - p->damping) / dn;
    a.damping_over_n = p->damping / dn;
    a.damping = p->damping;
    a.long_first = p->hlong_first.p;
    a.long_nseg = p->hlong_nseg.p;
    a.long_part = p->hlong_part.p;
    a.long_ticket = p->hlong_ticket.p;
    a.xd = p->xd.p;
    a.live = (int64_t)p->live;
    a.gpart = p->gpart.p;
    a.gticket = p->gticket.p;
    {
        KTimer kt(p->ctx, "pr_pull", s);
        hipLaunchKernelGGL(k_pr_pull_hub, dim3(p->hub_grid), dim3(kHubBlock), 0, s, a);
    }
    return check_launch("k_pr_pull_hub");
}

}  // namespace gx

GX_MODULE_WARMER(pr_hub)
