// gx_lcc.hip -- local clustering coefficient via degree-oriented triangle enumeration.
//
// Replaces LA_LCC -> LAGraph_lcc(&d, A, symmetric = !directed) (lcc.cpp:61-71), which
// SuiteSparse runs as a masked SpGEMM (C<S> = S*S-type, PLUS_PAIR) plus reductions.
// With N(v) = in(v) U out(v) (the undirected closure S, built on the device) and
// k = |N(v)|:
//     LCC(v) = #{(u, w) in E : u, w in N(v)} / (k (k - 1)),   0 when k < 2.
// Each triangle {a, b, c} of S contributes to a the number of stored directions between b
// and c (1 or 2: the popcount of that S entry's flag byte), and likewise for b and c.
// Triangles are enumerated once each on the degree-ordered orientation O of S (edge v->u
// when (deg u, u) > (deg v, v)), whose out-degrees are at most sqrt(2|E|).
//   orientation : stream compaction of S by 64-entry slabs (ballot masks + one scan);
//   triangles   : per vertex v, O(v) goes into an LDS hash table (flag byte kept with each
//                 key); the lists O(u), u in O(v), are walked by load-balanced waves and every
//                 x probed: a hit is the triangle {v, u, x}.  The three contributions are
//                 summed on chip (v in a register, u in an LDS slot per u, x in its hash slot)
//                 and leave as one 64-bit atomic per (vertex, contribution target).
//   tiers       : wave per vertex for |O(v)| <= kWaveMax, workgroup per vertex up to
//                 kBlockMax, a merge-intersection fallback beyond (not reached on
//                 degree-oriented graphs below ~2^25 edges).
// Counts are exact integers, so the result is deterministic and equal to the oracle bit for
// bit (one fp64 division per vertex).
#include <cstring>
#include <memory>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kLccBlock = 256;
constexpr int kWavesPerBlock = kLccBlock / kWave;
constexpr int kWaveMax = 256;          // wave tier: |O(v)| <= 256, table <= 512 slots
constexpr int kWaveSlots = 512;
constexpr int kBlockMax = 8192;        // workgroup tier: table of 16384 slots (128 KiB)
constexpr int kBlockSlots = 16384;
constexpr uint32_t kCntMask = (1u << 30) - 1;   // hash value: flag popcount << 30 | x count

__device__ __forceinline__ bool ranks_above(int64_t du, int32_t u, int64_t dv, int32_t v) {
    return du > dv || (du == dv && u > v);
}

__device__ __forceinline__ uint32_t hash_slot(int32_t x, uint32_t mask) {
    return ((uint32_t)x * 0x9E3779B1u) & mask;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- orientation by slab compaction ----
// One wave per 64-entry slab of S: lane = entry, its row found by a shuffle search over the
// slab's (at most 64) rows or a binary search; kept = the column ranks above the row.
__device__ __forceinline__ int64_t slab_row(const int64_t *__restrict__ rp, int64_t n, int64_t e0, int64_t e_last,
                                            int64_t ee, int lane) {
    const int64_t r0 = row_of_edge(rp, n, e0), r1 = row_of_edge(rp, n, e_last);
    if (r1 - r0 < kWave) {
        const int64_t rpk = rp[min(r0 + 1 + lane, n)];
        int o = 0;
#pragma unroll
        for (int step = kWave / 2; step > 0; step >>= 1)
            if (__shfl(rpk, o + step - 1, kWave) <= ee) o += step;
        return r0 + o;
    }
    int64_t lo = r0, hi = r1 + 1;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (rp[mid] <= ee) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kLccBlock) void k_orient_masks(const int64_t *__restrict__ rp,
                                                            const int32_t *__restrict__ ci, int64_t n, int64_t nnz,
                                                            int64_t nslabs, uint64_t *mask, int32_t *cnt) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t sl = ((int64_t)blockIdx.x * kLccBlock + threadIdx.x) / kWave; sl < nslabs; sl += nw) {
        const int64_t e0 = sl * kWave, e_last = min(e0 + kWave, nnz) - 1;
        const int64_t e = e0 + lane;
        const bool valid = e < nnz;
        const int64_t ee = valid ? e : e_last;
        const int64_t v = slab_row(rp, n, e0, e_last, ee, lane);
        const int32_t u = ci[ee];
        const bool keep = valid && ranks_above(rp[u + 1] - rp[u], u, rp[v + 1] - rp[v], (int32_t)v);
        const uint64_t m = __ballot(keep);
        if (lane == 0) {
            mask[sl] = m;
            cnt[sl] = __popcll(m);
        }
    }
}

__device__ __forceinline__ int64_t kept_before(const uint64_t *mask, const int64_t *cpre, int64_t e) {
    const int64_t sl = e / kWave;
    const int b = (int)(e % kWave);
    return cpre[sl] + (b ? __popcll(mask[sl] & ((1ull << b) - 1)) : 0);
}

__global__ void k_orient_rows(const int64_t *__restrict__ rp, const uint64_t *__restrict__ mask,
                              const int64_t *__restrict__ cpre, int64_t n, int64_t *orp) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x)
        orp[v] = kept_before(mask, cpre, rp[v]);
}

__global__ __launch_bounds__(kLccBlock) void k_orient_scatter(const int32_t *__restrict__ ci,
                                                              const uint8_t *__restrict__ fl, int64_t nnz,
                                                              const uint64_t *__restrict__ mask,
                                                              const int64_t *__restrict__ cpre, int32_t *oci,
                                                              uint8_t *ofl) {
    for (int64_t e = (int64_t)blockIdx.x * kLccBlock + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * kLccBlock) {
        const int64_t sl = e / kWave;
        const int b = (int)(e % kWave);
        const uint64_t m = mask[sl];
        if ((m >> b) & 1ull) {
            const int64_t pos = cpre[sl] + (b ? __popcll(m & ((1ull << b) - 1)) : 0);
            oci[pos] = ci[e];
            ofl[pos] = fl[e];
        }
    }
}

// ---- vertex tiers ----
// Tier lists.  A workgroup stages one kClassTile-vertex tile in LDS (positions from LDS
// atomics) and flushes each tier with one global atomic: per-wave appends to three shared
// counters were ~65K same-address atomics, ~11 ns each serialised.
constexpr int kClassTile = 4096;

__global__ __launch_bounds__(kLccBlock) void k_lcc_classify(const int64_t *__restrict__ orp, int64_t v0, int64_t v1,
                                                            int32_t *wave_list, uint32_t *wave_cnt,
                                                            int32_t *block_list, uint32_t *block_cnt,
                                                            int32_t *big_list, uint32_t *big_cnt) {
    __shared__ int32_t buf[3][kClassTile];
    __shared__ uint32_t cnt[3], base[3];
    int32_t *lists[3] = {wave_list, block_list, big_list};
    uint32_t *gcnt[3] = {wave_cnt, block_cnt, big_cnt};
    for (int64_t t0 = v0 + (int64_t)blockIdx.x * kClassTile; t0 < v1; t0 += (int64_t)gridDim.x * kClassTile) {
        const int64_t t1 = min(t0 + (int64_t)kClassTile, v1);
        if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
        __syncthreads();
        for (int64_t v = t0 + threadIdx.x; v < t1; v += kLccBlock) {
            const int64_t d = orp[v + 1] - orp[v];
            const int tier = d <= 0 ? -1 : (d <= kWaveMax ? 0 : (d <= kBlockMax ? 1 : 2));
            if (tier >= 0) buf[tier][atomicAdd(&cnt[tier], 1u)] = (int32_t)v;
        }
        __syncthreads();
        if (threadIdx.x < 3) base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(gcnt[threadIdx.x], cnt[threadIdx.x]) : 0u;
        __syncthreads();
        for (int t = 0; t < 3; t++)
            for (uint32_t i = threadIdx.x; i < cnt[t]; i += kLccBlock) lists[t][base[t] + i] = buf[t][i];
        __syncthreads();
    }
}

// Probe the lists O(u) of the u in [g, g + 64) of O(v) (one u per lane) against the table.
// Lanes walk the concatenated lists 64 entries at a time (owner lane by shuffle search).
// Returns v's contribution; u's contributions go to ucnt[lane], x's into the table values.
__device__ __forceinline__ unsigned long long probe_group(const int64_t *__restrict__ orp,
                                                          const int32_t *__restrict__ oci,
                                                          const uint8_t *__restrict__ ofl, int64_t b, int64_t d,
                                                          int64_t g, const int32_t *hkey, uint32_t *hval,
                                                          uint32_t hmask, uint32_t *ucnt, int lane) {
    const int64_t i = g + lane;
    const bool has = i < d;
    const int32_t u = has ? oci[b + i] : 0;
    const uint32_t fvu = has ? (uint32_t)__popc(ofl[b + i]) : 0u;
    const int64_t ub = has ? orp[u] : 0;
    const int32_t ul = has ? (int32_t)(orp[u + 1] - ub) : 0;
    int32_t incl = ul;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int32_t y = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += y;
    }
    const int32_t total = __shfl(incl, kWave - 1, kWave);
    const int32_t excl = incl - ul;
    unsigned long long tv = 0;
    for (int32_t e0 = 0; e0 < total; e0 += kWave) {
        const int32_t e_raw = e0 + lane;
        const bool act = e_raw < total;
        const int32_t e = act ? e_raw : total - 1;
        int o = 0;
#pragma unroll
        for (int step = kWave / 2; step > 0; step >>= 1)
            if (__shfl(incl, o + step - 1, kWave) <= e) o += step;
        const int64_t k = __shfl(ub, o, kWave) + (e - __shfl(excl, o, kWave));
        const uint32_t f_vu = __shfl(fvu, o, kWave);
        const int32_t x = oci[k];
        const uint32_t f_ux = (uint32_t)__popc(ofl[k]);
        if (act) {
            uint32_t h = hash_slot(x, hmask);
            int32_t key;
            while ((key = hkey[h]) != x && key != -1) h = (h + 1) & hmask;
            if (key == x) {
                tv += f_ux;                                      // v: directions between u and x
                atomicAdd(&ucnt[o], hval[h] >> 30);              // u: directions between v and x
                atomicAdd(&hval[h], f_vu);                       // x: directions between v and u
            }
        }
    }
    return tv;
}

__global__ __launch_bounds__(kLccBlock) void k_lcc_wave(const int64_t *__restrict__ orp,
                                                        const int32_t *__restrict__ oci,
                                                        const uint8_t *__restrict__ ofl,
                                                        const int32_t *__restrict__ list, uint32_t count,
                                                        unsigned long long *tc) {
    __shared__ int32_t s_key[kWavesPerBlock][kWaveSlots];
    __shared__ uint32_t s_val[kWavesPerBlock][kWaveSlots];
    __shared__ uint32_t s_ucnt[kWavesPerBlock][kWave];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    int32_t *hkey = s_key[wv];
    uint32_t *hval = s_val[wv];
    uint32_t *ucnt = s_ucnt[wv];
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    for (uint32_t li = blockIdx.x * kWavesPerBlock + wv; li < count; li += nw) {
        const int32_t v = list[li];
        const int64_t b = orp[v], d = orp[v + 1] - b;
        uint32_t slots = 64;
        while (slots < 2 * (uint32_t)d) slots <<= 1;
        const uint32_t hmask = slots - 1;
        for (uint32_t s = lane; s < slots; s += kWave) {
            hkey[s] = -1;
            hval[s] = 0;
        }
        wave_sync_lds();
        for (int64_t i = lane; i < d; i += kWave) {
            const int32_t x = oci[b + i];
            uint32_t h = hash_slot(x, hmask);
            while (atomicCAS(&hkey[h], -1, x) != -1) h = (h + 1) & hmask;   // keys of a row are distinct
            hval[h] = (uint32_t)__popc(ofl[b + i]) << 30;
        }
        wave_sync_lds();
        unsigned long long tv = 0;
        for (int64_t g = 0; g < d; g += kWave) {
            ucnt[lane] = 0;
            wave_sync_lds();
            tv += probe_group(orp, oci, ofl, b, d, g, hkey, hval, hmask, ucnt, lane);
            wave_sync_lds();
            const uint32_t c = ucnt[lane];
            if (c && g + lane < d) atomicAdd(&tc[oci[b + g + lane]], (unsigned long long)c);
        }
        for (uint32_t s = lane; s < slots; s += kWave) {
            const uint32_t c = hval[s] & kCntMask;
            if (c) atomicAdd(&tc[hkey[s]], (unsigned long long)c);
        }
        for (int off = 32; off > 0; off >>= 1) tv += __shfl_xor(tv, off, kWave);
        if (lane == 0 && tv) atomicAdd(&tc[v], tv);
        wave_sync_lds();
    }
}

__global__ __launch_bounds__(kLccBlock) void k_lcc_block(const int64_t *__restrict__ orp,
                                                         const int32_t *__restrict__ oci,
                                                         const uint8_t *__restrict__ ofl,
                                                         const int32_t *__restrict__ list, uint32_t count,
                                                         unsigned long long *tc) {
    __shared__ int32_t hkey[kBlockSlots];
    __shared__ uint32_t hval[kBlockSlots];
    __shared__ uint32_t s_ucnt[kWavesPerBlock][kWave];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    uint32_t *ucnt = s_ucnt[wv];
    for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
        const int32_t v = list[li];
        const int64_t b = orp[v], d = orp[v + 1] - b;
        uint32_t slots = 64;
        while (slots < 2 * (uint32_t)d) slots <<= 1;
        const uint32_t hmask = slots - 1;
        for (uint32_t s = threadIdx.x; s < slots; s += kLccBlock) {
            hkey[s] = -1;
            hval[s] = 0;
        }
        __syncthreads();
        for (int64_t i = threadIdx.x; i < d; i += kLccBlock) {
            const int32_t x = oci[b + i];
            uint32_t h = hash_slot(x, hmask);
            while (atomicCAS(&hkey[h], -1, x) != -1) h = (h + 1) & hmask;
            hval[h] = (uint32_t)__popc(ofl[b + i]) << 30;
        }
        __syncthreads();
        unsigned long long tv = 0;
        for (int64_t g = (int64_t)wv * kWave; g < d; g += kLccBlock) {
            ucnt[lane] = 0;
            wave_sync_lds();
            tv += probe_group(orp, oci, ofl, b, d, g, hkey, hval, hmask, ucnt, lane);
            wave_sync_lds();
            const uint32_t c = ucnt[lane];
            if (c && g + lane < d) atomicAdd(&tc[oci[b + g + lane]], (unsigned long long)c);
        }
        __syncthreads();
        for (uint32_t s = threadIdx.x; s < slots; s += kLccBlock) {
            const uint32_t c = hval[s] & kCntMask;
            if (c) atomicAdd(&tc[hkey[s]], (unsigned long long)c);
        }
        for (int off = 32; off > 0; off >>= 1) tv += __shfl_xor(tv, off, kWave);
        if (lane == 0 && tv) atomicAdd(&tc[v], tv);
        __syncthreads();
    }
}

// Fallback for |O(v)| > kBlockMax: thread per oriented edge (v, u) of one vertex, merge
// intersection of the sorted lists O(v) and O(u).
__global__ __launch_bounds__(kLccBlock) void k_lcc_merge_row(const int64_t *__restrict__ orp,
                                                             const int32_t *__restrict__ oci,
                                                             const uint8_t *__restrict__ ofl, int32_t v,
                                                             unsigned long long *tc) {
    const int64_t b = orp[v], ie_v = orp[v + 1];
    for (int64_t e = b + (int64_t)blockIdx.x * kLccBlock + threadIdx.x; e < ie_v;
         e += (int64_t)gridDim.x * kLccBlock) {
        const int32_t u = oci[e];
        const unsigned cvu = __popc(ofl[e]);
        int64_t i = b, j = orp[u];
        const int64_t je = orp[u + 1];
        unsigned long long tv = 0, tu = 0;
        while (i < ie_v && j < je) {
            const int32_t x = oci[i], y = oci[j];
            if (x < y) {
                i++;
            } else if (x > y) {
                j++;
            } else {
                tv += __popc(ofl[j]);
                tu += __popc(ofl[i]);
                atomicAdd(&tc[x], (unsigned long long)cvu);
                i++;
                j++;
            }
        }
        if (tv) atomicAdd(&tc[v], tv);
        if (tu) atomicAdd(&tc[u], tu);
    }
}

// Work estimate of vertex v for balancing ranks: |O(v)| + sum over u in O(v) of |O(u)|.
__global__ void k_lcc_work(const int64_t *__restrict__ orp, const int32_t *__restrict__ oci, int64_t n,
                           uint64_t *work) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        uint64_t w = 1;
        for (int64_t k = orp[v]; k < orp[v + 1]; k++) {
            const int32_t u = oci[k];
            w += 1 + (uint64_t)(orp[u + 1] - orp[u]);
        }
        work[v] = w;
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

// Degree-ordered orientation O of the closure S (CSR: orp, oci, ofl).
struct LccOrient {
    int64_t m = 0;
    DBuf<int64_t> orp;
    DBuf<int32_t> oci;
    DBuf<uint8_t> ofl;
};

int lcc_orient(gx_graph *g, LccOrient &O, hipStream_t s) {
    gx_ctx *ctx = g->ctx;
    const int64_t n = (int64_t)g->n;
    const DevCSR &S = g->S;
    const int64_t nnz = (int64_t)S.h_rp[n];
    const int64_t nslabs = (nnz + kWave - 1) / kWave;
    DBuf<uint64_t> mask;
    DBuf<int32_t> cnt;
    DBuf<int64_t> cpre;
    GX_TRY(mask.alloc(nslabs + 1));
    GX_TRY(cnt.alloc(nslabs + 1));
    GX_TRY(cpre.alloc(nslabs + 1));
    GX_TRY(O.orp.alloc(n + 1));
    GX_HIP_TRY(hipMemsetAsync(cnt.p + nslabs, 0, sizeof(int32_t), s));
    GX_HIP_TRY(hipMemsetAsync(mask.p + nslabs, 0, sizeof(uint64_t), s));
    KTimer kt(ctx, "lcc_orient", s);
    if (nslabs)
        hipLaunchKernelGGL(k_orient_masks, dim3(grid_for((uint64_t)nslabs * kWave, kLccBlock, 16384)), dim3(kLccBlock),
                           0, s, S.rp.p, S.ci.p, n, nnz, nslabs, mask.p, cnt.p);
    GX_TRY(check_launch("k_orient_masks"));
    size_t tmp_bytes = 0;
    GX_HIP_TRY(rocprim::exclusive_scan(nullptr, tmp_bytes, cnt.p, cpre.p, (int64_t)0, (size_t)(nslabs + 1),
                                       rocprim::plus<int64_t>(), s));
    DBuf<char> tmp;
    GX_TRY(tmp.alloc(tmp_bytes));
    GX_HIP_TRY(rocprim::exclusive_scan(tmp.p, tmp_bytes, cnt.p, cpre.p, (int64_t)0, (size_t)(nslabs + 1),
                                       rocprim::plus<int64_t>(), s));
    hipLaunchKernelGGL(k_orient_rows, dim3(grid_for(n + 1, 256, 16384)), dim3(256), 0, s, S.rp.p, mask.p, cpre.p, n,
                       O.orp.p);
    GX_TRY(check_launch("k_orient_rows"));
    GX_HIP_TRY(hipMemcpyAsync(&O.m, O.orp.p + n, 8, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    GX_TRY(O.oci.alloc(O.m));
    GX_TRY(O.ofl.alloc(O.m));
    if (nnz)
        hipLaunchKernelGGL(k_orient_scatter, dim3(grid_for(nnz, kLccBlock, 16384)), dim3(kLccBlock), 0, s, S.ci.p,
                           S.flag.p, nnz, mask.p, cpre.p, O.oci.p, O.ofl.p);
    GX_TRY(check_launch("k_orient_scatter"));
    GX_HIP_TRY(hipStreamSynchronize(s));   // the temporaries are freed on return
    return GX_SUCCESS;
}

// Adds the triangle contributions of every triangle whose lowest-ranked vertex (the
// orientation source) lies in [v0, v1) into tc (n counters).
int lcc_count_range(gx_graph *g, const LccOrient &O, int64_t v0, int64_t v1, unsigned long long *tc,
                    hipStream_t s) {
    gx_ctx *ctx = g->ctx;
    const int64_t n = (int64_t)g->n, nv = v1 - v0;
    if (nv <= 0 || O.m == 0) return GX_SUCCESS;
    DBuf<int32_t> lists;
    DBuf<uint32_t> counts;
    GX_TRY(lists.alloc(3 * (uint64_t)nv));
    GX_TRY(counts.alloc(3));
    GX_HIP_TRY(hipMemsetAsync(counts.p, 0, 12, s));
    hipLaunchKernelGGL(k_lcc_classify, dim3((unsigned)std::min<int64_t>((nv + kClassTile - 1) / kClassTile, 2048)),
                       dim3(kLccBlock), 0, s, O.orp.p, v0, v1, lists.p,
                       counts.p, lists.p + nv, counts.p + 1, lists.p + 2 * nv, counts.p + 2);
    GX_TRY(check_launch("k_lcc_classify"));
    uint32_t hc[3] = {0, 0, 0};
    GX_HIP_TRY(hipMemcpyAsync(hc, counts.p, 12, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    {
        KTimer kt(ctx, "lcc_triangles", s);
        if (hc[0])
            hipLaunchKernelGGL(k_lcc_wave, dim3(grid_for((uint64_t)hc[0] * kWave, kLccBlock, 8192)), dim3(kLccBlock),
                               0, s, O.orp.p, O.oci.p, O.ofl.p, lists.p, hc[0], tc);
        GX_TRY(check_launch("k_lcc_wave"));
        if (hc[1])
            hipLaunchKernelGGL(k_lcc_block, dim3(std::min<uint32_t>(hc[1], 4096)), dim3(kLccBlock), 0, s, O.orp.p,
                               O.oci.p, O.ofl.p, lists.p + nv, hc[1], tc);
        GX_TRY(check_launch("k_lcc_block"));
        if (hc[2]) {
            std::vector<int32_t> big(hc[2]);
            GX_HIP_TRY(hipMemcpyAsync(big.data(), lists.p + 2 * nv, hc[2] * 4, hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            for (int32_t v : big) {
                hipLaunchKernelGGL(k_lcc_merge_row, dim3(64), dim3(kLccBlock), 0, s, O.orp.p, O.oci.p, O.ofl.p, v,
                                   tc);
                GX_TRY(check_launch("k_lcc_merge_row"));
            }
        }
    }
    GX_HIP_TRY(hipStreamSynchronize(s));   // lists are freed on return
    (void)n;
    return GX_SUCCESS;
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
    LccOrient O;
    GX_TRY(lcc_orient(g, O, s));
    DBuf<unsigned long long> tc;
    DBuf<double> out;
    GX_TRY(tc.alloc(n));
    GX_TRY(out.alloc(n));
    GX_HIP_TRY(hipMemsetAsync(tc.p, 0, n * 8, s));
    GX_TRY(lcc_count_range(g, O, 0, n, tc.p, s));
    hipLaunchKernelGGL(k_lcc_final, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, g->S.rp.p, tc.p, n, out.p);
    GX_TRY(check_launch("k_lcc_final"));
    GX_TRY(device_end(ctx));
    GX_HIP_TRY(hipMemcpy(lcc, out.p, n * 8, hipMemcpyDeviceToHost));
    return GX_SUCCESS;
}

// ---- partitioned LCC: the graph is replicated, ranks split the orientation sources; the
// caller sums the n counters of all ranks (one all-reduce) and finishes locally ----
struct gx_lcc_part {
    gx_graph *g = nullptr;
    gx::LccOrient orient;
};

extern "C" int gx_lcc_part_create(gx_graph *g, gx_lcc_part **part) {
    if (!g || !part) return fail(GX_NULL_POINTER, "gx_lcc_part_create: null argument");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    GX_TRY(ensure_closure(g));
    auto p = std::make_unique<gx_lcc_part>();
    p->g = g;
    if (g->n) GX_TRY(lcc_orient(g, p->orient, g->ctx->stream));
    *part = p.release();
    return GX_SUCCESS;
}

extern "C" int gx_lcc_part_ranges(gx_lcc_part *part, int nranks, uint64_t *ranges) {
    if (!part || !ranges) return fail(GX_NULL_POINTER, "gx_lcc_part_ranges: null argument");
    if (nranks < 1) return fail(GX_INVALID_VALUE, "gx_lcc_part_ranges: nranks < 1");
    gx_graph *g = part->g;
    const int64_t n = (int64_t)g->n;
    hipStream_t s = g->ctx->stream;
    std::vector<uint64_t> w(n);
    if (n) {
        DBuf<uint64_t> work;
        GX_TRY(work.alloc(n));
        hipLaunchKernelGGL(k_lcc_work, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, part->orient.orp.p,
                           part->orient.oci.p, n, work.p);
        GX_TRY(check_launch("k_lcc_work"));
        GX_HIP_TRY(hipMemcpyAsync(w.data(), work.p, n * 8, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
    }
    uint64_t total = 0;
    for (uint64_t x : w) total += x;
    ranges[0] = 0;
    uint64_t acc = 0;
    int64_t v = 0;
    for (int k = 1; k < nranks; k++) {
        const uint64_t target = (uint64_t)((long double)total * k / nranks);
        while (v < n && acc + w[v] <= target) acc += w[v++];
        ranges[k] = (uint64_t)v;
    }
    ranges[nranks] = (uint64_t)n;
    return GX_SUCCESS;
}

extern "C" int gx_lcc_part_counts(gx_lcc_part *part, uint64_t v0, uint64_t v1, uint64_t *tc, void *stream) {
    if (!part || !tc) return fail(GX_NULL_POINTER, "gx_lcc_part_counts: null argument");
    gx_graph *g = part->g;
    if (v0 > v1 || v1 > g->n) return fail(GX_INVALID_INDEX, "gx_lcc_part_counts: bad vertex range");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the null stream (torch's default)
    return lcc_count_range(g, part->orient, (int64_t)v0, (int64_t)v1, (unsigned long long *)tc, s);
}

extern "C" int gx_lcc_part_finish(gx_lcc_part *part, const uint64_t *tc, double *lcc, void *stream) {
    if (!part || !tc || !lcc) return fail(GX_NULL_POINTER, "gx_lcc_part_finish: null argument");
    gx_graph *g = part->g;
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the null stream (torch's default)
    if (g->n) {
        hipLaunchKernelGGL(k_lcc_final, dim3(grid_for(g->n, 256, 8192)), dim3(256), 0, s, g->S.rp.p,
                           (const unsigned long long *)tc, (int64_t)g->n, lcc);
        GX_TRY(check_launch("k_lcc_final"));
    }
    return GX_SUCCESS;
}

extern "C" int gx_lcc_part_free(gx_lcc_part *part) {
    delete part;
    return GX_SUCCESS;
}
