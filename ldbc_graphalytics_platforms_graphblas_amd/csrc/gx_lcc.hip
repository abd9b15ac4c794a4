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
//   transpose   : I = O^T by a radix sort of (x, v) keys on x only.
//   triangles   : each triangle {v, u, x} (v -> u, v -> x, u -> x) is found at its middle
//                 vertex u: O(u) goes into an LDS hash table (flag popcount kept with each
//                 key) and the lists O(v), v in I(u), are walked by load-balanced waves and
//                 probed -- sum |O(v)| probes over oriented edges, 0.45x of probing O(u) per
//                 (v, u).  The three contributions are summed on chip (u in a register, v in
//                 an LDS slot per v, x in its hash slot) and leave as one 64-bit atomic per
//                 (work item, contribution target).
//   tiers       : work item (u, 64 in-neighbours) per wave for |O(u)| <= 512 (512- or
//                 1024-slot tables), (u, 256) per workgroup up to kBlockMax (LDS sized to the
//                 tier's largest |O(u)|), a merge-intersection fallback beyond (not reached
//                 on degree-oriented graphs below ~2^25 edges).
// Oriented entries are packed as (vertex << 2) | popcount(flag), so n < 2^29.
// Counts are exact integers, so the result is deterministic and equal to the oracle bit for
// bit (one fp64 division per vertex).
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kLccBlock = 256;
constexpr int kWavesPerBlock = kLccBlock / kWave;
constexpr int kWaveMax = 256;          // wave tiers: |O(u)| <= 256 (512-slot tables) ...
constexpr int kWave2Max = 512;         // ... and <= 512 (1024-slot tables)
constexpr int kBlockMax = 8192;        // workgroup tier: table sized to the tier's largest |O(u)|
constexpr int kBlockSlots = 16384;     //   (dynamic LDS, at most 128 KiB)
constexpr uint32_t kCntMask = (1u << 30) - 1;   // hash value: flag popcount << 30 | x count
constexpr uint32_t kVMask = (1u << 29) - 1;     // in-orientation entry: core bit 31 | v << 2 | popcount
constexpr uint32_t kCoreBit = 1u << 31;

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

// ---- orientation by slab compaction (one wave per 64-entry slab of S, lane = entry) ----
__global__ __launch_bounds__(kLccBlock) void k_orient_masks(const int64_t *__restrict__ rp,
                                                            const int32_t *__restrict__ ci,
                                                            const int64_t *__restrict__ srow, int64_t n, int64_t nnz,
                                                            int64_t nslabs, uint64_t *mask, int32_t *cnt) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t sl = ((int64_t)blockIdx.x * kLccBlock + threadIdx.x) / kWave; sl < nslabs; sl += nw) {
        const int64_t e0 = sl * kWave, e_last = min(e0 + kWave, nnz) - 1;
        const int64_t e = e0 + lane;
        const bool valid = e < nnz;
        const int64_t ee = valid ? e : e_last;
        const int64_t v = slab_row_of(rp, srow, n, sl, ee, lane);
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

// Oriented entries are packed as (x << 2) | popcount(flag): one 4-byte load per probe.
__global__ __launch_bounds__(kLccBlock) void k_orient_scatter(const int32_t *__restrict__ ci,
                                                              const uint8_t *__restrict__ fl, int64_t nnz,
                                                              const uint64_t *__restrict__ mask,
                                                              const int64_t *__restrict__ cpre, uint32_t *ocode) {
    for (int64_t e = (int64_t)blockIdx.x * kLccBlock + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * kLccBlock) {
        const int64_t sl = e / kWave;
        const int b = (int)(e % kWave);
        const uint64_t m = mask[sl];
        if ((m >> b) & 1ull) {
            const int64_t pos = cpre[sl] + (b ? __popcll(m & ((1ull << b) - 1)) : 0);
            ocode[pos] = ((uint32_t)ci[e] << 2) | (uint32_t)__popc(fl[e]);
        }
    }
}

// In-orientation I (transpose of O): keys (x << 32) | (v << 2 | p) for every v -> x.
__global__ void k_orient_tkeys(const int64_t *__restrict__ orp, const uint32_t *__restrict__ ocode, int64_t n,
                               uint64_t *keys) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        for (int64_t k = orp[v]; k < orp[v + 1]; k++) {
            const uint32_t c = ocode[k];
            keys[k] = ((uint64_t)(c >> 2) << 32) | (((uint32_t)v << 2) | (c & 3u));
        }
}

__global__ void k_keys_to_in_csr(const uint64_t *__restrict__ keys, int64_t m, int64_t n, int64_t *irp,
                                 uint32_t *icode) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t <= n) {
        const uint64_t target = (uint64_t)t << 32;
        int64_t lo = 0, hi = m;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        irp[t] = lo;
    }
    for (int64_t k = t; k < m; k += (int64_t)gridDim.x * blockDim.x) icode[k] = (uint32_t)(keys[k] & 0xffffffffu);
}

// ---- work items ----
// A triangle {v, u, x} with v -> u, v -> x, u -> x (ranks v < u < x) is found once, at its
// middle vertex u: O(u) goes into an LDS hash table and the lists O(v) of the in-neighbours
// v in I(u) are probed against it.  This costs sum over oriented edges (v, u) of |O(v)|,
// less than half of probing O(u) for every (v, u) (2.4 G -> 1.06 G probes on SYN-cit).
// Work item = (u, chunk of I(u)): kWaveGroup in-neighbours for the wave tier, kBlockGroup for
// the workgroup tier, so hubs with large in-lists spread over many waves.
constexpr int kWaveGroup = kWave;
constexpr int kBlockGroup = kLccBlock;
constexpr int kClassTile = 4096;

__global__ __launch_bounds__(kLccBlock) void k_lcc_items(const int64_t *__restrict__ orp,
                                                         const int64_t *__restrict__ irp, int64_t v0, int64_t v1,
                                                         uint64_t *items0, uint64_t *items1, uint64_t *items2,
                                                         int32_t *big_list, uint32_t *counts /* 4 tiers + max d */) {
    constexpr int kTiers = 4;
    __shared__ uint32_t tot[kTiers], base[kTiers], off[kTiers];
    uint64_t *items[3] = {items0, items1, items2};
    for (int64_t t0 = v0 + (int64_t)blockIdx.x * kClassTile; t0 < v1; t0 += (int64_t)gridDim.x * kClassTile) {
        const int64_t t1 = min(t0 + (int64_t)kClassTile, v1);
        if (threadIdx.x < kTiers) {
            tot[threadIdx.x] = 0;
            off[threadIdx.x] = 0;
        }
        __syncthreads();
        for (int pass = 0; pass < 2; pass++) {
            for (int64_t u = t0 + threadIdx.x; u < t1; u += kLccBlock) {
                const int64_t d = orp[u + 1] - orp[u], e = irp[u + 1] - irp[u];
                if (d == 0 || e == 0) continue;
                const int tier = d <= kWaveMax ? 0 : (d <= kWave2Max ? 1 : (d <= kBlockMax ? 2 : 3));
                const int64_t group = tier == 2 ? kBlockGroup : kWaveGroup;
                const uint32_t ni = tier == 3 ? 1u : (uint32_t)((e + group - 1) / group);
                if (pass == 0) {
                    atomicAdd(&tot[tier], ni);
                    if (tier == 2) atomicMax(&counts[4], (uint32_t)d);
                } else {
                    const uint32_t pos = base[tier] + atomicAdd(&off[tier], ni);
                    if (tier == 3) {
                        big_list[pos] = (int32_t)u;
                    } else {
                        for (uint32_t j = 0; j < ni; j++) items[tier][pos + j] = ((uint64_t)u << 32) | j;
                    }
                }
            }
            __syncthreads();
            if (pass == 0 && threadIdx.x < kTiers)
                base[threadIdx.x] = tot[threadIdx.x] ? atomicAdd(&counts[threadIdx.x], tot[threadIdx.x]) : 0u;
            __syncthreads();
        }
    }
}

// Build the hash table of O(u) (key x, value popcount(u,x) << 30) with `nthreads` threads.
__device__ __forceinline__ void table_build(const int64_t *__restrict__ orp, const uint32_t *__restrict__ ocode,
                                            int32_t u, int32_t *hkey, uint32_t *hval, uint32_t slots, int tid,
                                            int nthreads) {
    const int64_t b = orp[u], d = orp[u + 1] - b;
    const uint32_t hmask = slots - 1;
    for (int64_t i = tid; i < d; i += nthreads) {
        const uint32_t c = ocode[b + i];
        const int32_t x = (int32_t)(c >> 2);
        uint32_t h = hash_slot(x, hmask);
        while (atomicCAS(&hkey[h], -1, x) != -1) h = (h + 1) & hmask;   // keys of a row are distinct
        hval[h] = (c & 3u) << 30;
    }
}

// Per-wave LDS scratch of probe_in_group: the nonempty lists by rank, and the list starts
// falling in the current 64-entry window.
struct WaveScratch {
    uint64_t rank[kWave];   // (O(v) start - list offset) as 48-bit signed | popcount(v,u) << 48 | lane << 56
    uint8_t mark[kWave];
};

// Which list holds position E0 + lane of the concatenated lists, and where that entry is in
// ocode: lists starting inside the window mark their offset, one ballot turns the marks into a
// mask, and the list's rank is cb (lists started before the window) plus the marks at or below
// the lane.  Replaces a 6-step shuffle binary search (six dependent ds_bpermute per window).
__device__ __forceinline__ int64_t probe_locate(WaveScratch *ws, int32_t excl, int32_t vl, int lane, int32_t E0,
                                                int32_t total, int &cb, uint64_t &pk, bool &act) {
    if (vl > 0 && excl >= E0 && excl < E0 + kWave) ws->mark[excl - E0] = 1;
    wave_sync_lds();
    const unsigned long long M = __ballot(ws->mark[lane] != 0);
    ws->mark[lane] = 0;
    const int32_t e = E0 + lane;
    act = e < total;
    const unsigned long long upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1ull);
    const int r = cb + __popcll(M & upto) - 1;
    cb += __popcll(M);
    pk = act ? ws->rank[r] : 0ull;
    wave_sync_lds();
    return ((int64_t)(pk << 16) >> 16) + e;
}

// Probe the lists O(v) of the (up to 64) in-neighbours icode[ib .. ie) of u, one per lane,
// against the table of O(u).  Lanes walk the concatenated lists 64 entries at a time; the next
// window's entries are located and loaded before the current one is probed.  Returns u's
// contribution; v's go to vcnt[lane], x's into the table values.
__device__ __forceinline__ unsigned long long probe_in_group(const int64_t *__restrict__ orp,
                                                             const uint32_t *__restrict__ ocode,
                                                             const uint32_t *__restrict__ icode, int64_t ib,
                                                             int64_t ie, const int32_t *hkey, uint32_t *hval,
                                                             uint32_t hmask, uint32_t *vcnt, int lane,
                                                             WaveScratch *ws) {
    const int64_t i = ib + lane;
    const bool has = i < ie;
    const uint32_t ic = has ? icode[i] : 0u;
    const int32_t v = (int32_t)((ic >> 2) & kVMask);
    const uint32_t p_vu = ic & 3u;
    // a dense-core in-neighbour (core bit): its triangles {v, u, x} lie wholly in the core
    // (u and x rank above v) and are counted by the core's MFMA pass (k_lcc_core_mfma)
    const bool walk = has && !(ic & kCoreBit);
    const int64_t vb = walk ? orp[v] : 0;
    const int32_t vl = walk ? (int32_t)(orp[v + 1] - vb) : 0;
    int32_t incl = vl;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int32_t y = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += y;
    }
    const int32_t total = __shfl(incl, kWave - 1, kWave);
    const int32_t excl = incl - vl;
    const unsigned long long ne = __ballot(vl > 0);
    if (vl > 0)
        ws->rank[__popcll(ne & ((1ull << lane) - 1ull))] =
            ((uint64_t)(vb - excl) & 0xffffffffffffull) | ((uint64_t)p_vu << 48) | ((uint64_t)lane << 56);
    ws->mark[lane] = 0;
    unsigned long long tu = 0;
    if (total == 0) return tu;
    int cb = 0;
    uint64_t pk;
    bool act;
    int64_t k = probe_locate(ws, excl, vl, lane, 0, total, cb, pk, act);
    uint32_t c = act ? ocode[k] : 0u;
    for (int32_t e0 = 0; e0 < total; e0 += kWave) {
        const uint32_t cc = c;
        const uint64_t pc = pk;
        const bool ac = act;
        if (e0 + kWave < total) {
            k = probe_locate(ws, excl, vl, lane, e0 + kWave, total, cb, pk, act);
            c = act ? ocode[k] : 0u;
        }
        if (ac) {
            const int32_t x = (int32_t)(cc >> 2);
            uint32_t h = hash_slot(x, hmask);
            int32_t key;
            while ((key = hkey[h]) != x && key != -1) h = (h + 1) & hmask;
            if (key == x) {
                tu += cc & 3u;                                         // u: directions between v and x
                atomicAdd(&vcnt[pc >> 56], hval[h] >> 30);             // v: directions between u and x
                atomicAdd(&hval[h], (uint32_t)(pc >> 48) & 3u);        // x: directions between v and u
            }
        }
    }
    return tu;
}

__device__ __forceinline__ uint32_t table_slots(int64_t d) {
    uint32_t slots = 64;
    while (slots < 2 * (uint32_t)d) slots <<= 1;
    return slots;
}

template <int kWaveSlots>
__global__ __launch_bounds__(kLccBlock) void k_lcc_wave(const int64_t *__restrict__ orp,
                                                        const uint32_t *__restrict__ ocode,
                                                        const int64_t *__restrict__ irp,
                                                        const uint32_t *__restrict__ icode,
                                                        const uint64_t *__restrict__ items, uint32_t count,
                                                        unsigned long long *tc) {
    __shared__ int32_t s_key[kWavesPerBlock][kWaveSlots];
    __shared__ uint32_t s_val[kWavesPerBlock][kWaveSlots];
    __shared__ uint32_t s_vcnt[kWavesPerBlock][kWave];
    __shared__ WaveScratch s_ws[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    int32_t *hkey = s_key[wv];
    uint32_t *hval = s_val[wv];
    uint32_t *vcnt = s_vcnt[wv];
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    for (uint32_t li = blockIdx.x * kWavesPerBlock + wv; li < count; li += nw) {
        const uint64_t item = items[li];
        const int32_t u = (int32_t)(item >> 32);
        const int64_t ib = irp[u] + (int64_t)(uint32_t)item * kWaveGroup, ie = min(irp[u + 1], ib + kWaveGroup);
        const uint32_t slots = table_slots(orp[u + 1] - orp[u]);
        for (uint32_t s = lane; s < slots; s += kWave) {
            hkey[s] = -1;
            hval[s] = 0;
        }
        vcnt[lane] = 0;
        wave_sync_lds();
        table_build(orp, ocode, u, hkey, hval, slots, lane, kWave);
        wave_sync_lds();
        unsigned long long tu =
            probe_in_group(orp, ocode, icode, ib, ie, hkey, hval, slots - 1, vcnt, lane, &s_ws[wv]);
        wave_sync_lds();
        const uint32_t c = vcnt[lane];
        if (c && ib + lane < ie) atomicAdd(&tc[(icode[ib + lane] >> 2) & kVMask], (unsigned long long)c);
        for (uint32_t s = lane; s < slots; s += kWave) {
            const uint32_t cx = hval[s] & kCntMask;
            if (cx) atomicAdd(&tc[hkey[s]], (unsigned long long)cx);
        }
        for (int off = 32; off > 0; off >>= 1) tu += __shfl_xor(tu, off, kWave);
        if (lane == 0 && tu) atomicAdd(&tc[u], tu);
        wave_sync_lds();
    }
}

__global__ __launch_bounds__(kLccBlock) void k_lcc_block(const int64_t *__restrict__ orp,
                                                         const uint32_t *__restrict__ ocode,
                                                         const int64_t *__restrict__ irp,
                                                         const uint32_t *__restrict__ icode,
                                                         const uint64_t *__restrict__ items, uint32_t count,
                                                         uint32_t max_slots, unsigned long long *tc) {
    extern __shared__ uint32_t dyn[];   // max_slots keys, then max_slots values
    int32_t *hkey = reinterpret_cast<int32_t *>(dyn);
    uint32_t *hval = dyn + max_slots;
    __shared__ uint32_t s_vcnt[kWavesPerBlock][kWave];
    __shared__ WaveScratch s_ws[kWavesPerBlock];
    __shared__ unsigned long long s_tu[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    uint32_t *vcnt = s_vcnt[wv];
    for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
        const uint64_t item = items[li];
        const int32_t u = (int32_t)(item >> 32);
        const int64_t ib0 = irp[u] + (int64_t)(uint32_t)item * kBlockGroup, ie0 = min(irp[u + 1], ib0 + kBlockGroup);
        const uint32_t slots = table_slots(orp[u + 1] - orp[u]);
        for (uint32_t s = threadIdx.x; s < slots; s += kLccBlock) {
            hkey[s] = -1;
            hval[s] = 0;
        }
        vcnt[lane] = 0;
        __syncthreads();
        table_build(orp, ocode, u, hkey, hval, slots, threadIdx.x, kLccBlock);
        __syncthreads();
        const int64_t ib = ib0 + (int64_t)wv * kWave, ie = min(ie0, ib + kWave);
        unsigned long long tu = 0;
        if (ib < ie) tu = probe_in_group(orp, ocode, icode, ib, ie, hkey, hval, slots - 1, vcnt, lane, &s_ws[wv]);
        wave_sync_lds();
        const uint32_t c = vcnt[lane];
        if (c && ib + lane < ie) atomicAdd(&tc[(icode[ib + lane] >> 2) & kVMask], (unsigned long long)c);
        for (int off = 32; off > 0; off >>= 1) tu += __shfl_xor(tu, off, kWave);
        if (lane == 0) s_tu[wv] = tu;
        __syncthreads();
        for (uint32_t s = threadIdx.x; s < slots; s += kLccBlock) {
            const uint32_t cx = hval[s] & kCntMask;
            if (cx) atomicAdd(&tc[hkey[s]], (unsigned long long)cx);
        }
        if (threadIdx.x == 0) {
            unsigned long long t = 0;
            for (int w = 0; w < kWavesPerBlock; w++) t += s_tu[w];
            if (t) atomicAdd(&tc[u], t);
        }
        __syncthreads();
    }
}

// Fallback for |O(u)| > kBlockMax: thread per in-neighbour v of one u, merge intersection of
// the sorted lists O(v) and O(u).
__global__ __launch_bounds__(kLccBlock) void k_lcc_merge_in(const int64_t *__restrict__ orp,
                                                            const uint32_t *__restrict__ ocode,
                                                            const int64_t *__restrict__ irp,
                                                            const uint32_t *__restrict__ icode, int32_t u,
                                                            unsigned long long *tc) {
    const int64_t ub = orp[u], ue = orp[u + 1];
    for (int64_t t = irp[u] + (int64_t)blockIdx.x * kLccBlock + threadIdx.x; t < irp[u + 1];
         t += (int64_t)gridDim.x * kLccBlock) {
        const uint32_t ic = icode[t];
        if (ic & kCoreBit) continue;   // wholly in the dense core (k_lcc_core_mfma)
        const int32_t v = (int32_t)((ic >> 2) & kVMask);
        const uint32_t p_vu = ic & 3u;
        int64_t i = orp[v], j = ub;
        const int64_t ie = orp[v + 1];
        unsigned long long tv = 0, tu = 0;
        while (i < ie && j < ue) {
            const uint32_t a = ocode[i], b = ocode[j];
            if ((a >> 2) < (b >> 2)) {
                i++;
            } else if ((a >> 2) > (b >> 2)) {
                j++;
            } else {
                tv += b & 3u;   // v: directions between u and x
                tu += a & 3u;   // u: directions between v and x
                atomicAdd(&tc[a >> 2], (unsigned long long)p_vu);
                i++;
                j++;
            }
        }
        if (tv) atomicAdd(&tc[v], tv);
        if (tu) atomicAdd(&tc[u], tu);
    }
}

// Work estimate of vertex u for balancing ranks: sum over v in I(u) of 1 + |O(v)|, plus
// |O(u)|.  One wave per vertex (hubs have long in-lists).
__global__ __launch_bounds__(kLccBlock) void k_lcc_work(const int64_t *__restrict__ orp,
                                                        const int64_t *__restrict__ irp,
                                                        const uint32_t *__restrict__ icode, int64_t n,
                                                        uint64_t *work) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t u = ((int64_t)blockIdx.x * kLccBlock + threadIdx.x) / kWave; u < n; u += nw) {
        uint64_t w = 0;
        for (int64_t k = irp[u] + lane; k < irp[u + 1]; k += kWave) {
            const int32_t v = (int32_t)((icode[k] >> 2) & kVMask);
            w += 1 + (uint64_t)(orp[v + 1] - orp[v]);
        }
        for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off, kWave);
        if (lane == 0) work[u] = w + 1 + (uint64_t)(orp[u + 1] - orp[u]);
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

// ---- dense core on the matrix cores ----
// The vertices of closure degree > dcut (the top of the orientation order, so every triangle
// whose lowest-ranked vertex is in the core lies wholly in it) form a small, dense K x K block
// of S: on SYN-cit the 4 K highest-degree vertices hold 15.5 % of the hash kernels' probe work
// at 9 % density, the 8 K highest 34 % at 5 % (tools/dense_tiles.py).  Its
// triangles are counted as a masked dense product: with W[j][k] the number of stored directions
// between core vertices j and k (0, 1, 2) and B = (W > 0),
//     t(i) = 1/2 sum_j B[i][j] (W B)[j][i],
// each core triangle {i, j, k} adding w(j, k) at i, as the hash kernels do.  W B is an int8
// GEMM on v_mfma_i32_32x32x32_i8 (exact int32 sums), the mask and the row sums fused into its
// epilogue, 64 x 64 output tiles whose mask is empty skipped.  The hash kernels skip the
// in-neighbours v in the core (core bit of the in-orientation entry), i.e. exactly the core's
// triangles.
constexpr int kCoreWG = 128;   // output tile of a workgroup (4 waves of 64 x 64)

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));

// closure degree and id of every vertex (a stable descending sort of the degrees follows)
__global__ void k_core_degkeys(const int64_t *__restrict__ srp, int64_t n, uint32_t *__restrict__ deg,
                               int32_t *__restrict__ ids) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        deg[v] = (uint32_t)(srp[v + 1] - srp[v]);
        ids[v] = (int32_t)v;
    }
}

// core index of the first K vertices of the degree-descending order (coreidx pre-filled -1)
__global__ void k_core_place(const int32_t *__restrict__ sorted_ids, int32_t K, int32_t *__restrict__ coreidx,
                             int32_t *__restrict__ corev) {
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < K; i += gridDim.x * blockDim.x) {
        const int32_t v = sorted_ids[i];
        coreidx[v] = i;
        corev[i] = v;
    }
}

// W and B rows of the core (one wave per core vertex), and the 64 x 64 tiles holding entries
__global__ __launch_bounds__(256) void k_core_fill(const int64_t *__restrict__ srp, const int32_t *__restrict__ sci,
                                                   const uint8_t *__restrict__ sflag, const int32_t *__restrict__ coreidx,
                                                   const int32_t *__restrict__ corev, int32_t K, int32_t Kp,
                                                   int8_t *__restrict__ W, int8_t *__restrict__ B,
                                                   uint8_t *__restrict__ tmask) {
    const int lane = threadIdx.x & (kWave - 1);
    const int32_t nt = Kp / 64;
    for (int32_t i = (blockIdx.x * 256 + threadIdx.x) / kWave; i < K; i += gridDim.x * 256 / kWave) {
        const int32_t v = corev[i];
        for (int64_t e = srp[v] + lane; e < srp[v + 1]; e += kWave) {
            const int32_t c = coreidx[sci[e]];
            if (c < 0) continue;
            W[(int64_t)i * Kp + c] = (int8_t)__popc((uint32_t)sflag[e]);
            B[(int64_t)i * Kp + c] = 1;
            tmask[(i / 64) * nt + c / 64] = 1;
        }
    }
}

// the core bit on every in-orientation entry whose source v is in the core
__global__ void k_core_mark_in(uint32_t *__restrict__ icode, int64_t m, const int32_t *__restrict__ coreidx) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t ic = icode[k];
        if (coreidx[(ic >> 2) & kVMask] >= 0) icode[k] = ic | kCoreBit;
    }
}

// P = W B over 128 x 128 workgroup tiles, each wave 64 x 64 (2 x 2 MFMA tiles of 32 x 32, k
// steps of 32), then t(i) += sum_j B[j][i] P[j][i] over the tile's rows j.  W and B are
// symmetric, row-major Kp x Kp int8: the A operand (rows j) and the B operand (column i = row
// i of B) are both 16 contiguous bytes per lane (lane l: row l & 31, k = 16 (l >> 5) + 0..15).
// C/D: column lane & 31, row (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
__global__ __launch_bounds__(256) void k_lcc_core_mfma(const int8_t *__restrict__ W, const int8_t *__restrict__ B,
                                                       const uint8_t *__restrict__ tmask, int32_t Kp,
                                                       unsigned long long *__restrict__ tcore) {
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int32_t nwg = Kp / kCoreWG;
    const int32_t J0 = (int32_t)(blockIdx.x / nwg) * kCoreWG + (wv >> 1) * 64;
    const int32_t I0 = (int32_t)(blockIdx.x % nwg) * kCoreWG + (wv & 1) * 64;
    if (!tmask[(J0 / 64) * (Kp / 64) + I0 / 64]) return;   // B[j][i] = 0 over the tile: nothing to add
    const int r = lane & 31, h = lane >> 5;
    const int8_t *a0 = W + (int64_t)(J0 + r) * Kp + 16 * h, *a1 = a0 + (int64_t)32 * Kp;
    const int8_t *b0 = B + (int64_t)(I0 + r) * Kp + 16 * h, *b1 = b0 + (int64_t)32 * Kp;
    i32x16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[m][n][q] = 0;
    i32x4 fa0 = *reinterpret_cast<const i32x4 *>(a0), fa1 = *reinterpret_cast<const i32x4 *>(a1);
    i32x4 fb0 = *reinterpret_cast<const i32x4 *>(b0), fb1 = *reinterpret_cast<const i32x4 *>(b1);
    for (int32_t k = 32; k <= Kp; k += 32) {
        i32x4 na0, na1, nb0, nb1;
        if (k < Kp) {   // the next k step's fragments, in flight while this one multiplies
            na0 = *reinterpret_cast<const i32x4 *>(a0 + k);
            na1 = *reinterpret_cast<const i32x4 *>(a1 + k);
            nb0 = *reinterpret_cast<const i32x4 *>(b0 + k);
            nb1 = *reinterpret_cast<const i32x4 *>(b1 + k);
        }
        acc[0][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0, fb0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0, fb1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1, fb0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1, fb1, acc[1][1], 0, 0, 0);
        if (k < Kp) {
            fa0 = na0;
            fa1 = na1;
            fb0 = nb0;
            fb1 = nb1;
        }
    }
    // epilogue: lane's column i = I0 + 32 n + r; its rows j = J0 + 32 m + 8 g + 4 h + (0..3);
    // the mask B[j][i] = B[i][j] (symmetric): four contiguous bytes of row i per (m, g)
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int32_t i = I0 + 32 * n + r;
        const int8_t *brow = B + (int64_t)i * Kp;
        int64_t s = 0;
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const uint32_t mk = *reinterpret_cast<const uint32_t *>(brow + J0 + 32 * m + 8 * g + 4 * h);
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if ((mk >> (8 * q)) & 0xffu) s += acc[m][n][4 * g + q];
            }
        s += __shfl_xor(s, 32, kWave);
        if (h == 0 && s) atomicAdd(&tcore[i], (unsigned long long)s);
    }
}

// tc[corev[i]] += tcore[i] / 2 (each core pair (j, k) came in both orders)
__global__ void k_core_final(const unsigned long long *__restrict__ tcore, const int32_t *__restrict__ corev, int32_t K,
                             unsigned long long *__restrict__ tc) {
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < K; i += gridDim.x * blockDim.x)
        if (tcore[i]) atomicAdd(&tc[corev[i]], tcore[i] / 2);
}

// Degree-ordered orientation O of the closure S (CSR orp / ocode) and its transpose I
// (irp / icode, entries (v << 2) | popcount of the v -> u entry).
struct LccOrient {
    int64_t m = 0;
    DBuf<int64_t> orp, irp;
    DBuf<uint32_t> ocode, icode;
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
    GX_TRY(O.irp.alloc(n + 1));
    DBuf<int64_t> srow;
    GX_TRY(srow.alloc(nslabs + 1));
    GX_HIP_TRY(hipMemsetAsync(cnt.p + nslabs, 0, sizeof(int32_t), s));
    GX_HIP_TRY(hipMemsetAsync(mask.p + nslabs, 0, sizeof(uint64_t), s));
    KTimer kt(ctx, "lcc_orient", s);
    GX_TRY(slab_rows(S.rp.p, n, nslabs, srow.p, s));
    if (nslabs)
        hipLaunchKernelGGL(k_orient_masks, dim3(grid_for((uint64_t)nslabs * kWave, kLccBlock, 16384)), dim3(kLccBlock),
                           0, s, S.rp.p, S.ci.p, srow.p, n, nnz, nslabs, mask.p, cnt.p);
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
    GX_TRY(O.ocode.alloc(O.m, 16));
    GX_TRY(O.icode.alloc(O.m, 16));
    if (nnz)
        hipLaunchKernelGGL(k_orient_scatter, dim3(grid_for(nnz, kLccBlock, 16384)), dim3(kLccBlock), 0, s, S.ci.p,
                           S.flag.p, nnz, mask.p, cpre.p, O.ocode.p);
    GX_TRY(check_launch("k_orient_scatter"));
    // transpose: sort (x, v|p) keys by x only (bits 32 .. 32+log2 n), then row pointers
    DBuf<uint64_t> k0, k1;
    GX_TRY(k0.alloc(O.m + 1));
    GX_TRY(k1.alloc(O.m + 1));
    if (O.m) {
        hipLaunchKernelGGL(k_orient_tkeys, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, O.orp.p, O.ocode.p, n,
                           k0.p);
        GX_TRY(check_launch("k_orient_tkeys"));
        int hb = 1;
        while ((1ll << hb) <= n) hb++;
        size_t sbytes = 0;
        GX_HIP_TRY(rocprim::radix_sort_keys(nullptr, sbytes, k0.p, k1.p, (size_t)O.m, 32, 32 + hb, s));
        DBuf<char> stmp;
        GX_TRY(stmp.alloc(sbytes));
        GX_HIP_TRY(rocprim::radix_sort_keys(stmp.p, sbytes, k0.p, k1.p, (size_t)O.m, 32, 32 + hb, s));
        GX_HIP_TRY(hipStreamSynchronize(s));   // stmp is freed at scope end
    }
    hipLaunchKernelGGL(k_keys_to_in_csr, dim3(grid_for((uint64_t)n + 1, 256, 1u << 30)), dim3(256), 0, s, k1.p, O.m, n,
                       O.irp.p, O.icode.p);
    GX_TRY(check_launch("k_keys_to_in_csr"));
    GX_HIP_TRY(hipStreamSynchronize(s));   // the temporaries are freed on return
    return GX_SUCCESS;
}

// The work items of the middle vertices in [v0, v1), by tier (k_lcc_items).
struct LccItems {
    DBuf<uint64_t> items0, items1, items2;
    DBuf<int32_t> big;
    std::vector<int32_t> h_big;
    uint32_t hc[5] = {0, 0, 0, 0, 0};   // items per tier, then the largest workgroup-tier |O(u)|
};

int lcc_items(const LccOrient &O, int64_t v0, int64_t v1, LccItems &L, hipStream_t s) {
    const int64_t nv = v1 - v0;
    if (nv <= 0 || O.m == 0) return GX_SUCCESS;
    const uint64_t icap = (uint64_t)nv + (uint64_t)O.m / kWaveGroup + 64;
    DBuf<uint32_t> counts;
    GX_TRY(L.items0.alloc(icap));
    GX_TRY(L.items1.alloc(icap));
    GX_TRY(L.items2.alloc(icap));
    GX_TRY(L.big.alloc(nv));
    GX_TRY(counts.alloc(5));
    GX_HIP_TRY(hipMemsetAsync(counts.p, 0, 20, s));
    hipLaunchKernelGGL(k_lcc_items, dim3((unsigned)std::min<int64_t>((nv + kClassTile - 1) / kClassTile, 2048)),
                       dim3(kLccBlock), 0, s, O.orp.p, O.irp.p, v0, v1, L.items0.p, L.items1.p, L.items2.p, L.big.p,
                       counts.p);
    GX_TRY(check_launch("k_lcc_items"));
    GX_HIP_TRY(hipMemcpyAsync(L.hc, counts.p, 20, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    if (L.hc[3]) {
        L.h_big.resize(L.hc[3]);
        GX_HIP_TRY(hipMemcpyAsync(L.h_big.data(), L.big.p, L.hc[3] * 4, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
    }
    return GX_SUCCESS;
}

// Adds the contributions of every triangle whose middle vertex is one of the items' into tc
// (n counters).
int lcc_count_items(gx_graph *g, const LccOrient &O, const LccItems &L, unsigned long long *tc, hipStream_t s) {
    gx_ctx *ctx = g->ctx;
    if (O.m == 0) return GX_SUCCESS;
    const uint32_t *hc = L.hc;
    const uint64_t *items0 = L.items0.p, *items1 = L.items1.p, *items2 = L.items2.p;
    {
        KTimer kt(ctx, "lcc_triangles", s);
        if (hc[0])
            hipLaunchKernelGGL(k_lcc_wave<512>, dim3(grid_for((uint64_t)hc[0] * kWave, kLccBlock, 8192)),
                               dim3(kLccBlock), 0, s, O.orp.p, O.ocode.p, O.irp.p, O.icode.p, items0, hc[0], tc);
        GX_TRY(check_launch("k_lcc_wave<512>"));
        if (hc[1])
            hipLaunchKernelGGL(k_lcc_wave<1024>, dim3(grid_for((uint64_t)hc[1] * kWave, kLccBlock, 8192)),
                               dim3(kLccBlock), 0, s, O.orp.p, O.ocode.p, O.irp.p, O.icode.p, items1, hc[1], tc);
        GX_TRY(check_launch("k_lcc_wave<1024>"));
        if (hc[2]) {
            const uint32_t slots = std::max<uint32_t>(64, std::min<uint32_t>(kBlockSlots, [&] {
                uint32_t x = 64;
                while (x < 2 * hc[4]) x <<= 1;
                return x;
            }()));
            if (slots * 8 > 65536)
                GX_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_lcc_block),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(slots * 8)));
            hipLaunchKernelGGL(k_lcc_block, dim3(std::min<uint32_t>(hc[2], 4096)), dim3(kLccBlock),
                               (size_t)slots * 8, s, O.orp.p, O.ocode.p, O.irp.p, O.icode.p, items2, hc[2], slots,
                               tc);
        }
        GX_TRY(check_launch("k_lcc_block"));
        if (hc[3]) {
            for (int32_t u : L.h_big) {
                hipLaunchKernelGGL(k_lcc_merge_in, dim3(64), dim3(kLccBlock), 0, s, O.orp.p, O.ocode.p, O.irp.p,
                                   O.icode.p, u, tc);
                GX_TRY(check_launch("k_lcc_merge_in"));
            }
        }
    }
    return GX_SUCCESS;
}

int lcc_count_range(gx_graph *g, const LccOrient &O, int64_t v0, int64_t v1, unsigned long long *tc,
                    hipStream_t s) {
    LccItems L;
    GX_TRY(lcc_items(O, v0, v1, L, s));
    GX_TRY(lcc_count_items(g, O, L, tc, s));
    GX_HIP_TRY(hipStreamSynchronize(s));   // item lists are freed on return
    return GX_SUCCESS;
}

// What gx_lcc keeps on the graph between calls (gx_graph::lcc), next to the cached closure
// it is derived from: the orientation O, its transpose I and the work items (~2.2 ms of
// sorts, scans and host round trips per call on SYN-cit when rebuilt).
struct LccCache {
    LccOrient O;
    LccItems L;
    DBuf<unsigned long long> tc;
    DBuf<double> out;
    // dense core (GX_LCC_CORE = its largest size; 0: none)
    int32_t K = 0, Kp = 0;
    DBuf<int32_t> coreidx, corev;
    DBuf<int8_t> W, B;
    DBuf<uint8_t> tmask;
    DBuf<unsigned long long> tcore;
};

// The dense core of gx_lcc (k_lcc_core_mfma): the vertices of closure degree above the
// (kmax + 1)-th largest degree, at most kmax of them; their W / B rows and tile mask, and the
// core bit on the in-orientation entries.  Built once with the cached orientation.
int lcc_core_build(gx_graph *g, LccCache &C, int32_t kmax, hipStream_t s) {
    const int64_t n = (int64_t)g->n;
    const DevCSR &S = g->S;
    if (kmax <= 0 || n <= kmax) return GX_SUCCESS;
    int32_t K = 0;
    {
        DBuf<uint32_t> d0, d1;
        DBuf<int32_t> i0, i1;
        GX_TRY(d0.alloc(n));
        GX_TRY(d1.alloc(n));
        GX_TRY(i0.alloc(n));
        GX_TRY(i1.alloc(n));
        hipLaunchKernelGGL(k_core_degkeys, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, S.rp.p, n, d0.p, i0.p);
        GX_TRY(check_launch("k_core_degkeys"));
        GX_TRY(sort_pairs_desc_u32_i32(d0.p, d1.p, i0.p, i1.p, (size_t)n, s));
        std::vector<uint32_t> top((size_t)kmax + 1);
        GX_HIP_TRY(hipMemcpyAsync(top.data(), d1.p, top.size() * 4, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        const uint32_t dcut = top[(size_t)kmax];
        while (K < kmax && top[(size_t)K] > dcut) K++;   // every vertex of degree > dcut: upward closed
        if (K < kCoreWG) return GX_SUCCESS;
        C.K = K;
        C.Kp = (K + kCoreWG - 1) / kCoreWG * kCoreWG;
        GX_TRY(C.coreidx.alloc(n));
        GX_TRY(C.corev.alloc(K));
        GX_HIP_TRY(hipMemsetAsync(C.coreidx.p, 0xff, n * 4, s));
        hipLaunchKernelGGL(k_core_place, dim3(grid_for(K, 256, 1024)), dim3(256), 0, s, i1.p, K, C.coreidx.p, C.corev.p);
        GX_TRY(check_launch("k_core_place"));
        GX_HIP_TRY(hipStreamSynchronize(s));   // the sort buffers are freed at the end of the block
    }
    const int64_t kp = C.Kp, nt = kp / 64;
    GX_TRY(C.W.alloc(kp * kp, 16));
    GX_TRY(C.B.alloc(kp * kp, 16));
    GX_TRY(C.tmask.alloc(nt * nt));
    GX_TRY(C.tcore.alloc(kp));
    GX_HIP_TRY(hipMemsetAsync(C.W.p, 0, kp * kp, s));
    GX_HIP_TRY(hipMemsetAsync(C.B.p, 0, kp * kp, s));
    GX_HIP_TRY(hipMemsetAsync(C.tmask.p, 0, nt * nt, s));
    hipLaunchKernelGGL(k_core_fill, dim3(grid_for((uint64_t)K * kWave, 256, 8192)), dim3(256), 0, s, S.rp.p, S.ci.p,
                       S.flag.p, C.coreidx.p, C.corev.p, K, C.Kp, C.W.p, C.B.p, C.tmask.p);
    GX_TRY(check_launch("k_core_fill"));
    if (C.O.m)
        hipLaunchKernelGGL(k_core_mark_in, dim3(grid_for(C.O.m, 256, 16384)), dim3(256), 0, s, C.O.icode.p, C.O.m,
                           C.coreidx.p);
    GX_TRY(check_launch("k_core_mark_in"));
    GX_HIP_TRY(hipStreamSynchronize(s));
    return GX_SUCCESS;
}

int lcc_core_count(gx_graph *g, LccCache &C, unsigned long long *tc, hipStream_t s) {
    if (!C.K) return GX_SUCCESS;
    KTimer kt(g->ctx, "lcc_core", s);
    GX_HIP_TRY(hipMemsetAsync(C.tcore.p, 0, (size_t)C.Kp * 8, s));
    const int32_t nwg = C.Kp / kCoreWG;
    hipLaunchKernelGGL(k_lcc_core_mfma, dim3((unsigned)nwg * nwg), dim3(256), 0, s, C.W.p, C.B.p, C.tmask.p, C.Kp,
                       C.tcore.p);
    GX_TRY(check_launch("k_lcc_core_mfma"));
    hipLaunchKernelGGL(k_core_final, dim3(grid_for(C.K, 256, 1024)), dim3(256), 0, s, C.tcore.p, C.corev.p, C.K, tc);
    return check_launch("k_core_final");
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_lcc(gx_graph *g, double *lcc) {
    if (!g || !lcc) return fail(GX_NULL_POINTER, "gx_lcc: null argument");
    if (g->n >= (1ull << 29))
        return fail(GX_NOT_IMPLEMENTED, "gx_lcc: more than 2^29 vertices (packed oriented entries)");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    if (n == 0) return GX_SUCCESS;
    GX_TRY(device_begin(ctx));
    GX_TRY(ensure_closure(g));
    auto *C = static_cast<LccCache *>(g->lcc.get());
    if (!C) {
        auto fresh = std::make_shared<LccCache>();
        GX_TRY(lcc_orient(g, fresh->O, s));
        // the dense core (GX_LCC_CORE = its largest size, 0 none), before the items are cut:
        // its in-orientation entries carry the core bit the hash kernels skip
        const char *ce = std::getenv("GX_LCC_CORE");
        GX_TRY(lcc_core_build(g, *fresh, ce ? std::atoi(ce) : 0, s));
        GX_TRY(lcc_items(fresh->O, 0, n, fresh->L, s));
        GX_TRY(fresh->tc.alloc(n));
        GX_TRY(fresh->out.alloc(n));
        g->lcc = fresh;
        C = fresh.get();
    }
    GX_HIP_TRY(hipMemsetAsync(C->tc.p, 0, n * 8, s));
    GX_TRY(lcc_count_items(g, C->O, C->L, C->tc.p, s));
    GX_TRY(lcc_core_count(g, *C, C->tc.p, s));
    hipLaunchKernelGGL(k_lcc_final, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, g->S.rp.p, C->tc.p, n, C->out.p);
    GX_TRY(check_launch("k_lcc_final"));
    GX_TRY(device_end(ctx));
    GX_TRY(download(ctx, lcc, C->out.p, (uint64_t)n, Xfer::Raw64));
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
    if (g->n >= (1ull << 29))
        return fail(GX_NOT_IMPLEMENTED, "gx_lcc_part_create: more than 2^29 vertices (packed oriented entries)");
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
        hipLaunchKernelGGL(k_lcc_work, dim3(grid_for((uint64_t)n * kWave, kLccBlock, 8192)), dim3(kLccBlock), 0, s,
                           part->orient.orp.p, part->orient.irp.p, part->orient.icode.p, n, work.p);
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

GX_MODULE_WARMER(lcc)
