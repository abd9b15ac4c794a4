// gx_cdlp.hip -- community detection by synchronous label propagation (Graphalytics CDLP).
//
// Replaces LAGraph_cdlp (cdlp.cpp:54-67; semantics LAGraph_cdlp.c:37-121) and the fork's
// CUDA_CDLP::LAGraph_cdlp_gpu (cdlp_cuda.cu:118-251, kernels cdlp_kernel.cu:449-1140).
// Every iteration each vertex takes min(argmax_l #neighbour labels == l) over its
// out-neighbours and, for directed graphs, its in-neighbours too (a reciprocal edge counts
// twice, LAGraph_cdlp.c:47-50).  A vertex without neighbours keeps its label.
// Unlike the reference CUDA kernels this is exact and deterministic: counts are built with
// atomics that never lose an update (the reference's LDS insert is unlocked,
// cdlp_kernel.cu:685-694), in-edges are included for directed graphs, and degree-0 vertices
// are written (cdlp_kernel.cu:108-112, 1060-1063).
//   deg <= 32        : one thread per vertex, labels in registers (vote, else a register sort).
//   deg <= 64        : one wave per vertex, labels in registers, counts by ballots.
//   deg <= kLdsHash/2: one wave per vertex, open-addressing hash table in that wave's LDS
//   (kLightSlots slots for deg <= kLightSlots/2, kLdsHash slots above).
//   deg <= 2048      : one 256-thread workgroup per vertex, 4K-slot LDS table (4 per CU).
//   deg <= 4096      : one 512-thread workgroup per vertex, 8K-slot LDS table (2 per CU).
//   deg <= 8192      : one 1024-thread workgroup per vertex, 16K-slot hash table in LDS
//                      (workgroups loop over the medium-vertex list, one per CU).
//   larger           : 4096-label chunks histogrammed in LDS by separate workgroups, merged
//                      into a per-vertex global table (2*deg slots, cleared per iteration),
//                      then one reduce workgroup per vertex.
// The winner is the maximum of the 64-bit key (count << 32) | ~label, i.e. the highest
// count and among equal counts the smallest label.
#include <algorithm>
#include <cstdlib>
#include <memory>
#include <vector>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kCdlpBlock = 256;
constexpr int kLdsHash = 1024;   // slots per wave (8 KiB per wave of int32 key + int32 count)
constexpr int kLightSlots = 256; // slots per wave for light vertices of degree <= 128
constexpr uint32_t kEmpty = 0xffffffffu;

struct CdlpArgs {
    const int64_t *rpA;
    const int32_t *ciA;
    const int64_t *rpT;   // null for undirected graphs
    const int32_t *ciT;
    const int32_t *lab;
    int32_t *nxt;
    int64_t n;
    int *changed;
    int64_t v0, v1;       // vertices updated by this call (the whole graph, or one rank's range)
    // active set (gx_cdlp, from the third iteration): a vertex none of whose neighbours changed
    // label in the previous iteration keeps its label, so only vertices with act[v] == stamp
    // are recomputed, unless *dense (too many changes) or act is null (every vertex)
    const int32_t *act;
    int32_t stamp;
    const int *dense;
    // first iteration of an undirected graph: labels are still the vertex ids, so every label
    // occurs once and the result is the smallest neighbour label (the fork's
    // cdlp_first_iteration_findmin, cdlp_kernel.cu:76-116, without its directed-graph error)
    int first;
    // sparse iteration: k_cdlp_sparse_wave / _group recompute the active vertices of degree
    // <= kMidMax from the lists k_cdlp_mark built, and the tier kernels (the huge ones aside)
    // have nothing to do unless *dense
    int sparse;
    int cshards;   // *changed is cshards words kFlagStride apart (raise_flag_sharded)
    // own-label check of a dense active iteration ran (k_cdlp_keep_*): k_cdlp_tiny recomputes
    // every tiny vertex although the iteration is sparse (null: never)
    const int *keep = nullptr;
    // recount bound (gx_cdlp; null: off): the count of v's label among its neighbour entries is
    // at least vlb[v] - vchg[v] -- vlb the count when v's label was last computed, vchg the
    // changed neighbour entries k_cdlp_mark has counted since
    int32_t *vlb = nullptr;
    int32_t *vchg = nullptr;
    const int *hvalid = nullptr;   // k_cdlp_mark counted every change (the change list was complete)
};

// v's label was computed with at least c occurrences in this iteration's input.
__device__ __forceinline__ void bound_set(const CdlpArgs &a, int64_t v, uint32_t c) {
    if (a.vlb) {
        a.vlb[v] = (int32_t)c;
        a.vchg[v] = 0;
    }
}

// An active iteration whose change list was complete: v's label still holds a strict majority
// (each changed entry lowers its count by at most one), so it is the unique mode and v keeps it.
__device__ __forceinline__ bool bound_keeps(const CdlpArgs &a, int64_t v, int64_t d) {
    return a.vlb && a.sparse && *a.hvalid && 2 * ((int64_t)a.vlb[v] - a.vchg[v]) > d;
}

__device__ __forceinline__ bool tier_idle(const CdlpArgs &a) { return a.sparse && *a.dense == 0; }

__device__ __forceinline__ bool keep_on(const CdlpArgs &a) { return a.keep && *a.keep != 0; }

// Uniform per launch: whether every vertex is recomputed.
__device__ __forceinline__ bool all_active(const CdlpArgs &a) { return !a.act || *a.dense; }

__device__ __forceinline__ bool active(const CdlpArgs &a, bool all, int64_t v) { return all || a.act[v] == a.stamp; }

__device__ __forceinline__ int32_t label_at(const CdlpArgs &a, int64_t ob, int64_t od, int64_t ib,
                                            int64_t k) {
    return k < od ? a.lab[a.ciA[ob + k]] : a.lab[a.ciT[ib + (k - od)]];
}

// Where a vertex's labels come from: out-edges [ob, ob + od) of A, then in-edges [ib, ib + id)
// of A' (directed graphs).
struct VMeta {
    int64_t ob, ib;
    int32_t od, id;
};

__device__ __forceinline__ VMeta vmeta(const CdlpArgs &a, int64_t v) {
    VMeta m;
    m.ob = a.rpA[v];
    m.od = (int32_t)(a.rpA[v + 1] - m.ob);
    m.ib = 0;
    m.id = 0;
    if (a.rpT) {
        m.ib = a.rpT[v];
        m.id = (int32_t)(a.rpT[v + 1] - m.ib);
    }
    return m;
}

// An inactive vertex reads as degree 0 (no label loads; it keeps its label).
__device__ __forceinline__ VMeta vmeta_act(const CdlpArgs &a, bool all, int64_t v) {
    if (active(a, all, v)) return vmeta(a, v);
    VMeta m;
    m.ob = m.ib = 0;
    m.od = m.id = 0;
    return m;
}

__device__ __forceinline__ int32_t col_at(const CdlpArgs &a, const VMeta &m, int64_t k) {
    return k < m.od ? a.ciA[m.ob + k] : a.ciT[m.ib + (k - m.od)];
}

// Where label k of a vertex is read: an index into lsrc(a), the label array (through the column).
__device__ __forceinline__ int64_t src_at(const CdlpArgs &a, const VMeta &m, int64_t k) { return col_at(a, m, k); }

__device__ __forceinline__ const int32_t *lsrc(const CdlpArgs &a) { return a.lab; }

__device__ __forceinline__ uint32_t hash_slot(uint32_t l, int log2ts) {
    return (l * 2654435761u) >> (32 - log2ts);
}

// Adds `c` occurrences of label l to an open-addressing LDS table of 2^log2ts slots.
__device__ __forceinline__ void lds_table_add(uint32_t *K, uint32_t *C, uint32_t l, uint32_t c, int log2ts) {
    const uint32_t mask = (1u << log2ts) - 1u;
    uint32_t h = hash_slot(l, log2ts);
    for (;;) {
        const uint32_t prev = atomicCAS(&K[h], kEmpty, l);
        if (prev == kEmpty || prev == l) {
            atomicAdd(&C[h], c);
            return;
        }
        h = (h + 1) & mask;
    }
}

// Wave-uniform call (every lane of the wave reaches it; `valid` marks lanes holding a label).
// In each of kPeel rounds, the lanes whose label equals the first remaining lane's go in as
// one add of their count. The wave's most repeated labels - the common case once CDLP's labels
// start to agree - then do not serialise up to 64 same-address LDS atomics. The other lanes
// insert one at a time.
template <int kPeel = 1>
__device__ __forceinline__ void lds_table_add_wave(uint32_t *K, uint32_t *C, uint32_t l, bool valid, int log2ts) {
    const int lane = (int)(threadIdx.x & (kWave - 1));
#pragma unroll
    for (int r = 0; r < kPeel; r++) {
        const unsigned long long act = __ballot(valid);
        if (!act) return;
        const int first = __ffsll((long long)act) - 1;
        const uint32_t lead = __shfl(l, first, kWave);
        const bool same = valid && l == lead;
        const unsigned long long grp = __ballot(same);
        if (lane == first) lds_table_add(K, C, lead, (uint32_t)__popcll(grp), log2ts);
        valid = valid && !same;
    }
    if (valid) lds_table_add(K, C, l, 1u, log2ts);
}

__device__ __forceinline__ unsigned long long pack(uint32_t count, uint32_t label) {
    return ((unsigned long long)count << 32) | (unsigned long long)(kEmpty - label);
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        unsigned long long o = __shfl_xor(v, off, kWave);
        v = o > v ? o : v;
    }
    return v;
}

// ---- strict-majority fast path -------------------------------------------------------
// A label held by more than half of a vertex's d neighbours is its unique most frequent
// label, so it is the CDLP result whatever the tie rule.  Boyer-Moore voting finds the only
// possible candidate in one pass; pairwise merges of (candidate, count) in any order keep it
// (each merge cancels pairs of different labels); counting the candidate exactly then
// decides.  Once CDLP labels settle, almost every vertex has such a label (SYN-7_5 from the
// third iteration on: every vertex of degree > 16, 61 % of those <= 16), and the hash table,
// the shuffle counts or the register compares are skipped.
struct Vote {
    uint32_t c;   // candidate label (kEmpty: none)
    uint32_t n;   // surplus
};

__device__ __forceinline__ Vote vote_add(Vote v, uint32_t l, bool valid) {
    if (!valid) return v;
    if (v.n == 0) return {l, 1u};
    return v.c == l ? Vote{v.c, v.n + 1u} : Vote{v.c, v.n - 1u};
}

__device__ __forceinline__ Vote vote_merge(Vote a, Vote b) {
    if (a.c == b.c) return {a.c, a.n + b.n};
    return a.n >= b.n ? Vote{a.c, a.n - b.n} : Vote{b.c, b.n - a.n};
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor(v, off, kWave));
    return v;
}

// Merge down to lane 0 (xor butterflies would leave different candidates in different lanes).
__device__ __forceinline__ Vote wave_vote(Vote v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        Vote o;
        o.c = __shfl_down(v.c, off, kWave);
        o.n = __shfl_down(v.n, off, kWave);
        v = vote_merge(v, o);
    }
    return v;
}

// Tiny vertices (deg <= kTiny, including isolated ones): one THREAD per vertex, labels in
// registers (all loads in flight), 64 vertices per wave instead of one (two thirds of the
// vertices of a power-law graph have degree <= 8, 84 % of SYN-7_5's <= 32).  The strict-
// majority vote first; else the labels are sorted in registers (a bitonic network, unrolled)
// and the longest run wins, the first one (smallest label) among equal runs.
constexpr int kTiny = 32;

__device__ __forceinline__ void sort_regs(uint32_t (&L)[kTiny]) {
#pragma unroll
    for (int k = 2; k <= kTiny; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < kTiny; i++) {
                const int l = i ^ j;
                if (l > i) {
                    const uint32_t x = L[i], y = L[l];
                    const bool up = (i & k) == 0;
                    L[i] = up ? min(x, y) : max(x, y);
                    L[l] = up ? max(x, y) : min(x, y);
                }
            }
}

__global__ __launch_bounds__(kCdlpBlock) void k_cdlp_tiny(CdlpArgs a) {
    const bool kp = keep_on(a);
    if (tier_idle(a) && !kp) return;
    bool any = false;
    const bool all = all_active(a) || kp;
    for (int64_t v = a.v0 + (int64_t)blockIdx.x * kCdlpBlock + threadIdx.x; v < a.v1;
         v += (int64_t)gridDim.x * kCdlpBlock) {
        const int64_t ob = a.rpA[v], od = a.rpA[v + 1] - ob;
        int64_t ib = 0, id = 0;
        if (a.rpT) {
            ib = a.rpT[v];
            id = a.rpT[v + 1] - ib;
        }
        const int64_t d = od + id;
        if (d > kTiny) continue;
        const int32_t old = a.lab[v];
        int32_t best = old;
        if (d > 0 && active(a, all, v)) {
            uint32_t L[kTiny];
#pragma unroll
            for (int k = 0; k < kTiny; k++) L[k] = k < d ? (uint32_t)label_at(a, ob, od, ib, k) : kEmpty;
            Vote vt{kEmpty, 0u};
#pragma unroll
            for (int k = 0; k < kTiny; k++) vt = vote_add(vt, L[k], k < d);
            uint32_t nc = 0;
#pragma unroll
            for (int k = 0; k < kTiny; k++) nc += (k < d && L[k] == vt.c) ? 1u : 0u;
            uint32_t cnt = 0;   // the winner's count (the recount bound)
            if (a.first) {
                uint32_t mn = kEmpty;
#pragma unroll
                for (int k = 0; k < kTiny; k++) mn = min(mn, L[k]);   // padding is kEmpty
                best = (int32_t)mn;
            } else if (2 * (int64_t)nc > d) {
                best = (int32_t)vt.c;   // strict majority
                cnt = nc;
            } else {
                sort_regs(L);           // labels ascending, the padding last
                uint32_t bc = 0, bl = kEmpty, run = 0, prev = kEmpty;
#pragma unroll
                for (int k = 0; k < kTiny; k++) {
                    run = L[k] == prev ? run + 1u : 1u;
                    prev = L[k];
                    if (k < d && run > bc) {
                        bc = run;
                        bl = L[k];
                    }
                }
                best = (int32_t)bl;
                cnt = bc;
            }
            bound_set(a, v, cnt);
        }
        a.nxt[v] = best;
        any |= best != old;
    }
    if (__ballot(any) && (threadIdx.x & (kWave - 1)) == 0) raise_flag_sharded(a.changed, a.cshards);
}

// Small vertices (kTiny < deg <= 64), from a list: one wave per vertex, labels in registers,
// counts by shuffles; no LDS, so the kernel runs at full occupancy.
__global__ __launch_bounds__(kCdlpBlock) void k_cdlp_small(CdlpArgs a, const int32_t *__restrict__ sv,
                                                           int32_t nsmall) {
    if (tier_idle(a)) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t gw = ((int64_t)blockIdx.x * kCdlpBlock + threadIdx.x) / kWave;
    const int64_t nw = (int64_t)gridDim.x * (kCdlpBlock / kWave);
    bool any = false;
    const bool all = all_active(a);
    for (int64_t i = gw; i < nsmall; i += nw) {
        const int64_t v = sv[i];
        const VMeta m = vmeta_act(a, all, v);
        const int64_t ob = m.ob, od = m.od, ib = m.ib, id = m.id;
        const int64_t d = od + id;
        const int32_t old = a.lab[v];
        const uint32_t my = lane < d ? (uint32_t)label_at(a, ob, od, ib, lane) : kEmpty;
        const uint32_t cand = __shfl(wave_vote(Vote{my, lane < d ? 1u : 0u}).c, 0, kWave);
        int32_t best;
        uint32_t cnt = 0;   // the winner's count (the recount bound)
        const uint32_t ncand = (uint32_t)__popcll(__ballot(lane < d && my == cand));
        if (d == 0) {
            best = old;   // inactive (or isolated)
        } else if (a.first) {
            best = (int32_t)wave_min_u32(my);
        } else if (2 * (int64_t)ncand > d) {
            best = (int32_t)cand;   // strict majority
            cnt = ncand;
        } else {
            // one round per distinct label: the first remaining lane's label, its lanes by one
            // ballot (lane reads, no LDS; the d shuffles this replaces were ds_bpermute each)
            unsigned long long rem = __ballot(lane < d);
            uint32_t bc = 0, bl = kEmpty;
            while (rem) {
                const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)my, __ffsll((long long)rem) - 1);
                const unsigned long long eq = __ballot(my == l) & rem;
                const uint32_t c = (uint32_t)__popcll(eq);
                if (c > bc || (c == bc && l < bl)) {
                    bc = c;
                    bl = l;
                }
                rem &= ~eq;
            }
            best = (int32_t)bl;
            cnt = bc;
        }
        if (lane == 0) {
            a.nxt[v] = best;
            any |= best != old;
            if (d > 0) bound_set(a, v, cnt);
        }
    }
    if (any) raise_flag_sharded(a.changed, a.cshards);
}

// Light vertices (64 < deg <= kSlots/2), from a list: one wave per vertex, an LDS hash table of
// 2 deg slots per wave.  Two instances: kLightSlots for deg <= kLightSlots/2 (2 KiB per wave,
// so LDS does not cap occupancy) and kLdsHash for the rest.
template <int kSlots>
__global__ __launch_bounds__(kCdlpBlock) void k_cdlp_light(CdlpArgs a, const int32_t *__restrict__ lv,
                                                           int32_t nlight) {
    if (tier_idle(a)) return;
    __shared__ uint32_t keys[kCdlpBlock / kWave][kSlots];
    __shared__ uint32_t cnts[kCdlpBlock / kWave][kSlots];
    constexpr int R = kSlots / (2 * kWave);   // label rounds of the largest vertex of the tier
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    uint32_t *K = keys[wv];
    uint32_t *C = cnts[wv];
    const int64_t nw = (int64_t)gridDim.x * (kCdlpBlock / kWave);
    int64_t i = ((int64_t)blockIdx.x * kCdlpBlock + threadIdx.x) / kWave;
    if (i >= nlight) return;
    bool any = false;
    const bool all = all_active(a);
    // software-pipelined over the wave's vertices like k_cdlp_mid: the next vertex's
    // dependent loads are issued one link at a time between this vertex's LDS phases
    int64_t v = lv[i];
    VMeta m = vmeta_act(a, all, v);
    uint32_t L[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t k = (int64_t)r * kWave + lane;
        L[r] = k < (int64_t)m.od + m.id ? (uint32_t)lsrc(a)[src_at(a, m, k)] : kEmpty;
    }
    for (;;) {
        const int64_t d = (int64_t)m.od + m.id;
        const int64_t inext = i + nw;
        const bool more = inext < nlight;
        const int64_t vn = more ? (int64_t)lv[inext] : v;      // next vertex, link 1
        const int32_t old = a.lab[v];
        // strict-majority fast path (a wave-uniform branch)
        Vote vt{kEmpty, 0u};
#pragma unroll
        for (int r = 0; r < R; r++) vt = vote_add(vt, L[r], (int64_t)r * kWave + lane < d);
        uint32_t cand = __shfl(wave_vote(vt).c, 0, kWave);
        int64_t nc = 0;
#pragma unroll
        for (int r = 0; r < R; r++)
            if ((int64_t)r * kWave < d) nc += __popcll(__ballot((int64_t)r * kWave + lane < d && L[r] == cand));
        if (a.first) {
            uint32_t mn = kEmpty;
#pragma unroll
            for (int r = 0; r < R; r++) mn = (int64_t)r * kWave + lane < d ? min(mn, L[r]) : mn;
            cand = wave_min_u32(mn);
        }
        const bool maj = 2 * nc > d || a.first || d == 0;   // d == 0: inactive, keeps its label
        int log2ts = 1;
        while ((1ll << log2ts) < 2 * d) log2ts++;
        const int ts = 1 << log2ts;
        if (!maj) {
            for (int s = lane; s < ts; s += kWave) {
                K[s] = kEmpty;
                C[s] = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const VMeta mn = vmeta_act(a, all, vn);                 // link 2
        const int64_t dn = more ? (int64_t)mn.od + mn.id : 0;
        if (!maj) {
#pragma unroll
            for (int r = 0; r < R; r++)
                if ((int64_t)r * kWave < d) lds_table_add_wave(K, C, L[r], (int64_t)r * kWave + lane < d, log2ts);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        int64_t cn[R];                                          // link 3
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int64_t k = (int64_t)r * kWave + lane;
            cn[r] = k < dn ? src_at(a, mn, k) : -1;
        }
        unsigned long long key = 0;
        if (!maj) {
            for (int s = lane; s < ts; s += kWave) {
                const uint32_t c = C[s];
                if (c) {
                    const unsigned long long kk = pack(c, K[s]);
                    key = kk > key ? kk : key;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) L[r] = cn[r] >= 0 ? (uint32_t)lsrc(a)[cn[r]] : kEmpty;   // link 4
        const unsigned long long wk = maj ? 0ull : wave_max_u64(key);
        const int32_t best = d == 0 ? old : maj ? (int32_t)cand : (int32_t)(kEmpty - (uint32_t)(wk & 0xffffffffu));
        // the winner's count (the recount bound; 0 for the first iteration's minimum)
        const uint32_t cnt = a.first ? 0u : maj ? (uint32_t)nc : (uint32_t)(wk >> 32);
        if (!maj) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (lane == 0) {
            a.nxt[v] = best;
            any |= best != old;
            if (d > 0) bound_set(a, v, cnt);
        }
        if (!more) break;
        i = inext;
        v = vn;
        m = mn;
    }
    if (any) raise_flag_sharded(a.changed, a.cshards);
}

// Huge vertices (deg > kMidMax): the label multiset is cut into kHugeChunk-label chunks; a
// 1024-thread workgroup histograms one chunk in a 64 KiB LDS table, then adds each distinct
// label once into the vertex's global table, so global atomics scale with distinct labels per
// chunk, not with the degree.  A global slot is one 64-bit word, (epoch << 58) | (count << 31) |
// label, claimed and counted by one CAS: a slot whose epoch is not this iteration's is empty, so
// the tables are never cleared (but once every kHugeEpochs iterations) and never scanned.  Every
// successful CAS knows the label's count so far; a label's last update carries its final count,
// so the maximum of (count << 32) | ~label over the updates is the vertex's winner.  Each
// workgroup folds its updates into one 64-bit atomicMax on the vertex's key.
constexpr int kHugeBlock = 1024;
constexpr int kHugeChunk = 4096;
constexpr int kHugeSlots = 2 * kHugeChunk;
constexpr int kHugeEpochs = 63;                   // epochs 1..63 in the top 6 bits; 0: never used
constexpr int64_t kHugeMaxDeg = (1ll << 27) - 1;  // the count field (bits 31..57)

__global__ __launch_bounds__(kHugeBlock) void k_cdlp_huge_insert(CdlpArgs a, const int32_t *__restrict__ hv,
                                                                 const int64_t *__restrict__ hoff,
                                                                 const int32_t *__restrict__ hlog2,
                                                                 const int32_t *__restrict__ cvert,
                                                                 const int64_t *__restrict__ cbeg,
                                                                 unsigned long long *gtab, uint32_t epoch,
                                                                 unsigned long long *vkey) {
    __shared__ uint32_t K[kHugeSlots];
    __shared__ uint32_t C[kHugeSlots];
    __shared__ unsigned long long red[kHugeBlock / kWave];
    constexpr int kLog2 = 13;   // log2(kHugeSlots)
    const int tid = threadIdx.x;
    const int32_t hi = cvert[blockIdx.x];
    const int64_t v = hv[hi];
    if (!active(a, all_active(a), v)) return;
    const int64_t ob = a.rpA[v], od = a.rpA[v + 1] - ob;
    int64_t ib = 0, id = 0;
    if (a.rpT) {
        ib = a.rpT[v];
        id = a.rpT[v + 1] - ib;
    }
    // the recount bound: a vertex whose label provably keeps a strict majority skips the
    // recount (every chunk of the vertex decides alike)
    if (bound_keeps(a, v, od + id)) return;
    const int64_t k0 = cbeg[blockIdx.x], k1 = min(k0 + kHugeChunk, od + id);
    for (int s = tid; s < kHugeSlots; s += kHugeBlock) {
        K[s] = kEmpty;
        C[s] = 0;
    }
    __syncthreads();
    constexpr int R = kHugeChunk / kHugeBlock;   // the chunk's gathers all in flight first
    uint32_t L[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t k = k0 + (int64_t)r * kHugeBlock + tid;
        L[r] = k < k1 ? (uint32_t)label_at(a, ob, od, ib, k) : kEmpty;
    }
    if (a.first) {   // the chunk's smallest label, as a count-1 key (no tables)
        uint32_t mn = kEmpty;
#pragma unroll
        for (int r = 0; r < R; r++) mn = k0 + (int64_t)r * kHugeBlock + tid < k1 ? min(mn, L[r]) : mn;
        mn = wave_min_u32(mn);
        if ((tid & (kWave - 1)) == 0 && mn != kEmpty) atomicMax(&vkey[hi], pack(1u, mn));
        return;
    }
#pragma unroll
    for (int r = 0; r < R; r++)
        if (k0 + (int64_t)r * kHugeBlock < k1) lds_table_add_wave(K, C, L[r], k0 + (int64_t)r * kHugeBlock + tid < k1, kLog2);
    __syncthreads();
    const int log2ts = hlog2[hi];
    const int64_t ts = 1ll << log2ts;
    unsigned long long *GT = gtab + hoff[hi];
    const unsigned long long ep = (unsigned long long)epoch << 58;
    unsigned long long key = 0;
    for (int s = tid; s < kHugeSlots; s += kHugeBlock) {
        const uint32_t c = C[s];
        if (!c) continue;
        const uint32_t l = K[s];
        int64_t h = hash_slot(l, log2ts);
        unsigned long long old = GT[h];   // a stale copy only costs a failed CAS
        for (;;) {
            const bool live = (old & (63ull << 58)) == ep;
            if (live && (uint32_t)(old & 0x7fffffffu) != l) {   // another label's slot: probe on
                h = (h + 1) & (ts - 1);
                old = GT[h];
                continue;
            }
            const unsigned long long nw = live ? old + ((unsigned long long)c << 31)
                                               : ep | ((unsigned long long)c << 31) | (unsigned long long)l;
            const unsigned long long prev = atomicCAS(&GT[h], old, nw);
            if (prev == old) {
                const unsigned long long kk = pack((uint32_t)((nw >> 31) & kHugeMaxDeg), l);
                key = kk > key ? kk : key;
                break;
            }
            old = prev;
        }
    }
    key = wave_max_u64(key);
    if ((tid & (kWave - 1)) == 0) red[tid / kWave] = key;
    __syncthreads();
    if (tid == 0) {
        unsigned long long m = red[0];
        for (int w = 1; w < kHugeBlock / kWave; w++) m = red[w] > m ? red[w] : m;
        if (m) atomicMax(&vkey[hi], m);
    }
}

__global__ void k_cdlp_huge_final(CdlpArgs a, const int32_t *__restrict__ hv, int32_t nhuge,
                                  unsigned long long *vkey) {
    for (int32_t hi = blockIdx.x * blockDim.x + threadIdx.x; hi < nhuge; hi += gridDim.x * blockDim.x) {
        const int64_t v = hv[hi];
        // recomputed (a key), or inactive / kept by the majority bound (its label stays)
        const unsigned long long k = vkey[hi];
        const int32_t best = k ? (int32_t)(kEmpty - (uint32_t)(k & 0xffffffffu)) : a.lab[v];
        if (k) bound_set(a, v, a.first ? 0u : (uint32_t)(k >> 32));
        vkey[hi] = 0;   // clean for the next iteration
        a.nxt[v] = best;
        if (best != a.lab[v]) raise_flag_sharded(a.changed, a.cshards);
    }
}

__global__ void k_cdlp_fill_u32(uint32_t *p, uint32_t v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// Medium-tier shapes (k_cdlp_mid below): 1024 threads / 16K slots (128 KiB, one workgroup
// per CU) for deg <= 8192, 512 / 8K for deg <= 4096 and 256 / 4K (32 KiB, four workgroups per
// CU) for deg <= 2048, which keeps four vertices in flight per CU for the many mid vertices
// near the bottom of the range.
constexpr int kMidBlock = 1024;
constexpr int kMidSlots = 16384;
constexpr int64_t kMidMax = kMidSlots / 2;
constexpr int kMid2Block = 256;
constexpr int kMid2Slots = 4096;
constexpr int64_t kMid2Max = kMid2Slots / 2;
constexpr int kMid4Block = 512;   // deg <= 4096: 8K slots (64 KiB), two workgroups per CU
constexpr int kMid4Slots = 8192;
constexpr int64_t kMid4Max = kMid4Slots / 2;

// Medium vertices (kLdsHash/2 < deg <= kMidSlots/2): one workgroup per vertex with a
// kMidSlots-slot hash table in LDS; workgroups loop over the medium-vertex list so the table
// is reused without a relaunch.  Three sizes (kMid2 / kMid4 / kMid): 256 threads, 4K slots,
// 4 per CU; 512, 8K, 2 per CU; 1024, 16K, 1 per CU.
// Software-pipelined over the list: a vertex's labels sit at the end of a chain of dependent
// loads (list -> row pointers -> column ids -> labels, ~1 us each), so the next vertex's chain
// is issued one link at a time between the current vertex's LDS phases (clear, insert, scan):
// each load's wait lands after the LDS work that follows its issue.
template <int kMidBlock, int kMidSlots>
__global__ __launch_bounds__(kMidBlock) void k_cdlp_mid(CdlpArgs a, const int32_t *__restrict__ mv, int32_t nmid) {
    if (tier_idle(a)) return;
    __shared__ uint32_t K[kMidSlots];
    __shared__ uint32_t C[kMidSlots];
    __shared__ unsigned long long red[kMidBlock / kWave];
    __shared__ uint32_t cnt[kMidBlock / kWave];
    __shared__ uint32_t bcast[1];
    constexpr int R = kMidSlots / (2 * kMidBlock);
    const int tid = threadIdx.x;
    bool any = false;
    int32_t i = blockIdx.x;
    if (i >= nmid) return;
    const bool all = all_active(a);
    int64_t v = mv[i];
    VMeta m = vmeta_act(a, all, v);
    uint32_t L[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t k = (int64_t)r * kMidBlock + tid;
        L[r] = k < (int64_t)m.od + m.id ? (uint32_t)lsrc(a)[src_at(a, m, k)] : kEmpty;
    }
    for (;;) {
        const int64_t d = (int64_t)m.od + m.id;
        const int32_t inext = i + (int32_t)gridDim.x;
        const bool more = inext < nmid;
        // link 1 of the next vertex: its id
        const int64_t vn = more ? (int64_t)mv[inext] : v;
        // strict-majority fast path: the workgroup's candidate, then its exact count (the
        // first iteration of an undirected graph: the smallest label).  d, a.first and so the
        // branches are the same in every thread; an inactive vertex (d == 0) skips it all.
        uint32_t cand = kEmpty;
        bool maj = true;
        uint32_t ccount = 0;   // the candidate's count (the recount bound; 0 in the first iteration)
        if (d > 0 && a.first) {
            uint32_t mn = kEmpty;
#pragma unroll
            for (int r = 0; r < R; r++) mn = (int64_t)r * kMidBlock + tid < d ? min(mn, L[r]) : mn;
            mn = wave_min_u32(mn);
            if ((tid & (kWave - 1)) == 0) cnt[tid / kWave] = mn;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kMidBlock / kWave; j++) cand = min(cand, cnt[j]);
        } else if (d > 0) {
            Vote vt{kEmpty, 0u};
#pragma unroll
            for (int r = 0; r < R; r++) vt = vote_add(vt, L[r], (int64_t)r * kMidBlock + tid < d);
            vt = wave_vote(vt);
            if ((tid & (kWave - 1)) == 0) red[tid / kWave] = ((unsigned long long)vt.c << 32) | vt.n;
            __syncthreads();
            if (tid == 0) {
                Vote w{(uint32_t)(red[0] >> 32), (uint32_t)red[0]};
                for (int j = 1; j < kMidBlock / kWave; j++) w = vote_merge(w, Vote{(uint32_t)(red[j] >> 32), (uint32_t)red[j]});
                bcast[0] = w.c;
            }
            __syncthreads();
            cand = bcast[0];
            uint32_t mc = 0;
#pragma unroll
            for (int r = 0; r < R; r++) mc += ((int64_t)r * kMidBlock + tid < d && L[r] == cand) ? 1u : 0u;
            mc = wave_sum_u32(mc);
            if ((tid & (kWave - 1)) == 0) cnt[tid / kWave] = mc;
            __syncthreads();
            uint32_t nc = 0;
#pragma unroll
            for (int j = 0; j < kMidBlock / kWave; j++) nc += cnt[j];
            maj = 2 * (int64_t)nc > d;
            ccount = nc;
        }
        int log2ts = 1;
        while ((1ll << log2ts) < 2 * d) log2ts++;
        const int ts = 1 << log2ts;
        if (!maj) {
            for (int s = tid; s < ts; s += kMidBlock) {
                K[s] = kEmpty;
                C[s] = 0;
            }
            __syncthreads();
        }
        // link 2: its row pointers
        const VMeta mn = vmeta_act(a, all, vn);
        const int64_t dn = more ? (int64_t)mn.od + mn.id : 0;
        if (!maj) {
#pragma unroll
            for (int r = 0; r < R; r++)
                if ((int64_t)r * kMidBlock < d) lds_table_add_wave(K, C, L[r], (int64_t)r * kMidBlock + tid < d, log2ts);
            __syncthreads();
        }
        // link 3: its column ids
        int64_t cn[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int64_t k = (int64_t)r * kMidBlock + tid;
            cn[r] = k < dn ? src_at(a, mn, k) : -1;
        }
        unsigned long long key = 0;
        if (!maj) {
            for (int s = tid; s < ts; s += kMidBlock) {
                const uint32_t c = C[s];
                if (c) {
                    const unsigned long long kk = pack(c, K[s]);
                    key = kk > key ? kk : key;
                }
            }
        }
        // link 4: its labels
#pragma unroll
        for (int r = 0; r < R; r++) L[r] = cn[r] >= 0 ? (uint32_t)lsrc(a)[cn[r]] : kEmpty;
        if (maj) {
            if (tid == 0) {
                const int32_t best = d == 0 ? a.lab[v] : (int32_t)cand;
                a.nxt[v] = best;
                any |= best != a.lab[v];
                if (d > 0) bound_set(a, v, ccount);
            }
        } else {
            key = wave_max_u64(key);
            if ((tid & (kWave - 1)) == 0) red[tid / kWave] = key;
            __syncthreads();
            if (tid == 0) {
                unsigned long long mx = red[0];
                for (int w = 1; w < kMidBlock / kWave; w++) mx = red[w] > mx ? red[w] : mx;
                const int32_t best = (int32_t)(kEmpty - (uint32_t)(mx & 0xffffffffu));
                a.nxt[v] = best;
                any |= best != a.lab[v];
                bound_set(a, v, (uint32_t)(mx >> 32));
            }
        }
        if (d > 0) __syncthreads();   // red / cnt / bcast and the table are free for the next vertex
        if (!more) break;
        i = inext;
        v = vn;
        m = mn;
    }
    if (any) raise_flag_sharded(a.changed, a.cshards);
}

// The iteration's changed flag to pinned host memory: one lane's store over PCIe, instead of a
// 4-byte hipMemcpyAsync, which ran as a ~40 us blit kernel (profiles/r01_cdlp_kernel_stats.csv).
// Bit 0: a label changed; bit 1: the iteration's active set overflowed (*dense).
__global__ void k_cdlp_flag_out(const int *__restrict__ changed, int shards, const int *dense, int *hflag) {
    const int t = threadIdx.x;   // one lane per shard (shards <= kWave)
    const bool set = t < shards && changed[t * kFlagStride] != 0;
    const bool any = __ballot(set) != 0;
    if (t == 0) *hflag = (any ? 1 : 0) | (dense && *dense ? 2 : 0);
}

// Active set of the next iteration (gx_cdlp).  k_cdlp_changed lists the vertices whose label
// changed in the last iteration (prev != cur), as chunks of kMarkChunk neighbours, and sets
// prev = cur for them: prev (the buffer the iteration writes) then equals cur everywhere, so
// a sparse iteration writes only its active vertices.  k_cdlp_mark gives every in- and
// out-neighbour in a listed chunk act = stamp and appends each newly marked vertex of degree
// <= kMidMax to one of three lists by degree (<= 512, <= 2048, <= 8192), which
// k_cdlp_sparse_wave / k_cdlp_sparse_group recompute; huge vertices keep their tier kernels,
// which skip inactive ones.  SYN-7_5 from the fifth iteration on: ~500 changes and ~780 active
// vertices (3 % of the entries).
// Every list is kCdlpSubs shards with a counter each, the counters kCntStride words apart:
// device-scope atomics on one address serialise (one counter for all: ~23 K wave atomics,
// ~700 us on SYN-cit), and so do counters that share a 128-byte line.  An overflowing shard
// sets *dense, and the tier kernels recompute every vertex.
// Shard j of a list is read by the waves (workgroups) w with w % kCdlpSubs == j: every
// shard gets the same share of the grid (a whole-grid sweep of each shard in turn left all
// but a few waves idle and cost a dependent-load chain per shard: ~120 us on SYN-7_5).
constexpr int kCdlpSubs = 256;
constexpr int kCntStride = 32;             // 128 bytes between two counters
constexpr int kCdlpLists = 4;              // change chunks, then the three activation lists
constexpr int64_t kMarkChunk = 2048;
constexpr int64_t kSparseWaveMax = 512;    // wave per vertex, 1024-slot tables
constexpr int64_t kSparseG2Max = kMid2Max; // 256-thread workgroup, 4K slots
// the rest up to kMidMax: 1024-thread workgroup, 16K slots

__device__ __forceinline__ int64_t cdlp_degree(const int64_t *rpA, const int64_t *rpT, int64_t v) {
    int64_t d = rpA[v + 1] - rpA[v];
    if (rpT) d += rpT[v + 1] - rpT[v];
    return d;
}

__device__ __forceinline__ unsigned int shard_count(const unsigned int *count, int j, int64_t cap) {
    return (unsigned int)min((int64_t)count[j * kCntStride], cap);
}

// One reservation per workgroup and 256 vertices.
__global__ __launch_bounds__(256) void k_cdlp_changed(int32_t *__restrict__ prev, const int32_t *__restrict__ cur,
                                                      const int64_t *__restrict__ rpA, const int64_t *__restrict__ rpT,
                                                      int64_t n, uint64_t *list, int64_t sub, unsigned int *count,
                                                      int *dense) {
    __shared__ uint32_t wtot[256 / kWave];
    __shared__ uint32_t bbase;
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    if (blockIdx.x == 0 && threadIdx.x == 0) *dense = 0;   // k_cdlp_mark only ever raises it
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < n; b0 += (int64_t)gridDim.x * 256) {
        const int64_t v = b0 + threadIdx.x;
        const int32_t cv = v < n ? cur[v] : 0;
        const bool ch = v < n && prev[v] != cv;
        if (ch) prev[v] = cv;
        const uint32_t chunks = ch ? (uint32_t)((cdlp_degree(rpA, rpT, v) + kMarkChunk - 1) / kMarkChunk) : 0u;
        uint32_t pre = chunks;   // inclusive prefix within the wave
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const uint32_t t = __shfl_up(pre, off, kWave);
            if (lane >= off) pre += t;
        }
        if (lane == kWave - 1) wtot[wv] = pre;
        pre -= chunks;
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 256 / kWave; w++) {
            const uint32_t t = wtot[w];
            before += w < wv ? t : 0u;
            total += t;
        }
        if (total) {
            if (threadIdx.x == 0) {
                const int j = (int)((b0 / 256) % kCdlpSubs);
                unsigned int *cnt = count + j * kCntStride;
                // past capacity only the overflow matters: stop adding
                unsigned int base = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (base <= (unsigned int)sub) base = atomicAdd(cnt, total);
                bbase = base;
            }
            __syncthreads();
            const unsigned int base = bbase + before + pre;
            const int j = (int)((b0 / 256) % kCdlpSubs);
            for (uint32_t c = 0; c < chunks; c++)
                if (base + c < (unsigned int)sub) list[(int64_t)j * sub + base + c] = ((uint64_t)v << 32) | c;
        }
        __syncthreads();   // wtot and bbase are free again
    }
}

// One wave per listed chunk; appends go to shard (wave index mod kCdlpSubs) of their list, one
// reservation per wave, list and 64 neighbours.
__global__ __launch_bounds__(256) void k_cdlp_mark(const int64_t *__restrict__ rpA, const int32_t *__restrict__ ciA,
                                                   const int64_t *__restrict__ rpT, const int32_t *__restrict__ ciT,
                                                   const uint64_t *__restrict__ list, int64_t sub,
                                                   unsigned int *counts, int32_t *act, int32_t stamp, int *dense,
                                                   int32_t *al, int64_t asub, int32_t *vchg, int *hvalid) {
    __shared__ int over;
    if (threadIdx.x == 0) over = 0;
    __syncthreads();
    if (counts[threadIdx.x * kCntStride] > (unsigned int)sub) over = 1;   // kCdlpSubs == blockDim.x
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0 && hvalid) *hvalid = over ? 0 : 1;
    if (over) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *dense = 1;
        return;
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave;
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);   // a multiple of kCdlpSubs
    const int j = (int)(gw % kCdlpSubs);
    const int64_t c = counts[j * kCntStride];
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int64_t i = gw / kCdlpSubs; i < c; i += nw / kCdlpSubs) {
        const uint64_t e = list[(int64_t)j * sub + i];
        const int64_t u = (int64_t)(e >> 32);
        const int64_t ob = rpA[u], od = rpA[u + 1] - ob;
        const int64_t ib = rpT ? rpT[u] : 0, id = rpT ? rpT[u + 1] - ib : 0;
        const int64_t k0 = (int64_t)(uint32_t)e * kMarkChunk, k1 = min(k0 + kMarkChunk, od + id);
        for (int64_t kb = k0; kb < k1; kb += kWave) {
            const int64_t k = kb + lane;
            int64_t w = -1;
            if (k < k1) w = k < od ? ciA[ob + k] : ciT[ib + (k - od)];
            const bool fresh = w >= 0 && atomicExch(&act[w], stamp) != stamp;
            // the recount bound: every changed neighbour entry of w
            if (vchg && w >= 0) atomicAdd(&vchg[w], 1);
            const int64_t dw = fresh ? cdlp_degree(rpA, rpT, w) : 0;
            // activation list 1 + L: L = 0 (wave), 1 (256-thread group), 2 (1024-thread group)
            const int L = !fresh || dw > kMidMax ? -1 : dw <= kSparseWaveMax ? 0 : dw <= kSparseG2Max ? 1 : 2;
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const unsigned long long m = __ballot(L == q);
                if (!m) continue;
                unsigned int b = 0;
                if (lane == 0) b = atomicAdd(&counts[((1 + q) * kCdlpSubs + j) * kCntStride], (unsigned int)__popcll(m));
                b = __shfl(b, 0, kWave);
                if (L == q) {
                    const unsigned int idx = b + (unsigned int)__popcll(m & below);
                    if (idx < (unsigned int)asub) al[((int64_t)q * kCdlpSubs + j) * asub + idx] = (int32_t)w;
                    else *dense = 1;
                }
            }
        }
    }
}

// Sparse iterations, active vertices of degree <= kSparseWaveMax: one wave each (the light
// tier's method: strict-majority vote, else a 2d-slot LDS hash table).  When *dense and the
// iteration has no tier kernels (a sparse-only iteration, fl != null), every vertex of the
// fallback list fl is recomputed instead.
// The role bodies take their block index and block count (bid, nblk) and their LDS (lds) as
// arguments, so k_cdlp_sparse_fused can run several roles in one launch.
constexpr int kSparseWaveSlots = 2 * kSparseWaveMax;
constexpr size_t kSparseWaveLds = (size_t)2 * (256 / kWave) * kSparseWaveSlots * sizeof(uint32_t);

__device__ __forceinline__ void sparse_wave_role(const CdlpArgs &a, const int32_t *__restrict__ wl, int64_t asub,
                                                 const unsigned int *wcount, const int32_t *__restrict__ fl,
                                                 int64_t fn, int64_t bid, int64_t nblk, uint32_t *lds) {
    const bool full = *a.dense != 0;
    if (full && !fl) return;
    constexpr int kSlots = kSparseWaveSlots;
    constexpr int R = kSparseWaveMax / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    uint32_t *K = lds + (threadIdx.x / kWave) * kSlots;
    uint32_t *C = lds + (256 / kWave) * kSlots + (threadIdx.x / kWave) * kSlots;
    const int64_t gw = (bid * 256 + threadIdx.x) / kWave;
    const int64_t nw = nblk * (256 / kWave);   // a multiple of kCdlpSubs
    const int j = (int)(gw % kCdlpSubs);
    const int32_t *src = full ? fl : wl + (int64_t)j * asub;
    const int64_t c = full ? fn : (int64_t)shard_count(wcount, j, asub);
    const int64_t step = full ? nw : nw / kCdlpSubs;
    bool any = false;
    for (int64_t i = full ? gw : gw / kCdlpSubs; i < c; i += step) {
        const int64_t v = src[i];
        const VMeta m = vmeta(a, v);
        const int64_t d = (int64_t)m.od + m.id;
        if (bound_keeps(a, v, d)) continue;   // its label provably stays (nxt already holds it)
        uint32_t L[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int64_t k = (int64_t)r * kWave + lane;
            L[r] = k < d ? (uint32_t)a.lab[col_at(a, m, k)] : kEmpty;
        }
        const int32_t old = a.lab[v];
        Vote vt{kEmpty, 0u};
#pragma unroll
        for (int r = 0; r < R; r++) vt = vote_add(vt, L[r], (int64_t)r * kWave + lane < d);
        const uint32_t cand = __shfl(wave_vote(vt).c, 0, kWave);
        int64_t nc = 0;
#pragma unroll
        for (int r = 0; r < R; r++)
            if ((int64_t)r * kWave < d) nc += __popcll(__ballot((int64_t)r * kWave + lane < d && L[r] == cand));
        int32_t best = old;
        uint32_t cnt = 0;   // the winner's count (the recount bound)
        if (d > 0 && 2 * nc > d) {
            best = (int32_t)cand;
            cnt = (uint32_t)nc;
        } else if (d > 0) {
            int log2ts = 1;
            while ((1ll << log2ts) < 2 * d) log2ts++;
            const int ts = 1 << log2ts;
            for (int t = lane; t < ts; t += kWave) {
                K[t] = kEmpty;
                C[t] = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < R; r++)
                if ((int64_t)r * kWave < d) lds_table_add_wave(K, C, L[r], (int64_t)r * kWave + lane < d, log2ts);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            unsigned long long key = 0;
            for (int t = lane; t < ts; t += kWave) {
                const uint32_t cc = C[t];
                if (cc) {
                    const unsigned long long kk = pack(cc, K[t]);
                    key = kk > key ? kk : key;
                }
            }
            const unsigned long long wk = wave_max_u64(key);
            best = (int32_t)(kEmpty - (uint32_t)(wk & 0xffffffffu));
            cnt = (uint32_t)(wk >> 32);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (lane == 0) {
            a.nxt[v] = best;
            any |= best != old;
            if (d > 0) bound_set(a, v, cnt);
        }
    }
    if (any) raise_flag_sharded(a.changed, a.cshards);
}


// Sparse iterations, active vertices of kSparseWaveMax < degree <= kMidMax: one workgroup each,
// kMaxDeg / kBlock labels per thread in registers, the strict-majority vote, else a kSlots-slot
// LDS table (the mid tier's method, without its pipelining).  Shapes: 256 threads / 4K slots
// (four or more workgroups per CU) for both lists; a vertex above 2048 without a majority (its
// 2d slots do not fit; none from SYN-7_5's fourth iteration on) is appended to `redo`, which
// the 1024-thread / 16K-slot instance then recomputes (rin: that list, *rcount entries).
// Fallback when *dense in a sparse-only iteration: every vertex of fl then fl2.
template <int kBlock, int kSlots>
constexpr size_t sparse_group_lds() {
    return (size_t)2 * kSlots * sizeof(uint32_t) + (kBlock / kWave) * (sizeof(unsigned long long) + sizeof(uint32_t)) +
           sizeof(uint32_t);
}

template <int kBlock, int kSlots, int kMaxDeg>
__device__ __forceinline__ void sparse_group_role(const CdlpArgs &a, const int32_t *__restrict__ gl, int64_t asub,
                                                  const unsigned int *gcount, const int32_t *__restrict__ fl,
                                                  int64_t fn, const int32_t *__restrict__ fl2, int64_t fn2,
                                                  int32_t *redo, unsigned int *rcount, const int32_t *__restrict__ rin,
                                                  int64_t bid, int64_t nblk, uint32_t *lds) {
    const bool full = !rin && *a.dense != 0;
    if (full && !fl && !fl2) return;
    uint32_t *K = lds;
    uint32_t *C = lds + kSlots;
    unsigned long long *red = reinterpret_cast<unsigned long long *>(lds + 2 * kSlots);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(red + kBlock / kWave);
    uint32_t *bcast = cnt + kBlock / kWave;
    constexpr int R = kMaxDeg / kBlock;
    constexpr int NW = kBlock / kWave;
    const int tid = threadIdx.x;
    const int j = (int)(bid % kCdlpSubs);   // the block count is a multiple of kCdlpSubs
    const int32_t *src = rin ? rin : full ? fl : gl + (int64_t)j * asub;
    const int64_t c = rin ? (int64_t)*rcount : full ? fn + fn2 : (int64_t)shard_count(gcount, j, asub);
    const int64_t step = rin || full ? nblk : nblk / kCdlpSubs;
    bool any = false;
    for (int64_t i = rin || full ? bid : bid / kCdlpSubs; i < c; i += step) {
        const int64_t v = full && i >= fn ? fl2[i - fn] : src[i];   // full: fn == 0 when fl is null
        const VMeta m = vmeta(a, v);
        const int64_t d = (int64_t)m.od + m.id;
        if (bound_keeps(a, v, d)) continue;   // uniform in the workgroup; nxt already holds the label
        uint32_t L[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int64_t k = (int64_t)r * kBlock + tid;
            L[r] = k < d ? (uint32_t)a.lab[col_at(a, m, k)] : kEmpty;
        }
        Vote vt{kEmpty, 0u};
#pragma unroll
        for (int r = 0; r < R; r++) vt = vote_add(vt, L[r], (int64_t)r * kBlock + tid < d);
        vt = wave_vote(vt);
        if ((tid & (kWave - 1)) == 0) red[tid / kWave] = ((unsigned long long)vt.c << 32) | vt.n;
        __syncthreads();
        if (tid == 0) {
            Vote w{(uint32_t)(red[0] >> 32), (uint32_t)red[0]};
            for (int q = 1; q < NW; q++) w = vote_merge(w, Vote{(uint32_t)(red[q] >> 32), (uint32_t)red[q]});
            bcast[0] = w.c;
        }
        __syncthreads();
        const uint32_t cand = bcast[0];
        uint32_t mc = 0;
#pragma unroll
        for (int r = 0; r < R; r++) mc += ((int64_t)r * kBlock + tid < d && L[r] == cand) ? 1u : 0u;
        mc = wave_sum_u32(mc);
        if ((tid & (kWave - 1)) == 0) cnt[tid / kWave] = mc;
        __syncthreads();
        uint32_t nc = 0;
#pragma unroll
        for (int q = 0; q < NW; q++) nc += cnt[q];
        int32_t best = (int32_t)cand;
        uint32_t wcount = nc;   // the winner's count (the recount bound)
        if (2 * (int64_t)nc <= d && 2 * d > kSlots) {
            // no majority and no room for the table: the 16K-slot instance recomputes it
            if (tid == 0) redo[atomicAdd(rcount, 1u)] = (int32_t)v;
            __syncthreads();   // red / cnt / bcast are free for the next vertex
            continue;
        }
        if (2 * (int64_t)nc <= d) {
            int log2ts = 1;
            while ((1ll << log2ts) < 2 * d) log2ts++;
            const int ts = 1 << log2ts;
            for (int t = tid; t < ts; t += kBlock) {
                K[t] = kEmpty;
                C[t] = 0;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < R; r++)
                if ((int64_t)r * kBlock < d) lds_table_add_wave(K, C, L[r], (int64_t)r * kBlock + tid < d, log2ts);
            __syncthreads();
            unsigned long long key = 0;
            for (int t = tid; t < ts; t += kBlock) {
                const uint32_t cc = C[t];
                if (cc) {
                    const unsigned long long kk = pack(cc, K[t]);
                    key = kk > key ? kk : key;
                }
            }
            key = wave_max_u64(key);
            if ((tid & (kWave - 1)) == 0) red[tid / kWave] = key;   // red was last read before bcast
            __syncthreads();
            unsigned long long mx = red[0];
            for (int q = 1; q < NW; q++) mx = red[q] > mx ? red[q] : mx;
            best = (int32_t)(kEmpty - (uint32_t)(mx & 0xffffffffu));
            wcount = (uint32_t)(mx >> 32);
        }
        if (tid == 0) {
            const int32_t old = a.lab[v];
            a.nxt[v] = best;
            any |= best != old;
            if (d > 0) bound_set(a, v, wcount);
        }
        __syncthreads();   // red / cnt / bcast / the table are free for the next vertex
    }
    if (any) raise_flag_sharded(a.changed, a.cshards);
}

template <int kBlock, int kSlots, int kMaxDeg>
__global__ __launch_bounds__(kBlock) void k_cdlp_sparse_group(CdlpArgs a, const int32_t *__restrict__ gl,
                                                              int64_t asub, const unsigned int *gcount,
                                                              const int32_t *__restrict__ fl, int64_t fn,
                                                              const int32_t *__restrict__ fl2, int64_t fn2,
                                                              int32_t *redo, unsigned int *rcount,
                                                              const int32_t *__restrict__ rin) {
    __shared__ uint32_t lds[(sparse_group_lds<kBlock, kSlots>() + 3) / 4];
    sparse_group_role<kBlock, kSlots, kMaxDeg>(a, gl, asub, gcount, fl, fn, fl2, fn2, redo, rcount, rin, blockIdx.x,
                                               gridDim.x, lds);
}

// The three sparse roles of an iteration in one launch (GX_CDLP_SPARSE_FUSED, the default):
// blocks [0, 8S) recompute the wave list, [8S, 12S) the 2048-degree list, [12S, 20S) the
// 8192-degree list (S = kCdlpSubs), each as its own kernel would.  The roles are independent
// (they read `cur` and write disjoint vertices), and in a sparse iteration each is a short
// chain of dependent loads, so one launch overlaps them instead of running them in turn.
// Block b of a launch plays block boff + b, so three launches of one role range each are the
// unfused form (an inlined role in two kernels crashes this compiler's call-graph update).
struct SparseFusedArgs {
    const int32_t *al;
    int64_t asub;
    const unsigned int *cnt;   // the three lists' counters (kCdlpSubs * kCntStride apart)
    const int32_t *fw, *fg2, *fg4, *fg;   // fallback lists (sparse-only iterations) or null
    int64_t nfw, nfg2, nfg4, nfg;
    int32_t *redo;
    unsigned int *rcount;
};

__global__ __launch_bounds__(256) void k_cdlp_sparse_fused(CdlpArgs a, SparseFusedArgs f, int boff) {
    constexpr size_t kLds = kSparseWaveLds > sparse_group_lds<kMid2Block, kMid2Slots>()
                                ? kSparseWaveLds
                                : sparse_group_lds<kMid2Block, kMid2Slots>();
    __shared__ uint32_t lds[(kLds + 3) / 4];
    const int64_t S = kCdlpSubs, shards = S * f.asub;
    const int64_t b = (int64_t)blockIdx.x + boff;
    if (b < 8 * S) {
        sparse_wave_role(a, f.al, f.asub, f.cnt, f.fw, f.nfw, b, 8 * S, lds);
    } else {
        sparse_group_role<kMid2Block, kMid2Slots, kMid2Max>(a, f.al + shards, f.asub, f.cnt + S * kCntStride, f.fg2,
                                                            f.nfg2, nullptr, 0, nullptr, nullptr, nullptr, b - 8 * S,
                                                            4 * S, lds);
    }
}

// The 8192-degree list on 512-thread workgroups, 16 labels per thread in registers: as a third
// role of k_cdlp_sparse_fused (256 threads, 32 labels each) it set the fused kernel's registers
// to 175 VGPRs, two workgroups per CU for every role.
constexpr int kSparseBigBlock = 512;
__global__ __launch_bounds__(kSparseBigBlock) void k_cdlp_sparse_big(CdlpArgs a, SparseFusedArgs f) {
    __shared__ uint32_t lds[(sparse_group_lds<kSparseBigBlock, kMid2Slots>() + 3) / 4];
    const int64_t S = kCdlpSubs, shards = S * f.asub;
    sparse_group_role<kSparseBigBlock, kMid2Slots, kMidMax>(a, f.al + 2 * shards, f.asub, f.cnt + 2 * S * kCntStride,
                                                            f.fg4, f.nfg4, f.fg, f.nfg, f.redo, f.rcount, nullptr,
                                                            blockIdx.x, gridDim.x, lds);
}

// ---- own-label check (dense active iterations) ----------------------------------------
// From the third iteration on, a vertex whose own label is held by more than half of its
// neighbours keeps it: that label is then the unique mode (SYN-7_5: every vertex of degree
// > 16 but 17 % passes at the third iteration, all but 0.05 % of the entries at the fourth).
// When an iteration's active set overflowed (*dense), one edge-parallel pass counts, per
// vertex of degree > kTiny, the neighbours holding its label; the vertices that fail go to
// the sparse iteration's activation lists (huge ones are stamped for their tier), tiny ones
// are recomputed by k_cdlp_tiny, and the iteration turns sparse (*dense = 0).  This replaces
// the tier kernels' pass over every vertex (~0.5 ms per dense iteration on SYN-7_5).
//
// Edge-parallel layout of a CSR (built once per graph): bit k of word s says that a
// non-empty row starts at entry 64 s + k, sne[s] is the position in ne (the non-empty rows,
// ascending) of the row that holds entry 64 s.  Lane k of a 64-entry slab then finds its row
// as ne[sne[s] + popcount(bits up to k) - bit 0], without a search.
__global__ __launch_bounds__(256) void k_keep_flags(const int64_t *__restrict__ rp, int64_t n, int64_t *flag) {
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n; v += (int64_t)gridDim.x * 256)
        flag[v] = rp[v + 1] > rp[v] ? 1 : 0;
}

// ne holds each row with its sign bit set when its degree (out + in) is at most kTiny: those
// are k_cdlp_tiny's, the check skips their entries.
__global__ __launch_bounds__(256) void k_keep_layout(const int64_t *__restrict__ rp, int64_t n,
                                                     const int64_t *__restrict__ nepos, const int64_t *__restrict__ rpA,
                                                     const int64_t *__restrict__ rpT, int32_t *ne,
                                                     unsigned long long *bits, int32_t *sne) {
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n; v += (int64_t)gridDim.x * 256) {
        const int64_t b = rp[v], e = rp[v + 1];
        if (e == b) continue;
        const int32_t p = (int32_t)nepos[v];
        ne[p] = cdlp_degree(rpA, rpT, v) > kTiny ? (int32_t)v : (int32_t)((uint32_t)v | 0x80000000u);
        atomicOr(&bits[b >> 6], 1ull << (b & 63));
        for (int64_t sl = (b + kWave - 1) / kWave; sl * kWave < e; sl++) sne[sl] = p;
    }
}

// Counts, for every row of degree > kTiny (out + in degree), the entries of this CSR whose
// label equals the row's own label, into kcnt.  A wave takes kKeepU consecutive 64-entry slabs
// with every load of the chunk issued before the first compare (the chain is bits / sne ->
// ne -> labels), and carries its last row's count across the slabs: one atomic per row and
// chunk.  The first launch of an iteration (A's entries) also records whether the check runs
// (*keep = *dense) and empties the activation lists.
struct alignas(64) KeepW8 {
    unsigned long long w[8];
};
struct alignas(32) KeepS8 {
    int32_t s[8];
};
constexpr int64_t kKeepPad = 32;   // the layout's slabs rounded up to this (the largest chunk)

template <int kKeepU>
__global__ __launch_bounds__(256) void k_cdlp_keep_count(const int32_t *__restrict__ ci, int64_t nnz,
                                                         const unsigned long long *__restrict__ bits,
                                                         const int32_t *__restrict__ sne, const int32_t *__restrict__ ne,
                                                         const int32_t *__restrict__ lab, uint32_t *kcnt,
                                                         const int *dense, int *keep, unsigned int *lcounts, int head) {
    const bool run = *dense != 0;
    if (head && blockIdx.x == 0) {
        if (threadIdx.x == 0) *keep = run ? 1 : 0;
        if (run)
            for (int i = threadIdx.x; i < 3 * kCdlpSubs; i += 256) lcounts[(int64_t)i * kCntStride] = 0u;
    }
    if (!run) return;
    const int lane = threadIdx.x & (kWave - 1);
    // wave-uniform in the compiler's view too: the slab words and row positions are scalar loads
    const int64_t gw = (int64_t)blockIdx.x * (256 / kWave) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);
    const int64_t nslabs = (nnz + kWave - 1) / kWave;
    const int64_t nchunks = (nslabs + kKeepU - 1) / kKeepU;
    const unsigned long long upto = lane == kWave - 1 ? ~0ull : (2ull << lane) - 1ull;
    for (int64_t ch = gw; ch < nchunks; ch += nw) {
        const int64_t sl0 = ch * kKeepU;
        // every load unconditional (clamped indices): predicated loads would each wait in turn.
        // The chunk's slab words and row positions are two wide scalar loads (the layout is
        // padded to whole chunks, zero words past the last slab).
        unsigned long long W[kKeepU];
        int32_t R[kKeepU], Cl[kKeepU], S[kKeepU];
#pragma unroll
        for (int h = 0; h < kKeepU / 8; h++) {
            const KeepW8 wb = *reinterpret_cast<const KeepW8 *>(bits + sl0 + 8 * h);
            const KeepS8 sb = *reinterpret_cast<const KeepS8 *>(sne + sl0 + 8 * h);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                W[8 * h + i] = wb.w[i];
                S[8 * h + i] = sb.s[i];
            }
        }
#pragma unroll
        for (int u = 0; u < kKeepU; u++) Cl[u] = ci[min(sl0 * kWave + u * kWave + lane, nnz - 1)];
#pragma unroll
        for (int u = 0; u < kKeepU; u++) R[u] = ne[S[u] + __popcll(W[u] & upto) - (int)(W[u] & 1ull)];
        uint32_t M = 0, V = 0;   // bit u: lane's entry of slab u is checked / holds the row's own label
#pragma unroll
        for (int u = 0; u < kKeepU; u++) {
            const int32_t x = lab[Cl[u]], y = lab[R[u] & 0x7fffffff];
            const bool valid = (sl0 + u) * kWave + lane < nnz && R[u] >= 0;
            V |= valid ? 1u << u : 0u;
            M |= valid && x == y ? 1u << u : 0u;
        }
        int32_t crow = -1;
        uint32_t ccnt = 0;
#pragma unroll
        for (int u = 0; u < kKeepU; u++) {
            const bool valid = (V >> u) & 1u;
            const int seg = __popcll(W[u] & upto);
            unsigned long long rem = __ballot(valid);
            while (rem) {
                const int lead = __ffsll((long long)rem) - 1;
                const int sg = __builtin_amdgcn_readlane(seg, lead);
                const int32_t r = __builtin_amdgcn_readlane(R[u], lead);
                const bool in = valid && seg == sg;
                const unsigned long long grp = __ballot(in);
                const uint32_t c = (uint32_t)__popcll(__ballot(in && ((M >> u) & 1u)));
                if (r == crow) {
                    ccnt += c;
                } else {
                    if (ccnt && lane == 0) atomicAdd(&kcnt[crow], ccnt);
                    crow = r;
                    ccnt = c;
                }
                rem &= ~grp;
            }
        }
        if (ccnt && lane == 0) atomicAdd(&kcnt[crow], ccnt);
    }
}

// Column-sorted form of the count (the default where built; GX_CDLP_KEEP_SORTED=0: the slabs
// above).  The slab pass is bound by the texture units' line rate: rocprofv3 on SYN-7_5 shows
// TA busy 92 % of the launch for ~59 M L2 requests, one per label gather (its 64 lanes read 64
// different lines).  Here the entries of the rows the check reads are cut into blocks of at
// most kKeepBlock entries and a row span of at most kKeepRows rows, and each block's entries
// are sorted by column (built once per graph): a block's label gathers walk the label array in
// order, so a wave's lanes share lines (hub columns repeat many times per block).  Each entry
// keeps its column (4 B) and its row within the block (2 B); the rows' own labels and counts
// live in LDS, and one global atomic per (block, row) adds the count.
constexpr int64_t kKeepBlockMax = 1 << 20;   // GX_CDLP_KEEP_BLOCK (build time): 1024 .. 1 Mi
constexpr int kKeepRows = 1024;

// One wave per included row: the row's entries as (block << 32 | column) keys with the row's
// place in its block as the value (kpos: where the row's keys start; a row of kKeepBlock or
// more entries spans whole blocks of its own, from rblk).
__global__ __launch_bounds__(256) void k_keep_sorted_keys(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                          const int32_t *__restrict__ rows, const int64_t *__restrict__ kpos,
                                                          const int32_t *__restrict__ rblk,
                                                          const int32_t *__restrict__ brow0, int64_t nrows,
                                                          int64_t kKeepBlock, uint64_t *keys, uint16_t *vals) {
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave; i < nrows;
         i += (int64_t)gridDim.x * (256 / kWave)) {
        const int64_t r = rows[i], b0 = rp[r], d = rp[r + 1] - b0;
        for (int64_t k = lane; k < d; k += kWave) {
            const int64_t b = d >= kKeepBlock ? rblk[i] + k / kKeepBlock : rblk[i];
            keys[kpos[i] + k] = ((uint64_t)b << 32) | (uint32_t)ci[b0 + k];
            vals[kpos[i] + k] = (uint16_t)(r - brow0[b]);
        }
    }
}

__global__ void k_keep_sorted_cols(const uint64_t *__restrict__ keys, int64_t m, int32_t *cols) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        cols[i] = (int32_t)(uint32_t)keys[i];
}

__global__ __launch_bounds__(256) void k_cdlp_keep_sorted(const int64_t *__restrict__ bstart,
                                                          const int32_t *__restrict__ brow0, int64_t nb,
                                                          const int32_t *__restrict__ scol,
                                                          const uint16_t *__restrict__ srow,
                                                          const int32_t *__restrict__ lab, int64_t n, uint32_t *kcnt,
                                                          const int *dense, int *keep, unsigned int *lcounts, int head) {
    const bool run = *dense != 0;
    if (head && blockIdx.x == 0) {
        if (threadIdx.x == 0) *keep = run ? 1 : 0;
        if (run)
            for (int i = threadIdx.x; i < 3 * kCdlpSubs; i += 256) lcounts[(int64_t)i * kCntStride] = 0u;
    }
    if (!run) return;
    __shared__ int32_t own[kKeepRows];
    __shared__ uint32_t cnt[kKeepRows];
    const int tid = threadIdx.x;
    for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const int64_t r0 = brow0[b], e0 = bstart[b], e1 = bstart[b + 1];
        const int span = (int)min((int64_t)kKeepRows, n - r0);
        for (int i = tid; i < span; i += 256) {
            own[i] = lab[r0 + i];
            cnt[i] = 0u;
        }
        __syncthreads();
        // rounds of U entries per thread, software-pipelined: a round's label gathers are issued,
        // then the next round's columns and rows, then the compares wait for the gathers only
        constexpr int U = 8;
        int32_t c[U];
        uint32_t lr[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t k = min(e0 + tid + (int64_t)u * 256, e1 - 1);
            c[u] = scol[k];
            lr[u] = srow[k];
        }
        for (int64_t e = e0 + tid; e < e1; e += 256 * U) {
            int32_t x[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = lab[c[u]];
            int32_t cn[U];
            uint32_t ln[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int64_t k = min(e + (int64_t)(U + u) * 256, e1 - 1);
                cn[u] = scol[k];
                ln[u] = srow[k];
            }
#pragma unroll
            for (int u = 0; u < U; u++)
                if (e + (int64_t)u * 256 < e1 && x[u] == own[lr[u]]) atomicAdd(&cnt[lr[u]], 1u);
#pragma unroll
            for (int u = 0; u < U; u++) {
                c[u] = cn[u];
                lr[u] = ln[u];
            }
        }
        __syncthreads();
        for (int i = tid; i < span; i += 256)
            if (cnt[i]) atomicAdd(&kcnt[r0 + i], cnt[i]);
        __syncthreads();   // own / cnt are free for the next block
    }
}

// Per vertex of degree > kTiny: keep (2 count > degree) or recompute: onto the activation list
// of its degree (the sparse kernels' lists, shard = wave index mod kCdlpSubs), or, huge, the
// iteration's stamp for the huge tier (a kept huge vertex loses a stamp k_cdlp_mark gave it).
// kcnt is left zero.  A full list sets *kover.
__global__ __launch_bounds__(256) void k_cdlp_keep_apply(const int64_t *__restrict__ rpA, const int64_t *__restrict__ rpT,
                                                         int64_t v0, int64_t v1, uint32_t *kcnt, int32_t *act,
                                                         int32_t stamp, const int *keep, unsigned int *counts,
                                                         int32_t *al, int64_t asub, int *kover, int32_t *vlb,
                                                         int32_t *vchg) {
    if (*keep == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave;
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);
    const int j = (int)(gw % kCdlpSubs);
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int64_t b = v0 + gw * kWave; b < v1; b += nw * kWave) {
        const int64_t v = b + lane;
        int L = -1;
        if (v < v1) {
            const int64_t d = cdlp_degree(rpA, rpT, v);
            if (d > kTiny) {
                const uint32_t c = kcnt[v];
                if (c) kcnt[v] = 0u;
                const bool kept = 2 * (int64_t)c > d;
                if (kept && vlb) {   // the recount bound: the own label's exact count
                    vlb[v] = (int32_t)c;
                    vchg[v] = 0;
                }
                if (d > kMidMax) {
                    if (!kept) act[v] = stamp;
                    else if (act[v] == stamp) act[v] = stamp - 1;

                } else if (!kept) {
                    L = d <= kSparseWaveMax ? 0 : d <= kSparseG2Max ? 1 : 2;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const unsigned long long m = __ballot(L == q);
            if (!m) continue;
            unsigned int base = 0;
            if (lane == 0) base = atomicAdd(&counts[((1 + q) * kCdlpSubs + j) * kCntStride], (unsigned int)__popcll(m));
            base = __shfl(base, 0, kWave);
            if (L == q) {
                const unsigned int idx = base + (unsigned int)__popcll(m & below);
                if (idx < (unsigned int)asub) al[((int64_t)q * kCdlpSubs + j) * asub + idx] = (int32_t)v;
                else *kover = 1;
            }
        }
    }
}

// The check's outcome: lists that fit make the iteration sparse; a full one leaves it dense
// (every tier kernel recomputes every vertex, as without the check).
__global__ void k_cdlp_keep_finish(int *dense, int *keep, int *kover) {
    if (*keep) {
        if (*kover) *keep = 0;
        else *dense = 0;
    }
    *kover = 0;
}

// First iteration of an undirected graph whose rows are sorted by column: every label is still
// its vertex id, so the result is the row's first column (the smallest neighbour), one load per
// vertex instead of a pass over every label (~470 us of tier kernels on SYN-7_5).
__global__ __launch_bounds__(256) void k_cdlp_first_sorted(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                           int64_t v0, int64_t v1, int32_t *nxt, int *changed,
                                                           int cshards) {
    bool any = false;
    for (int64_t v = v0 + (int64_t)blockIdx.x * 256 + threadIdx.x; v < v1; v += (int64_t)gridDim.x * 256) {
        const int64_t b = rp[v];
        const int32_t l = rp[v + 1] > b ? ci[b] : (int32_t)v;
        nxt[v] = l;
        any |= l != (int32_t)v;
    }
    if (__ballot(any) && (threadIdx.x & (kWave - 1)) == 0) raise_flag_sharded(changed, cshards);
}

// First iteration of a directed graph whose rows (A and A') are strictly sorted: every label is
// still its vertex id, a neighbour's label occurs once per direction, so the mode is the
// smallest reciprocal neighbour (out and in: count 2) if there is one, else the smallest
// neighbour of either direction.  Replaces the tiers' counting pass over every label (~0.45 ms
// of SYN-cit's first iteration: a random label gather per entry).  A wave takes 64 consecutive
// vertices: rows of at most kFirstSmall entries each are compared pair by pair in one lane's
// registers, rows up to `medmax` entries afterwards by 16-lane groups (four rows at once), longer
// ones by the whole wave (first_dir_merge).  (A list of the long rows for a second kernel cost
// 0.69 ms: returning atomics on one counter.)  SYN-cit: 0.14 ms against the tiers' ~0.45.

// Both rows of v merged G entries at a time by G lanes (each out-entry looked up among the
// in-chunk by a log2(G)-step search over the group's lanes), the chunk with the smaller last
// entry advanced.  Every common entry is met in the round that retires its chunk, and chunks
// retire in ascending order, so the first round with a hit holds the smallest one.  SYN-cit: at
// most 13 rounds of 64, 1.4 per long row (a reciprocal neighbour is usually near the front).
// Group-uniform: every lane of the group calls it (gl = lane within the group).  Returns the
// label: that entry, else the smallest entry of either row (from the first chunks).
template <int G>
__device__ __forceinline__ int32_t first_dir_merge(const int32_t *__restrict__ xr, int64_t od,
                                                   const int32_t *__restrict__ yr, int64_t id, int gl) {
    int64_t i = 0, j = 0;
    int32_t xa = gl < od ? xr[gl] : INT32_MAX;   // ids < n <= INT32_MAX
    int32_t yb = gl < id ? yr[gl] : INT32_MAX;
    const int32_t lo = min(__shfl(xa, 0, G), __shfl(yb, 0, G));
    while (i < od && j < id) {
        int pos = 0;   // entries of the in-chunk below xa
#pragma unroll
        for (int st = G / 2; st; st >>= 1) pos += __shfl(yb, pos + st - 1, G) < xa ? st : 0;
        const int32_t at = __shfl(yb, pos & (G - 1), G);
        uint32_t h = pos < G && at == xa && xa != INT32_MAX ? (uint32_t)xa : 0xffffffffu;
        if constexpr (G == kWave) {
            h = wave_min_u32(h);
        } else {
#pragma unroll
            for (int o = G / 2; o; o >>= 1) h = min(h, (uint32_t)__shfl_xor((int)h, o, G));
        }
        if (h != 0xffffffffu) return (int32_t)h;
        const int32_t xm = __shfl(xa, G - 1, G), ym = __shfl(yb, G - 1, G);
        if (xm <= ym) {
            i += G;
            xa = i + gl < od ? xr[i + gl] : INT32_MAX;
        }
        if (ym <= xm) {
            j += G;
            yb = j + gl < id ? yr[j + gl] : INT32_MAX;
        }
    }
    return lo;
}

template <int kFirstSmall>
__global__ __launch_bounds__(256) void k_cdlp_first_dir(const int64_t *__restrict__ rpA, const int32_t *__restrict__ ciA,
                                                        const int64_t *__restrict__ rpT, const int32_t *__restrict__ ciT,
                                                        int64_t n, int32_t *out, int *changed, int cshards, int medmax) {
    const int lane = threadIdx.x & (kWave - 1);
    bool any = false;
    // wave-uniform trips: v0 is the wave's first vertex
    for (int64_t v0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~(kWave - 1)); v0 < n; v0 += (int64_t)gridDim.x * 256) {
        const int64_t v = v0 + lane;
        const bool in = v < n;
        const int64_t ob = in ? rpA[v] : 0, od = in ? rpA[v + 1] - ob : 0;
        const int64_t ib = in ? rpT[v] : 0, id = in ? rpT[v + 1] - ib : 0;
        const int64_t wide = od > id ? od : id;
        const bool lng = wide > kFirstSmall;
        if (in && !lng) {
            // loads clamped into the row (or to entry 0: rows_sorted implies nnz > 0) and
            // issued four at a time while any lane's rows reach that far
            int32_t x[kFirstSmall], y[kFirstSmall];
            const int64_t ra = od ? ob : 0, rb = id ? ib : 0, la = od ? od - 1 : 0, lb = id ? id - 1 : 0;
#pragma unroll
            for (int k = 0; k < kFirstSmall; k++) {
                x[k] = -1;
                y[k] = -2;   // the paddings match nothing
            }
#pragma unroll
            for (int k0 = 0; k0 < kFirstSmall; k0 += 4) {
                if (!__any(wide > k0)) break;
#pragma unroll
                for (int k = k0; k < k0 + 4; k++) {
                    const int32_t a = ciA[ra + min((int64_t)k, la)], b = ciT[rb + min((int64_t)k, lb)];
                    x[k] = k < od ? a : -1;
                    y[k] = k < id ? b : -2;
                }
            }
            int32_t m = INT32_MAX;
#pragma unroll
            for (int i = 0; i < kFirstSmall; i++)
#pragma unroll
                for (int j = 0; j < kFirstSmall; j++) m = x[i] == y[j] ? min(m, x[i]) : m;
            const int32_t lo = min(od ? x[0] : INT32_MAX, id ? y[0] : INT32_MAX);
            const int32_t l = m != INT32_MAX ? m : od + id ? lo : (int32_t)v;
            out[v] = l;
            any |= l != (int32_t)v;
        }
        // rows of at most medmax entries each: four at a time, 16 lanes each; group g takes the
        // wave's g-th, (g+4)-th, ... such row (the shuffles of the row extents run wave-wide)
        const int grp = lane >> 4, gl = lane & 15;
        uint64_t mb = __ballot(in && lng && wide <= medmax);
        for (int k = 0; k < grp; k++) mb &= mb - 1;
        while (__ballot(mb != 0)) {
            const int b = mb ? __builtin_ctzll(mb) : 0;
            const int64_t uob = __shfl(ob, b), uod = __shfl(od, b), uib = __shfl(ib, b), uid = __shfl(id, b);
            if (mb) {
                const int32_t l = first_dir_merge<16>(ciA + uob, uod, ciT + uib, uid, gl);
                if (gl == 0) {
                    out[v0 + b] = l;
                    any |= l != (int32_t)(v0 + b);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; k++) mb &= mb - 1;
        }
        // the longer rows, one after the other, by the whole wave
        for (uint64_t bal = __ballot(in && lng && wide > medmax); bal; bal &= bal - 1) {
            const int b = __builtin_ctzll(bal);
            const int64_t u = v0 + b;
            const int64_t uob = __shfl(ob, b), uod = __shfl(od, b), uib = __shfl(ib, b), uid = __shfl(id, b);
            const int32_t l = first_dir_merge<kWave>(ciA + uob, uod, ciT + uib, uid, lane);
            if (lane == 0) {
                out[u] = l;
                any |= l != (int32_t)u;
            }
        }
    }
    if (__ballot(any) && (threadIdx.x & (kWave - 1)) == 0) raise_flag_sharded(changed, cshards);
}

// Whether every row of a CSR is sorted by column (strictly: rows hold no duplicates): the row
// starts as a bitmap over the entries, then one compare per entry.
__global__ __launch_bounds__(256) void k_row_start_bits(const int64_t *__restrict__ rp, int64_t n, uint32_t *bits) {
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n; v += (int64_t)gridDim.x * 256) {
        const int64_t b = rp[v];
        if (rp[v + 1] > b) atomicOr(&bits[b >> 5], 1u << (b & 31));
    }
}

__global__ __launch_bounds__(256) void k_rows_sorted(const int32_t *__restrict__ ci, int64_t nnz,
                                                     const uint32_t *__restrict__ bits, int *sorted) {
    bool bad = false;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k + 1 < nnz; k += (int64_t)gridDim.x * 256) {
        const int64_t k1 = k + 1;
        bad |= ci[k1] <= ci[k] && !((bits[k1 >> 5] >> (k1 & 31)) & 1u);
    }
    if (__ballot(bad) && (threadIdx.x & (kWave - 1)) == 0) *sorted = 0;
}

// Hub-first relabelling of a CSR: keys[e] = perm[row] << 32 | perm[col], sorted into the
// relabelled CSR (the PageRank plan's transform, gx_pr.hip).
__global__ void k_cdlp_permute_keys(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, int64_t n,
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

// out[v] = in[idx[v]]
__global__ void k_cdlp_gather_i32(const int32_t *__restrict__ in, const int32_t *__restrict__ idx, int64_t n,
                                  int32_t *__restrict__ out) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        out[v] = in[idx[v]];
}

// The graph CDLP runs on: the caller's (partitioned API, GX_CDLP_RELABEL=0) or its hub-first
// relabelling (gx_cdlp).  Label VALUES stay the caller's vertex ids either way, so the
// smallest-label tie rule is unchanged.
struct CdlpGraph {
    gx_ctx *ctx = nullptr;
    int64_t n = 0;
    bool directed = false;
    const int64_t *rpA = nullptr, *rpT = nullptr;
    const int32_t *ciA = nullptr, *ciT = nullptr;
    const int64_t *h_rpA = nullptr, *h_rpT = nullptr;
    int64_t nnzA = 0, nnzT = 0;
};

CdlpGraph cdlp_view(gx_graph *g) {
    CdlpGraph v;
    v.ctx = g->ctx;
    v.n = (int64_t)g->n;
    v.directed = g->directed;
    v.rpA = g->A.rp.p;
    v.ciA = g->A.ci.p;
    v.h_rpA = g->A.h_rp.data();
    v.nnzA = (int64_t)g->A.nnz;
    if (g->directed) {
        v.rpT = g->AT.rp.p;
        v.ciT = g->AT.ci.p;
        v.h_rpT = g->AT.h_rp.data();
        v.nnzT = (int64_t)g->AT.nnz;
    }
    return v;
}

// Staged labels of one iteration: the plan's sorted blocks and the output array.
__global__ void k_cdlp_iota(int32_t *a, int64_t n) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x)
        a[v] = (int32_t)v;
}

// Tier lists of the vertices in [v0, v1): medium vertices (LDS table per workgroup) and huge
// ones (chunked global hash segments); light vertices are found by k_cdlp_light itself.
struct CdlpPlan {
    int64_t v0 = 0, v1 = 0;
    size_t n_light = 0, n_mid2 = 0, n_mid = 0, n_huge = 0, n_chunks = 0;
    int64_t total = 0;
    DBuf<int32_t> d_hv, d_hl, d_mv, d_cvert, d_lv, d_mv2, d_sv, d_mv4;
    size_t n_small = 0, n_mid4 = 0, n_light_s = 0;
    DBuf<int32_t> d_lvs;                // light vertices with degree <= kLightSlots / 2
    DBuf<int32_t> d_wall;               // every vertex of degree <= kSparseWaveMax (sparse fallback)
    size_t n_wall = 0;
    DBuf<int64_t> d_hoff, d_cbeg;
    DBuf<unsigned long long> gtab;      // huge vertices' global tables (k_cdlp_huge_insert's words)
    uint32_t epoch = 0;                 // the last iteration's table epoch (1..kHugeEpochs)
    DBuf<unsigned long long> vkey;      // per huge vertex best key (zero between iterations)
};

// The recount bound's arrays (gx_cdlp, CdlpArgs::vlb / vchg / hvalid).
struct CdlpBound {
    int32_t *vlb, *vchg;
    int *hvalid;
};

// Switches read at every call (tests flip them within one process); unset means `dflt`.
bool env_on(const char *name, bool dflt = true) {
    const char *e = std::getenv(name);
    return e ? std::atoi(e) != 0 : dflt;
}

int cdlp_plan(const CdlpGraph &g, int64_t v0, int64_t v1, CdlpPlan &P, hipStream_t s) {
    std::vector<int32_t> hv, hl, mv, cvert, lv, mv2, sv, mv4, lvs, wall;
    std::vector<int64_t> hoff, cbeg;
    int64_t total = 0;
    for (int64_t v = v0; v < v1; v++) {
        int64_t d = g.h_rpA[v + 1] - g.h_rpA[v];
        if (g.directed) d += g.h_rpT[v + 1] - g.h_rpT[v];
        if (d <= kSparseWaveMax) wall.push_back((int32_t)v);
        if (d <= kTiny) {
            // k_cdlp_tiny scans the range itself
        } else if (d <= kWave) {
            sv.push_back((int32_t)v);
        } else if (d <= kLightSlots / 2) {
            lvs.push_back((int32_t)v);
        } else if (d <= kLdsHash / 2) {
            lv.push_back((int32_t)v);
        } else if (d <= kMid2Max) {
            mv2.push_back((int32_t)v);
        } else if (d <= kMid4Max) {
            mv4.push_back((int32_t)v);
        } else if (d <= kMidMax) {
            mv.push_back((int32_t)v);
        } else {
            if (d > kHugeMaxDeg) return fail(GX_INVALID_VALUE, "gx_cdlp: a vertex degree exceeds 2^27 - 1");
            int l2 = 1;
            while ((1ll << l2) < 2 * d) l2++;
            for (int64_t c = 0; c < d; c += kHugeChunk) {
                cvert.push_back((int32_t)hv.size());
                cbeg.push_back(c);
            }
            hv.push_back((int32_t)v);
            hl.push_back(l2);
            hoff.push_back(total);
            total += 1ll << l2;
        }
    }
    P.v0 = v0;
    P.v1 = v1;
    P.n_light = lv.size();
    P.n_light_s = lvs.size();
    P.n_small = sv.size();
    P.n_mid4 = mv4.size();
    if (!mv4.empty()) {
        GX_TRY(P.d_mv4.alloc(mv4.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_mv4.p, mv4.data(), mv4.size() * 4, hipMemcpyHostToDevice, s));
    }
    if (!sv.empty()) {
        GX_TRY(P.d_sv.alloc(sv.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_sv.p, sv.data(), sv.size() * 4, hipMemcpyHostToDevice, s));
    }
    P.n_mid2 = mv2.size();
    P.n_mid = mv.size();
    P.n_huge = hv.size();
    P.n_chunks = cvert.size();
    P.total = total;
    if (!hv.empty()) {
        GX_TRY(P.d_hv.alloc(hv.size()));
        GX_TRY(P.d_hl.alloc(hl.size()));
        GX_TRY(P.d_hoff.alloc(hoff.size()));
        GX_TRY(P.gtab.alloc(total));
        GX_TRY(P.vkey.alloc(hv.size()));
        GX_HIP_TRY(hipMemsetAsync(P.vkey.p, 0, hv.size() * 8, s));
        GX_HIP_TRY(hipMemsetAsync(P.gtab.p, 0, (size_t)total * 8, s));   // epoch 0: every slot empty
        P.epoch = 0;
        GX_TRY(P.d_cvert.alloc(cvert.size()));
        GX_TRY(P.d_cbeg.alloc(cbeg.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_hv.p, hv.data(), hv.size() * 4, hipMemcpyHostToDevice, s));
        GX_HIP_TRY(hipMemcpyAsync(P.d_hl.p, hl.data(), hl.size() * 4, hipMemcpyHostToDevice, s));
        GX_HIP_TRY(hipMemcpyAsync(P.d_hoff.p, hoff.data(), hoff.size() * 8, hipMemcpyHostToDevice, s));
        GX_HIP_TRY(hipMemcpyAsync(P.d_cvert.p, cvert.data(), cvert.size() * 4, hipMemcpyHostToDevice, s));
        GX_HIP_TRY(hipMemcpyAsync(P.d_cbeg.p, cbeg.data(), cbeg.size() * 8, hipMemcpyHostToDevice, s));
    }
    if (!mv.empty()) {
        GX_TRY(P.d_mv.alloc(mv.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_mv.p, mv.data(), mv.size() * 4, hipMemcpyHostToDevice, s));
    }
    if (!mv2.empty()) {
        GX_TRY(P.d_mv2.alloc(mv2.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_mv2.p, mv2.data(), mv2.size() * 4, hipMemcpyHostToDevice, s));
    }
    if (!lvs.empty()) {
        GX_TRY(P.d_lvs.alloc(lvs.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_lvs.p, lvs.data(), lvs.size() * 4, hipMemcpyHostToDevice, s));
    }
    P.n_wall = wall.size();
    if (!wall.empty()) {
        GX_TRY(P.d_wall.alloc(wall.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_wall.p, wall.data(), wall.size() * 4, hipMemcpyHostToDevice, s));
    }
    if (!lv.empty()) {
        GX_TRY(P.d_lv.alloc(lv.size()));
        GX_HIP_TRY(hipMemcpyAsync(P.d_lv.p, lv.data(), lv.size() * 4, hipMemcpyHostToDevice, s));
    }
    GX_HIP_TRY(hipStreamSynchronize(s));   // host vectors go out of scope
    return GX_SUCCESS;
}

// One synchronous iteration for the plan's vertices: nxt[v] for v in [v0, v1) from cur
// (the full label array); *changed is set when a label moved (caller zeroes it).
// The tier kernels write disjoint vertices and only read `cur`; on three streams they paid
// while they were slow (SYN-7_5 10.5 -> 9.8 ms), with the current tiers one stream is faster
// (3.39 -> 2.89 ms, SYN-cit 3.61 -> 3.37), so they run on one.
// The active vertices of a sparse iteration (k_cdlp_mark): kCdlpSubs shards of asub entries.
struct SparseLists {
    const int32_t *al;            // kCdlpLists - 1 lists of kCdlpSubs shards of asub entries
    int64_t asub;
    const unsigned int *counts;   // the change list's counters, then the three lists'
    bool only;                    // sparse-only: no tier kernels but the huge ones
    int32_t *redo;                // k_cdlp_sparse_group's vertices for the 16K-slot instance
    unsigned int *rcount;         // this iteration's redo count (zero at its start)
};

int cdlp_iteration(const CdlpGraph &g, CdlpPlan &P, const int32_t *cur, int32_t *nxt, int *changed, hipStream_t s,
                   const int32_t *act = nullptr, int32_t stamp = 0, const int *dense = nullptr, bool first = false,
                   const SparseLists *sl = nullptr, int cshards = 1, const int *keep = nullptr,
                   const CdlpBound *bd = nullptr) {
    gx_ctx *ctx = g.ctx;
    const int64_t n = g.n;
    CdlpArgs a{g.rpA,  g.ciA,  g.rpT, g.ciT,  cur,        nxt,     n,        changed,
               P.v0,   P.v1,   act,   stamp,  dense,      first && !g.directed ? 1 : 0,
               sl ? 1 : 0,     cshards};
    a.keep = keep;
    if (bd) {
        a.vlb = bd->vlb;
        a.vchg = bd->vchg;
        a.hvalid = bd->hvalid;
    }
    const bool tiers = !(sl && sl->only);   // sparse-only: the huge tier alone beside the sparse kernels
    if (sl) {
        // exit at once when *dense (the tier kernels below then recompute every vertex)
        KTimer kt(ctx, "cdlp_sparse", s);
        const unsigned int *cnt = sl->counts + kCdlpSubs * kCntStride;
        // a sparse-only iteration's fallback lists (nothing else recomputes these vertices)
        const bool o = sl->only;
        // GX_CDLP_SPARSE_FUSED=0: the three roles as three launches
        const SparseFusedArgs f{sl->al,
                                sl->asub,
                                cnt,
                                o ? P.d_wall.p : nullptr,
                                o ? P.d_mv2.p : nullptr,
                                o ? P.d_mv4.p : nullptr,
                                o ? P.d_mv.p : nullptr,
                                (int64_t)P.n_wall,
                                (int64_t)P.n_mid2,
                                (int64_t)P.n_mid4,
                                (int64_t)P.n_mid,
                                sl->redo,
                                sl->rcount};
        if (env_on("GX_CDLP_SPARSE_FUSED")) {
            hipLaunchKernelGGL(k_cdlp_sparse_fused, dim3(12 * kCdlpSubs), dim3(256), 0, s, a, f, 0);
            GX_TRY(check_launch("k_cdlp_sparse_fused"));
        } else {
            const int ranges[3] = {0, 8 * kCdlpSubs, 12 * kCdlpSubs};
            for (int q = 0; q < 2; q++) {
                hipLaunchKernelGGL(k_cdlp_sparse_fused, dim3(ranges[q + 1] - ranges[q]), dim3(256), 0, s, a, f,
                                   ranges[q]);
                GX_TRY(check_launch("k_cdlp_sparse_fused"));
            }
        }
        hipLaunchKernelGGL(k_cdlp_sparse_big, dim3(8 * kCdlpSubs), dim3(kSparseBigBlock), 0, s, a, f);
        GX_TRY(check_launch("k_cdlp_sparse_big"));
        hipLaunchKernelGGL((k_cdlp_sparse_group<kMidBlock, kMidSlots, kMidMax>), dim3(kCdlpSubs), dim3(kMidBlock), 0,
                           s, a, nullptr, (int64_t)0, nullptr, nullptr, (int64_t)0, nullptr, (int64_t)0, nullptr,
                           sl->rcount, sl->redo);
        GX_TRY(check_launch("k_cdlp_sparse_redo"));
        if (o && keep && P.v1 > P.v0) {   // the own-label check's tiny vertices (no tier kernels here)
            hipLaunchKernelGGL(k_cdlp_tiny, dim3(grid_for((uint64_t)(P.v1 - P.v0), kCdlpBlock, 8192)),
                               dim3(kCdlpBlock), 0, s, a);
            GX_TRY(check_launch("k_cdlp_tiny"));
        }
    }
    hipStream_t s1 = s, s2 = s;   // one stream: overlapped tier kernels slowed each other down
    if (tiers && P.n_mid2) {
        KTimer kt(ctx, "cdlp_mid2", s);
        const unsigned grid2 = (unsigned)std::min<size_t>(P.n_mid2, (size_t)std::max(1, ctx->num_cus) * 4);
        hipLaunchKernelGGL((k_cdlp_mid<kMid2Block, kMid2Slots>), dim3(grid2), dim3(kMid2Block), 0, s, a, P.d_mv2.p,
                           (int32_t)P.n_mid2);
        GX_TRY(check_launch("k_cdlp_mid2"));
    }
    if (P.n_huge) {
        KTimer kt(ctx, "cdlp_heavy", s1);
        uint32_t ep = P.epoch;
        if (!a.first) {   // a new epoch empties every table slot; past the last one, a real clear
            if (++ep > (uint32_t)kHugeEpochs) {
                GX_HIP_TRY(hipMemsetAsync(P.gtab.p, 0, (size_t)P.total * 8, s1));
                ep = 1;
            }
            P.epoch = ep;
        }
        hipLaunchKernelGGL(k_cdlp_huge_insert, dim3((unsigned)P.n_chunks), dim3(kHugeBlock), 0, s1, a, P.d_hv.p,
                           P.d_hoff.p, P.d_hl.p, P.d_cvert.p, P.d_cbeg.p, P.gtab.p, ep, P.vkey.p);
        GX_TRY(check_launch("k_cdlp_huge_insert"));
        hipLaunchKernelGGL(k_cdlp_huge_final, dim3(grid_for(P.n_huge, 64, 1024)), dim3(64), 0, s1, a, P.d_hv.p,
                           (int32_t)P.n_huge, P.vkey.p);
        GX_TRY(check_launch("k_cdlp_huge_final"));
    }
    if (tiers && P.n_light) {
        KTimer kt(ctx, "cdlp_light", s2);
        hipLaunchKernelGGL(k_cdlp_light<kLdsHash>, dim3(grid_for((uint64_t)P.n_light * kWave, kCdlpBlock, 8192)),
                           dim3(kCdlpBlock), 0, s2, a, P.d_lv.p, (int32_t)P.n_light);
        GX_TRY(check_launch("k_cdlp_light"));
    }
    if (tiers && P.n_mid) {
        KTimer kt(ctx, "cdlp_mid", s);
        const unsigned mid_grid = (unsigned)std::min<size_t>(P.n_mid, (size_t)std::max(1, ctx->num_cus));
        hipLaunchKernelGGL((k_cdlp_mid<kMidBlock, kMidSlots>), dim3(mid_grid), dim3(kMidBlock), 0, s, a, P.d_mv.p,
                           (int32_t)P.n_mid);
        GX_TRY(check_launch("k_cdlp_mid"));
    }
    if (tiers && P.n_mid4) {
        KTimer kt(ctx, "cdlp_mid4", s1);
        const unsigned grid4 = (unsigned)std::min<size_t>(P.n_mid4, (size_t)std::max(1, ctx->num_cus) * 2);
        hipLaunchKernelGGL((k_cdlp_mid<kMid4Block, kMid4Slots>), dim3(grid4), dim3(kMid4Block), 0, s1, a, P.d_mv4.p,
                           (int32_t)P.n_mid4);
        GX_TRY(check_launch("k_cdlp_mid4"));
    }
    if (tiers && P.n_small) {
        KTimer kt(ctx, "cdlp_small", s2);
        hipLaunchKernelGGL(k_cdlp_small, dim3(grid_for((uint64_t)P.n_small * kWave, kCdlpBlock, 8192)),
                           dim3(kCdlpBlock), 0, s2, a, P.d_sv.p, (int32_t)P.n_small);
        GX_TRY(check_launch("k_cdlp_small"));
    }
    if (tiers && P.n_light_s) {
        KTimer kt(ctx, "cdlp_light_s", s2);
        hipLaunchKernelGGL(k_cdlp_light<kLightSlots>, dim3(grid_for((uint64_t)P.n_light_s * kWave, kCdlpBlock, 8192)),
                           dim3(kCdlpBlock), 0, s2, a, P.d_lvs.p, (int32_t)P.n_light_s);
        GX_TRY(check_launch("k_cdlp_light_s"));
    }
    if (tiers && P.v1 > P.v0) {
        KTimer kt(ctx, "cdlp_tiny", s);
        hipLaunchKernelGGL(k_cdlp_tiny, dim3(grid_for((uint64_t)(P.v1 - P.v0), kCdlpBlock, 8192)), dim3(kCdlpBlock),
                           0, s, a);
        GX_TRY(check_launch("k_cdlp_tiny"));
    }
    return GX_SUCCESS;
}

}  // namespace
}  // namespace gx

using namespace gx;

namespace gx {
namespace {
// What gx_cdlp keeps on the graph between calls (gx_graph::cdlp): the hub-first relabelled
// graph, the staging plan, the tier lists (built on the host from the row pointers: ~3 ms of
// idle device per call on SYN-7_5 when rebuilt) and the label, flag and active-set buffers.
// Iteration-count-sized buffers grow on demand.
struct CdlpCache {
    bool relabel = false;
    CdlpGraph G;                          // the graph the iterations run on
    DBuf<int64_t> rpA, rpT;               // relabelled copies (relabel)
    DBuf<int32_t> ciA, ciT;
    std::vector<int64_t> h_rpA, h_rpT;
    DBuf<int32_t> order, perm;            // order[p]: the caller's vertex at p; perm = its inverse
    CdlpPlan P;
    DBuf<int32_t> la, lb, act, al, tmp;
    DBuf<uint64_t> clist;
    DBuf<int> changed, dense;
    DBuf<unsigned int> ccount;
    int *hflag = nullptr, *dflag = nullptr;
    int cap_iters = 0;
    int64_t sub = 0, asub = 0;
    bool rows_sorted = false;   // A's rows (and A''s, directed) sorted by column (k_rows_sorted)
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    // the own-label check's edge-parallel layout of G's A (and A'), its counters and flags
    // (keep, kover); built by the first call that needs it
    struct KeepCsr {
        DBuf<unsigned long long> bits;
        DBuf<int32_t> sne, ne;
        // column-sorted blocks (k_cdlp_keep_sorted): block b's entries are scol / srow
        // [bstart[b], bstart[b + 1]), its rows start at brow0[b]
        DBuf<int64_t> bstart;
        DBuf<int32_t> brow0, scol;
        DBuf<uint16_t> srow;
        int64_t nb = 0;
    } kA, kT;
    bool keep_sorted = false;   // kA / kT hold column-sorted blocks
    DBuf<uint32_t> kcnt;
    DBuf<int> kflags;
    bool keep_built = false;
    // entries the check reads: with the hub-first copy (rows by total degree, descending) the
    // rows of degree <= kTiny, which it skips, hold every entry from here on
    int64_t keep_nnzA = 0, keep_nnzT = 0;
    DBuf<int32_t> vlb, vchg;    // the recount bound (GX_CDLP_BOUND)
    DBuf<int> hvalid;
    DBuf<int32_t> redo;         // k_cdlp_sparse_group's vertices for the 16K-slot instance
    DBuf<unsigned int> rcnt;    // one redo count per iteration
    ~CdlpCache() {
        if (hflag) (void)hipHostFree(hflag);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

// Relabel one CSR of the graph by perm into (rp, ci).
int cdlp_relabel_csr(const DevCSR &M, int64_t n, const int32_t *perm, DBuf<int64_t> &rp, DBuf<int32_t> &ci,
                     hipStream_t s) {
    GX_TRY(rp.alloc(n + 1));
    GX_TRY(ci.alloc(M.nnz, 16));
    DBuf<uint64_t> keys, scratch;
    GX_TRY(keys.alloc(M.nnz));
    GX_TRY(scratch.alloc(M.nnz));
    if (M.nnz) {
        hipLaunchKernelGGL(k_cdlp_permute_keys, dim3(grid_for((M.nnz + 15) / 16, 256, 1u << 30)), dim3(256), 0, s,
                           M.rp.p, M.ci.p, n, (int64_t)M.nnz, perm, keys.p);
        GX_TRY(check_launch("k_cdlp_permute_keys"));
    }
    GX_TRY(sort_keys_to_csr(keys, scratch, M.nnz, n, rp.p, ci.p, s));
    GX_HIP_TRY(hipStreamSynchronize(s));   // keys die at return
    return GX_SUCCESS;
}

// Hub-first order by total degree (out + in), ties by id: the most gathered labels share the
// first lines of the label array (the PageRank plan's order, gx_pr.hip hub_order).
int cdlp_relabel(gx_graph *g, CdlpCache &C, hipStream_t s) {
    const int64_t n = (int64_t)g->n;
    std::vector<int64_t> deg(n);
    int64_t maxd = 0;
    for (int64_t v = 0; v < n; v++) {
        deg[v] = g->A.h_rp[v + 1] - g->A.h_rp[v];
        if (g->directed) deg[v] += g->AT.h_rp[v + 1] - g->AT.h_rp[v];
        maxd = std::max(maxd, deg[v]);
    }
    std::vector<int64_t> start((size_t)maxd + 2, 0);
    for (int64_t v = 0; v < n; v++) start[(size_t)(maxd - deg[v]) + 1]++;
    for (size_t k = 1; k < start.size(); k++) start[k] += start[k - 1];
    std::vector<int32_t> order(n), perm(n);
    for (int64_t v = 0; v < n; v++) {
        const int64_t pos = start[(size_t)(maxd - deg[v])]++;
        order[pos] = (int32_t)v;
        perm[v] = (int32_t)pos;
    }
    auto new_rp = [&](const HostRowPtr &h, std::vector<int64_t> &out) {
        out.assign(n + 1, 0);
        for (int64_t i = 0; i < n; i++) out[i + 1] = out[i] + (h[order[i] + 1] - h[order[i]]);
    };
    new_rp(g->A.h_rp, C.h_rpA);
    if (g->directed) new_rp(g->AT.h_rp, C.h_rpT);
    GX_TRY(C.order.alloc(n));
    GX_TRY(C.perm.alloc(n));
    GX_HIP_TRY(hipMemcpyAsync(C.order.p, order.data(), n * 4, hipMemcpyHostToDevice, s));
    GX_HIP_TRY(hipMemcpyAsync(C.perm.p, perm.data(), n * 4, hipMemcpyHostToDevice, s));
    GX_TRY(cdlp_relabel_csr(g->A, n, C.perm.p, C.rpA, C.ciA, s));
    if (g->directed) GX_TRY(cdlp_relabel_csr(g->AT, n, C.perm.p, C.rpT, C.ciT, s));
    C.G.rpA = C.rpA.p;
    C.G.ciA = C.ciA.p;
    C.G.h_rpA = C.h_rpA.data();
    if (g->directed) {
        C.G.rpT = C.rpT.p;
        C.G.ciT = C.ciT.p;
        C.G.h_rpT = C.h_rpT.data();
    }
    return GX_SUCCESS;
}

// The own-label check's layout of one CSR (k_keep_layout).
int keep_layout(const int64_t *rp, int64_t n, int64_t nnz, const int64_t *rpA, const int64_t *rpT, CdlpCache::KeepCsr &K,
                hipStream_t s) {
    const int64_t nslabs = (nnz + kWave - 1) / kWave;
    const size_t padded = (size_t)((nslabs + kKeepPad - 1) / kKeepPad * kKeepPad + kKeepPad);
    GX_TRY(K.bits.alloc(padded));
    GX_TRY(K.sne.alloc(padded));
    GX_TRY(K.ne.alloc((size_t)std::max<int64_t>(n, 1)));
    GX_HIP_TRY(hipMemsetAsync(K.bits.p, 0, padded * 8, s));
    GX_HIP_TRY(hipMemsetAsync(K.sne.p, 0, padded * 4, s));
    GX_HIP_TRY(hipMemsetAsync(K.ne.p, 0, (size_t)std::max<int64_t>(n, 1) * 4, s));
    if (n == 0 || nnz == 0) return GX_SUCCESS;
    DBuf<int64_t> flag, pos;
    GX_TRY(flag.alloc(n));
    GX_TRY(pos.alloc(n));
    hipLaunchKernelGGL(k_keep_flags, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, rp, n, flag.p);
    GX_TRY(check_launch("k_keep_flags"));
    GX_TRY(scan_exclusive_i64(flag.p, pos.p, (size_t)n, s));
    hipLaunchKernelGGL(k_keep_layout, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, rp, n, pos.p, rpA, rpT, K.ne.p,
                       K.bits.p, K.sne.p);
    GX_TRY(check_launch("k_keep_layout"));
    GX_HIP_TRY(hipStreamSynchronize(s));   // flag / pos die at return
    return GX_SUCCESS;
}

// The column-sorted blocks of one CSR (host row pointers h_rp, device rp / ci): the rows of
// total degree > kTiny in order, cut greedily into blocks of <= kKeepBlock entries whose rows
// span <= kKeepRows positions (a row of kKeepBlock or more entries takes whole blocks of its own).
int keep_sorted_build(const CdlpGraph &G, const int64_t *h_rp, const int64_t *rp, const int32_t *ci,
                      CdlpCache::KeepCsr &K, hipStream_t s) {
    const char *kb = std::getenv("GX_CDLP_KEEP_BLOCK");
    const int64_t kKeepBlock = kb ? std::min<int64_t>(kKeepBlockMax, std::max<int64_t>(1024, std::atoll(kb))) : 65536;
    std::vector<int32_t> rows, rblk, brow0;
    std::vector<int64_t> kpos, bsize;
    int64_t m = 0, cur_e = 0;
    bool open = false;
    for (int64_t v = 0; v < G.n; v++) {
        const int64_t dt = (G.h_rpA[v + 1] - G.h_rpA[v]) + (G.directed ? G.h_rpT[v + 1] - G.h_rpT[v] : 0);
        const int64_t d = h_rp[v + 1] - h_rp[v];
        if (dt <= kTiny || d == 0) continue;
        if (d >= kKeepBlock) {
            rows.push_back((int32_t)v);
            kpos.push_back(m);
            rblk.push_back((int32_t)brow0.size());
            for (int64_t k = 0; k < d; k += kKeepBlock) {
                brow0.push_back((int32_t)v);
                bsize.push_back(std::min(kKeepBlock, d - k));
            }
            m += d;
            open = false;
            continue;
        }
        if (!open || cur_e + d > kKeepBlock || v - brow0.back() >= kKeepRows) {
            brow0.push_back((int32_t)v);
            bsize.push_back(0);
            cur_e = 0;
            open = true;
        }
        rows.push_back((int32_t)v);
        kpos.push_back(m);
        rblk.push_back((int32_t)brow0.size() - 1);
        bsize.back() += d;
        cur_e += d;
        m += d;
    }
    K.nb = (int64_t)brow0.size();
    if (m == 0 || K.nb >= (1ll << 31)) {
        K.nb = 0;
        return GX_SUCCESS;
    }
    std::vector<int64_t> bstart(brow0.size() + 1, 0);
    for (size_t b = 0; b < bsize.size(); b++) bstart[b + 1] = bstart[b] + bsize[b];

    DBuf<int32_t> d_rows, d_rblk;
    DBuf<int64_t> d_kpos;
    DBuf<uint64_t> keys, keys2;
    DBuf<uint16_t> vals;
    GX_TRY(d_rows.alloc(rows.size()));
    GX_TRY(d_rblk.alloc(rblk.size()));
    GX_TRY(d_kpos.alloc(kpos.size()));
    GX_TRY(K.brow0.alloc(brow0.size()));
    GX_TRY(K.bstart.alloc(bstart.size()));
    GX_HIP_TRY(hipMemcpyAsync(d_rows.p, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, s));
    GX_HIP_TRY(hipMemcpyAsync(d_rblk.p, rblk.data(), rblk.size() * 4, hipMemcpyHostToDevice, s));
    GX_HIP_TRY(hipMemcpyAsync(d_kpos.p, kpos.data(), kpos.size() * 8, hipMemcpyHostToDevice, s));
    GX_HIP_TRY(hipMemcpyAsync(K.brow0.p, brow0.data(), brow0.size() * 4, hipMemcpyHostToDevice, s));
    GX_HIP_TRY(hipMemcpyAsync(K.bstart.p, bstart.data(), bstart.size() * 8, hipMemcpyHostToDevice, s));
    GX_TRY(keys.alloc((size_t)m));
    GX_TRY(keys2.alloc((size_t)m));
    GX_TRY(vals.alloc((size_t)m));
    GX_TRY(K.srow.alloc((size_t)m));
    hipLaunchKernelGGL(k_keep_sorted_keys, dim3(grid_for((uint64_t)rows.size() * kWave, 256, 16384)), dim3(256), 0, s,
                       rp, ci, d_rows.p, d_kpos.p, d_rblk.p, K.brow0.p, (int64_t)rows.size(), kKeepBlock, keys.p,
                       vals.p);
    GX_TRY(check_launch("k_keep_sorted_keys"));
    int end_bit = 32;
    while ((1ll << (end_bit - 32)) < K.nb) end_bit++;
    GX_TRY(sort_pairs_u64_u16(keys.p, keys2.p, vals.p, K.srow.p, (size_t)m, end_bit, s));
    keys.release();
    vals.release();
    GX_TRY(K.scol.alloc((size_t)m));
    hipLaunchKernelGGL(k_keep_sorted_cols, dim3(grid_for((uint64_t)m, 256, 8192)), dim3(256), 0, s, keys2.p, m, K.scol.p);
    GX_TRY(check_launch("k_keep_sorted_cols"));
    GX_HIP_TRY(hipStreamSynchronize(s));   // host vectors and the key buffers die at return
    return GX_SUCCESS;
}

int keep_build(CdlpCache &C, hipStream_t s) {
    const CdlpGraph &G = C.G;
    // the sorted blocks cost a device sort of the entries (~7 ms on SYN-7_5) and save ~0.1 ms
    // per call: built with the relabelled copy, i.e. once the graph serves a second CDLP run
    if (C.relabel && G.h_rpA && (!G.directed || G.h_rpT) && env_on("GX_CDLP_KEEP_SORTED")) {
        GX_TRY(keep_sorted_build(G, G.h_rpA, G.rpA, G.ciA, C.kA, s));
        if (G.directed) GX_TRY(keep_sorted_build(G, G.h_rpT, G.rpT, G.ciT, C.kT, s));
        C.keep_sorted = true;
    }
    GX_TRY(keep_layout(G.rpA, G.n, G.nnzA, G.rpA, G.rpT, C.kA, s));
    if (G.directed) GX_TRY(keep_layout(G.rpT, G.n, G.nnzT, G.rpA, G.rpT, C.kT, s));
    GX_TRY(C.kcnt.alloc((size_t)std::max<int64_t>(G.n, 1)));
    GX_HIP_TRY(hipMemsetAsync(C.kcnt.p, 0, (size_t)std::max<int64_t>(G.n, 1) * 4, s));
    GX_TRY(C.kflags.alloc(2));
    GX_HIP_TRY(hipMemsetAsync(C.kflags.p, 0, 2 * sizeof(int), s));
    C.keep_nnzA = G.nnzA;
    C.keep_nnzT = G.directed ? G.nnzT : 0;
    if (C.relabel && G.h_rpA && (!G.directed || G.h_rpT)) {
        auto deg = [&](int64_t i) {
            return (G.h_rpA[i + 1] - G.h_rpA[i]) + (G.directed ? G.h_rpT[i + 1] - G.h_rpT[i] : 0);
        };
        int64_t lo = 0, hi = G.n;   // the first position of degree <= kTiny (degrees non-increasing)
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo) / 2;
            if (deg(mid) > kTiny) lo = mid + 1;
            else hi = mid;
        }
        C.keep_nnzA = G.h_rpA[lo];
        if (G.directed) C.keep_nnzT = G.h_rpT[lo];
    }
    C.keep_built = true;
    return GX_SUCCESS;
}

// The staging plan: every entry's column, sorted within kStageBlock-entry blocks, and its
// position in the block.
int cdlp_cache(gx_graph *g, int iters, bool relabel, CdlpCache **out, hipStream_t s) {
    const int64_t n = (int64_t)g->n;
    auto *C = static_cast<CdlpCache *>(g->cdlp.get());
    if (C && C->relabel != relabel) {
        g->cdlp.reset();   // GX_CDLP_RELABEL changed between calls
        C = nullptr;
    }
    if (!C) {
        auto fresh = std::make_shared<CdlpCache>();
        fresh->relabel = relabel;
        GX_TRY(ensure_host_rp(g->ctx, g->A));
        fresh->G = cdlp_view(g);
        if (relabel) GX_TRY(cdlp_relabel(g, *fresh, s));
        GX_TRY(cdlp_plan(fresh->G, 0, n, fresh->P, s));
        GX_TRY(fresh->la.alloc(n));
        GX_TRY(fresh->lb.alloc(n));
        GX_TRY(fresh->act.alloc(n));
        fresh->sub = std::max<int64_t>(16, n / 32 / kCdlpSubs);   // entries per sub-list
        GX_TRY(fresh->clist.alloc((size_t)fresh->sub * kCdlpSubs));
        // active vertices per shard and list (GX_CDLP_ASUB: a test's small capacity, so lists overflow)
        fresh->asub = std::max<int64_t>(16, n / 8 / kCdlpSubs);
        if (const char *e = std::getenv("GX_CDLP_ASUB")) fresh->asub = std::max<int64_t>(1, std::atoll(e));
        GX_TRY(fresh->al.alloc((size_t)fresh->asub * kCdlpSubs * (kCdlpLists - 1)));
        GX_TRY(fresh->dense.alloc(1));
        GX_TRY(fresh->redo.alloc(std::max<size_t>(1, fresh->P.n_mid4 + fresh->P.n_mid)));
        // the caller's rows sorted (A, and A' for a directed graph): the first iteration is each
        // row's first column (undirected, k_cdlp_first_sorted) or the smallest reciprocal
        // neighbour (directed, k_cdlp_first_dir), on the caller's graph, then moved to the
        // relabelled order
        auto sorted_rows = [&](const DevCSR &M, bool *ok) -> int {
            const int64_t nnz = (int64_t)M.nnz;
            *ok = true;
            if (nnz == 0) return GX_SUCCESS;
            DBuf<uint32_t> bits;
            DBuf<int> flag;
            GX_TRY(bits.alloc((size_t)(nnz + 31) / 32));
            GX_TRY(flag.alloc(1));
            GX_HIP_TRY(hipMemsetAsync(bits.p, 0, (size_t)(nnz + 31) / 32 * 4, s));
            const int one = 1;
            GX_HIP_TRY(hipMemcpyAsync(flag.p, &one, sizeof(int), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_row_start_bits, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, M.rp.p, n, bits.p);
            GX_TRY(check_launch("k_row_start_bits"));
            hipLaunchKernelGGL(k_rows_sorted, dim3(grid_for(nnz, 256, 8192)), dim3(256), 0, s, M.ci.p, nnz, bits.p,
                               flag.p);
            GX_TRY(check_launch("k_rows_sorted"));
            int sorted = 0;
            GX_HIP_TRY(hipMemcpyAsync(&sorted, flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            *ok = sorted != 0;
            return GX_SUCCESS;
        };
        if (g->nnz > 0 && (!g->directed || g->AT.built)) {
            GX_TRY(fresh->tmp.alloc(n));
            bool okA = false, okT = true;
            GX_TRY(sorted_rows(g->A, &okA));
            if (g->directed && okA) GX_TRY(sorted_rows(g->AT, &okT));
            fresh->rows_sorted = okA && okT;
        }
        for (hipEvent_t &e : fresh->ev) GX_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        g->cdlp = fresh;
        C = fresh.get();
    }
    if (iters > C->cap_iters) {
        const int cap = std::max(iters, 16);
        GX_TRY(C->changed.alloc((size_t)cap * kFlagShards * kFlagStride));
        GX_TRY(C->ccount.alloc((size_t)cap * kCdlpLists * kCdlpSubs * kCntStride));
        GX_TRY(C->rcnt.alloc((size_t)cap));
        if (C->hflag) (void)hipHostFree(C->hflag);
        C->hflag = nullptr;
        GX_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&C->hflag), sizeof(int) * cap, hipHostMallocMapped));
        GX_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&C->dflag), C->hflag, 0));
        C->cap_iters = cap;
    }
    *out = C;
    return GX_SUCCESS;
}
}  // namespace
}  // namespace gx

extern "C" int gx_cdlp(gx_graph *g, int iters, uint64_t *labels) {
    if (!g || !labels) return fail(GX_NULL_POINTER, "gx_cdlp: null argument");
    if (iters < 0) return fail(GX_INVALID_VALUE, "gx_cdlp: negative iteration count");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    if (n == 0) return GX_SUCCESS;
    GX_TRY(device_begin(ctx));
    if (g->directed) GX_TRY(ensure_transpose(g));
    // The relabelled copy costs ~90 ms to build on SYN-cit (4.2 M vertices) and saves ~1.3 ms
    // per call, so, like BFS's transpose, it is built once the graph serves a second CDLP run:
    // a one-off run (the Graphalytics executable's) stays in the caller's order.
    // GX_CDLP_RELABEL=0 never, 1 from the first run.
    g->cdlp_calls++;
    const char *re = std::getenv("GX_CDLP_RELABEL");
    const bool relabel = re ? std::atoi(re) != 0 : g->cdlp_calls >= 2;
    CdlpCache *C = nullptr;
    GX_TRY(cdlp_cache(g, std::max(iters, 1), relabel, &C, s));
    CdlpPlan &P = C->P;
    const CdlpGraph &G = C->G;
    GX_HIP_TRY(hipMemsetAsync(C->changed.p, 0, sizeof(int) * kFlagShards * kFlagStride * std::max(iters, 1), s));
    if (relabel) {
        // labels are the caller's vertex ids, at the relabelled positions
        GX_HIP_TRY(hipMemcpyAsync(C->la.p, C->order.p, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    } else {
        hipLaunchKernelGGL(k_cdlp_iota, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, C->la.p, n);
        GX_TRY(check_launch("k_cdlp_iota"));
    }
    // Early exit at a fixed point (LAGraph_cdlp.c:328-332), checked `lag` iterations late:
    // iteration it is queued before the host waits for iteration it-lag's flag, so the check
    // never drains the stream.  An iteration run after a fixed point changes no label.  Lag 2
    // (GX_CDLP_LAG=1: one) keeps two iterations queued: sparse iterations of ~60 us are shorter
    // than the host's launches for one.
    int *hflag = C->hflag, *dflag = C->dflag;
    hipEvent_t *ev = C->ev;
    // active set (GX_CDLP_ACTIVE=0: every vertex every iteration): from iteration 2 on, the
    // changes of the last iteration are listed (up to n / 32 of them) and their neighbours
    // marked with the iteration's stamp before the tier kernels run
    const bool use_active = env_on("GX_CDLP_ACTIVE");
    const bool active = use_active && iters > 2;
    // GX_CDLP_FIRST_SORTED=0: the first iteration by the tier kernels even when rows are sorted
    const bool first_sorted = env_on("GX_CDLP_FIRST_SORTED");
    // GX_CDLP_SPARSE=0: active vertices found by the tier kernels' act checks instead of lists
    const bool use_sparse = env_on("GX_CDLP_SPARSE");
    // GX_CDLP_SPARSE_ONLY=0: tier kernels launched (and idle) in sparse iterations too; =2:
    // every active iteration sparse-only (a test of the fallback lists)
    const char *so = std::getenv("GX_CDLP_SPARSE_ONLY");
    const int sparse_only = !use_sparse ? 0 : so ? std::atoi(so) : 1;
    const char *lg = std::getenv("GX_CDLP_LAG");
    const int lag = lg && std::atoi(lg) == 1 ? 1 : 2;
    const int64_t sub = C->sub;
    // GX_CDLP_KEEP=0: a dense active iteration runs the tier kernels over every vertex instead
    // of the own-label check
    const bool keep = active && use_sparse && env_on("GX_CDLP_KEEP");
    if (keep && !C->keep_built) GX_TRY(keep_build(*C, s));
    if (active) {
        hipLaunchKernelGGL(k_cdlp_fill_u32, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s,
                           reinterpret_cast<uint32_t *>(C->act.p), 0xffffffffu, n);   // stamp -1: never active
        GX_TRY(check_launch("k_cdlp_fill_u32"));
        GX_HIP_TRY(hipMemsetAsync(C->ccount.p, 0, sizeof(unsigned int) * kCdlpLists * kCdlpSubs * kCntStride * iters, s));
        GX_HIP_TRY(hipMemsetAsync(C->rcnt.p, 0, sizeof(unsigned int) * iters, s));
    }
    // the recount bound (GX_CDLP_BOUND=0: off): an active iteration skips the vertices whose
    // label provably keeps a strict majority
    CdlpBound bound{nullptr, nullptr, nullptr};
    if (env_on("GX_CDLP_BOUND")) {
        if (C->vlb.n < (size_t)n) {
            GX_TRY(C->vlb.alloc(n));
            GX_TRY(C->vchg.alloc(n));
            GX_TRY(C->hvalid.alloc(1));
            GX_HIP_TRY(hipMemsetAsync(C->vlb.p, 0, (size_t)n * 4, s));
            GX_HIP_TRY(hipMemsetAsync(C->vchg.p, 0, (size_t)n * 4, s));
            GX_HIP_TRY(hipMemsetAsync(C->hvalid.p, 0, sizeof(int), s));
        }
        bound = CdlpBound{C->vlb.p, C->vchg.p, C->hvalid.p};
    }
    const CdlpBound *bd = bound.vlb ? &bound : nullptr;
    int32_t *cur = C->la.p, *nxt = C->lb.p;
    for (int it = 0; it < iters; it++) {
        int *changed = C->changed.p + (size_t)it * kFlagShards * kFlagStride;
        if (active && it >= 2) {
            // nxt still holds the input of iteration it-1, cur its output
            unsigned int *cnt = C->ccount.p + (size_t)it * kCdlpLists * kCdlpSubs * kCntStride;
            {
                KTimer kt(ctx, "cdlp_mark", s);
                hipLaunchKernelGGL(k_cdlp_changed, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, nxt, cur, G.rpA,
                                   G.rpT, n, C->clist.p, sub, cnt, C->dense.p);
                GX_TRY(check_launch("k_cdlp_changed"));
                // 32 waves per shard of the change list (the grid must be a multiple of kCdlpSubs waves)
                hipLaunchKernelGGL(k_cdlp_mark, dim3(8 * kCdlpSubs), dim3(kCdlpSubs), 0, s, G.rpA, G.ciA, G.rpT, G.ciT,
                                   C->clist.p, sub, cnt, C->act.p, (int32_t)it, C->dense.p, C->al.p, C->asub,
                                   bd ? bd->vchg : nullptr, bd ? bd->hvalid : nullptr);
                GX_TRY(check_launch("k_cdlp_mark"));
            }
            // sparse-only (no idle tier launches, ~60 us per iteration on SYN-7_5) when iteration
            // it-1-lag, the last whose flags the host has seen, did not overflow its lists: changes
            // shrink as labels settle.  A wrong guess costs the fallback lists' full pass.
            const bool only = sparse_only == 2 || (sparse_only == 1 && it >= 3 + lag && (hflag[it - 1 - lag] & 2) == 0);
            // the own-label check where the iteration may be dense (in a sparse-only one its three
            // idle launches cost more than the rare dense case's fallback pass)
            int *kf = keep && (!only || sparse_only == 2) ? C->kflags.p : nullptr;
            if (kf) {
                KTimer kk(ctx, "cdlp_keep", s);
                // counts of the own label among each vertex's neighbours (exit unless *dense)
                // one wave per U slabs (the count kernel exits unless *dense); GX_CDLP_KEEP_U = 8 / 16 / 32
                const char *ku = std::getenv("GX_CDLP_KEEP_U");
                const int U = ku ? std::atoi(ku) : 16;
                auto count = [&](const int32_t *ci, int64_t nnz_, const CdlpCache::KeepCsr &K, int head) {
                    const unsigned grid = grid_for(
                        (uint64_t)std::max<int64_t>(1, (nnz_ + (int64_t)kWave * U - 1) / ((int64_t)kWave * U)) * kWave, 256,
                        16384);
                    const auto kern = U == 8 ? k_cdlp_keep_count<8> : U == 32 ? k_cdlp_keep_count<32> : k_cdlp_keep_count<16>;
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, ci, nnz_, K.bits.p, K.sne.p, K.ne.p, cur,
                                       C->kcnt.p, C->dense.p, kf, cnt + kCdlpSubs * kCntStride, head);
                    return check_launch("k_cdlp_keep_count");
                };
                auto sorted = [&](const CdlpCache::KeepCsr &K, int head) {
                    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(K.nb, 65536));
                    hipLaunchKernelGGL(k_cdlp_keep_sorted, dim3(grid), dim3(256), 0, s, K.bstart.p, K.brow0.p, K.nb,
                                       K.scol.p, K.srow.p, cur, n, C->kcnt.p, C->dense.p, kf,
                                       cnt + kCdlpSubs * kCntStride, head);
                    return check_launch("k_cdlp_keep_sorted");
                };
                if (C->keep_sorted && env_on("GX_CDLP_KEEP_SORTED")) {
                    GX_TRY(sorted(C->kA, 1));
                    if (G.directed) GX_TRY(sorted(C->kT, 0));
                } else {
                    GX_TRY(count(G.ciA, C->keep_nnzA, C->kA, 1));
                    if (G.directed) GX_TRY(count(G.ciT, C->keep_nnzT, C->kT, 0));
                }
                hipLaunchKernelGGL(k_cdlp_keep_apply, dim3(8 * kCdlpSubs), dim3(256), 0, s, G.rpA, G.rpT, (int64_t)0, n,
                                   C->kcnt.p, C->act.p, (int32_t)it, kf, cnt, C->al.p, C->asub, kf + 1,
                                   bd ? bd->vlb : nullptr, bd ? bd->vchg : nullptr);
                GX_TRY(check_launch("k_cdlp_keep_apply"));
                hipLaunchKernelGGL(k_cdlp_keep_finish, dim3(1), dim3(1), 0, s, C->dense.p, kf, kf + 1);
                GX_TRY(check_launch("k_cdlp_keep_finish"));
            }
            const SparseLists sl{C->al.p, C->asub, cnt, only, C->redo.p, C->rcnt.p + it};
            GX_TRY(cdlp_iteration(G, P, cur, nxt, changed, s, C->act.p, (int32_t)it, C->dense.p, false,
                                  use_sparse ? &sl : nullptr, kFlagShards, kf, bd));
        } else if (it == 0 && C->rows_sorted && first_sorted) {
            // on the caller's graph and vertex order (whose rows the check found sorted)
            KTimer kt(ctx, "cdlp_first", s);
            int32_t *out = relabel ? C->tmp.p : nxt;
            if (g->directed) {
                // GX_CDLP_FIRST_SMALL = 4 / 8 (default) / 16: the longest row one lane compares
                // (SYN-cit: 32 ran 0.43 ms, 16 0.20, 8 0.185)
                const char *fs = std::getenv("GX_CDLP_FIRST_SMALL");
                const int small = fs ? std::atoi(fs) : 8;
                const auto kern = small == 4 ? k_cdlp_first_dir<4> : small == 16 ? k_cdlp_first_dir<16> : k_cdlp_first_dir<8>;
                // GX_CDLP_FIRST_MED: rows up to this many entries merged by 16-lane groups (0: off;
                // SYN-cit first pass 0.174 ms off, 0.150 at 32, 0.158 at 64, 0.170 at 128)
                const char *fm = std::getenv("GX_CDLP_FIRST_MED");
                const int med = fm ? std::atoi(fm) : 32;
                // one wave per 64 vertices, no grid-stride trips (SYN-cit: 0.147 ms against 0.150
                // with 8192 blocks, 0.157 with 2048)
                hipLaunchKernelGGL(kern, dim3(grid_for(n, 256)), dim3(256), 0, s, g->A.rp.p, g->A.ci.p, g->AT.rp.p,
                                   g->AT.ci.p, n, out, changed, kFlagShards, med);
                GX_TRY(check_launch("k_cdlp_first_dir"));
            } else {
                hipLaunchKernelGGL(k_cdlp_first_sorted, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, g->A.rp.p,
                                   g->A.ci.p, (int64_t)0, n, out, changed, kFlagShards);
                GX_TRY(check_launch("k_cdlp_first_sorted"));
            }
            if (relabel) {   // nxt[p] = result of the caller's vertex order[p]
                hipLaunchKernelGGL(k_cdlp_gather_i32, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, C->tmp.p,
                                   C->order.p, n, nxt);
                GX_TRY(check_launch("k_cdlp_gather_i32"));
            }
        } else {
            // iteration 0: labels are the caller's vertex ids.  The smallest-neighbour shortcut
            // (`first`) assumes no row repeats a column; k_rows_sorted found the caller's rows
            // strictly ascending, i.e. duplicate-free (else the counting path runs).
            GX_TRY(cdlp_iteration(G, P, cur, nxt, changed, s, nullptr, 0, nullptr, it == 0 && C->rows_sorted, nullptr,
                                  kFlagShards, nullptr, bd));
        }
        hipLaunchKernelGGL(k_cdlp_flag_out, dim3(1), dim3(kWave), 0, s, changed, kFlagShards,
                           active && it >= 2 ? C->dense.p : nullptr, dflag + it);
        GX_TRY(check_launch("k_cdlp_flag_out"));
        GX_HIP_TRY(hipEventRecord(ev[it % 3], s));
        std::swap(cur, nxt);
        if (it >= lag) {
            GX_HIP_TRY(hipEventSynchronize(ev[(it - lag) % 3]));
            if (!(hflag[it - lag] & 1)) break;   // iteration it-lag was a fixed point, so is cur
        }
    }
    if (relabel) {   // back to the caller's vertex order
        hipLaunchKernelGGL(k_cdlp_gather_i32, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, cur, C->perm.p, n, nxt);
        GX_TRY(check_launch("k_cdlp_gather_i32"));
        cur = nxt;
    }
    GX_TRY(device_end(ctx));
    GX_TRY(download(ctx, labels, cur, (uint64_t)n, Xfer::Widen32));
    return GX_SUCCESS;
}

// ---- partitioned CDLP (one rank's vertex range; the caller exchanges labels) ----
struct gx_cdlp_part {
    gx_graph *g = nullptr;
    gx::CdlpPlan plan;
};

extern "C" int gx_cdlp_part_create(gx_graph *g, uint64_t v0, uint64_t v1, gx_cdlp_part **part) {
    if (!g || !part) return fail(GX_NULL_POINTER, "gx_cdlp_part_create: null argument");
    if (v0 > v1 || v1 > g->n) return fail(GX_INVALID_INDEX, "gx_cdlp_part_create: bad vertex range");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    if (g->directed) GX_TRY(ensure_transpose(g));
    GX_TRY(ensure_host_rp(g->ctx, g->A));
    auto p = std::make_unique<gx_cdlp_part>();
    p->g = g;
    GX_TRY(cdlp_plan(cdlp_view(g), (int64_t)v0, (int64_t)v1, p->plan, g->ctx->stream));
    *part = p.release();
    return GX_SUCCESS;
}

extern "C" int gx_cdlp_part_init(gx_cdlp_part *part, int32_t *labels, void *stream) {
    if (!part || !labels) return fail(GX_NULL_POINTER, "gx_cdlp_part_init: null argument");
    gx_graph *g = part->g;
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the null stream (torch's default)
    if (g->n) {
        hipLaunchKernelGGL(k_cdlp_iota, dim3(grid_for(g->n, 256, 8192)), dim3(256), 0, s, labels, (int64_t)g->n);
        GX_TRY(check_launch("k_cdlp_iota"));
    }
    return GX_SUCCESS;
}

extern "C" int gx_cdlp_part_step(gx_cdlp_part *part, const int32_t *labels, int32_t *next, int *changed,
                                 void *stream) {
    if (!part || !labels || !next || !changed) return fail(GX_NULL_POINTER, "gx_cdlp_part_step: null argument");
    gx_graph *g = part->g;
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the null stream (torch's default)
    return cdlp_iteration(cdlp_view(g), part->plan, labels, next, changed, s);
}

extern "C" int gx_cdlp_part_free(gx_cdlp_part *part) {
    delete part;
    return GX_SUCCESS;
}

GX_MODULE_WARMER(cdlp)
