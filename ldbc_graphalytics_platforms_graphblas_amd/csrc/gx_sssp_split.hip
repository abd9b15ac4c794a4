// gx_sssp_split.hip -- SSSP on a 1-D split of the vertices (config 4: datagen-8_5-fb,
// 8 GPUs, 1-D partition + RCCL all-gather).  Replaces LA_SSSP's delta-stepping
// (sssp.cpp:53-81) for a rank that owns the targets [v0, v1).
//
// Layout per rank: the edges u -> v of the whole graph whose target v is owned, by source
// (CSR over all n sources), light edges (w < delta) first.  The distance vector is replicated:
// every rank holds dist[n] and applies every improvement, so every rank takes the same
// scheduling decisions from the same counts.
//
// Round (bulk synchronous, delta-stepping after Meyer & Sanders; the bucket ring, fusion and
// pulled heavy phase of gx_sssp.hip restated for replicated state):
//   plan   one thread, from the replicated counts only: LIGHT (relax the frontier queued last
//          round), HEAVY / PULL (the heavy edges of the vertices settled since the last time:
//          pushed, or -- undirected, batch >= 1/8 of the vertices with edges -- pulled by the
//          owned vertices above fl(min settled distance + delta)), ADVANCE (open the next
//          non-empty slot of the 32-bucket ring, fused with the following ones while they hold
//          <= n/16 vertices), SPLIT (the overflow into a new ring window) or done;
//   prep   ADVANCE: the opened slots' pending vertices -> this round's frontier; SPLIT: the
//          overflow -> ring / new overflow; HEAVY / PULL: the batch marked (PULL: its minimum);
//   relax  up to 64 (vertex, 256-edge chunk) items of this rank's slice per wave; PULL: the
//          owned vertices a batch neighbour could still improve, a thread each (a wave for
//          rows past 32 heavy in-edges); a target whose distance drops is claimed once;
//   pairs  (vertex, distance bits) of the improved owned vertices + {count, done};
//   -- the caller all-gathers the pairs of every rank (gx_sssp_split_run: one rank, none) --
//   apply  every rank's pairs: dist = min, then the vertex joins the next frontier when its
//          bucket is <= cur (and the epoch's settled set), else its ring slot or the overflow.
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
constexpr int kW = 32;          // bucket ring slots
constexpr int kSmallDeg = 32;   // PULL: candidates up to this many heavy in-edges take a thread
constexpr int kBigCap = 1024;   // PULL: larger candidates listed per workgroup for its waves
constexpr unsigned long long kInf = 0x7FF0000000000000ull;   // +inf bits

enum : int32_t { kNone = 0, kLight = 1, kHeavy = 2, kAdvance = 3, kPull = 4, kSplit = 5 };

// Replicated decision state (identical on every rank after every apply) + this rank's item
// counters (which differ by rank and never enter a decision).
struct SplitState {
    int64_t cur;                  // last bucket of the group being settled
    int64_t win_base;             // ring window [win_base, win_base + kW)
    unsigned long long ovf_minb;  // smallest bucket on the overflow list being filled
    unsigned long long smin;      // PULL: smallest distance of the settled batch
    int32_t mode, round, epoch, done;
    int32_t epoch_round;          // round that opened the current epoch
    int32_t fc;                   // frontier list relaxed this round (LIGHT / ADVANCE)
    int32_t oe;                   // overflow list being filled; SPLIT reads oe ^ 1
    int32_t ostamp_tag;           // overflow dedupe tag (one per overflow generation)
    int32_t slot0, nslots;        // ADVANCE: ring slots opened
    int32_t consume, consume_n;   // ring slots to clear at the next plan
    uint32_t fv[2], fi[2];        // frontier vertices (replicated) / items (rank-local)
    uint32_t sv, sv_done;         // settled vertices of this epoch / heavy-relaxed so far
    uint32_t si, si_done;         // their heavy items (rank-local) / relaxed so far
    uint32_t hs0, hs1;            // HEAVY: items [hs0, hs1); HEAVY / PULL: vertices [sb0, sb1)
    uint32_t sb0, sb1;
    uint32_t ring_cnt[kW];
    uint32_t ovf_cnt[2];
    uint32_t nimp;                // improved owned vertices this round (rank-local)
    uint32_t pull_min;            // settled batch size from which the heavy phase is pulled (0: never)
    uint32_t fuse;                // ADVANCE opens further slots while the vertices stay <= fuse
    uint32_t nmode[6];            // rounds per mode (GX_SPLIT_VERBOSE)
    unsigned long long nitems[6]; // items / candidates per mode (rank-local)
    int8_t modelog[256];          // mode of rounds 1..256 (GX_SPLIT_VERBOSE)
    // The settled list is a ring (sverts: vertices, sitems: items; positions taken modulo the
    // capacity): a vertex re-settled in its epoch is listed again, so an epoch may list more
    // than n.  Only [sv_done, sv) is live when a round writes (a heavy round reads its batch
    // in prep / relax, before its apply lists anything), and a vertex is listed at most once
    // between two heavy phases, so n vertices and their items always fit.  Should
    // a write ever land on live entries, it is dropped, the run stops and err is set, which
    // the host turns into an error instead of returning distances.
    uint32_t sv_cap;
    uint64_t si_cap;
    int32_t err;
};

// Per-vertex records, one 16-B line each: the slice row (light entries [start, start + nl),
// heavy [start + nl, start + nl + nh)), and the vertex's stamps.
struct alignas(16) VRec {
    int64_t start;
    uint32_t nl, nh;
};
struct alignas(16) SRec {
    int32_t sstamp;   // epoch v joined the settled set
    int32_t hmark;    // round of the HEAVY / PULL phase that relaxed v's heavy edges (0: pending)
    int32_t bstamp;   // bucket v was last put into a ring slot for (low 32 bits + 1)
    int32_t ostamp;   // overflow tag v was last put on the overflow with
};

struct SplitBufs {
    const VRec *vrec;
    const int32_t *sci;           // owned target - v0
    const double *sw;
    const int64_t *orp;           // owned rows' heavy in-edges (PULL; undirected graphs)
    const int32_t *oci;
    const double *ow;
    unsigned long long *dist;     // replicated distances (fp64 bits)
    unsigned long long *lrel;     // distance v's light edges were queued for relaxing with
    SRec *srec;
    int32_t *qstamp;              // ADVANCE: round v was taken from the ring
    int32_t *istamp;              // round an owned vertex was last claimed as improved
    uint64_t *fitems[2];          // (u << 32 | chunk)
    uint64_t *sitems;             // heavy items of the settled vertices
    int32_t *sverts;              // settled vertices of the epoch (replicated set)
    int32_t *ring;                // kW slots of n vertices
    int32_t *ovf[2];
    int32_t *imp;                 // improved owned vertices (global ids)
    int64_t n, v0, v1;
    double delta, inv_delta;
    SplitState *st;
};

__device__ __forceinline__ int64_t sbucket(unsigned long long bits, double inv_delta) {
    const double q = __longlong_as_double((long long)bits) * inv_delta;
    return q < 4.0e18 ? (int64_t)q : (int64_t)4000000000000000000ll;
}

__device__ __forceinline__ uint32_t nchunks(int64_t len) { return (uint32_t)max<int64_t>(1, (len + kSChunk - 1) / kSChunk); }

// ---- tile reservations ----
// A kernel that queues vertices works in tiles of kSB * kPer elements per workgroup: each element
// takes its offsets inside the tile from LDS atomics, then one thread per queue reserves the
// tile's range with one global atomic.  A shared counter then sees one atomic per queue and
// tile instead of one per wave (same-address atomics serialise at ~11-20 ns each: the first
// version of this file spent most of its time there).
constexpr int kPer = 8;                    // elements per thread and tile
enum : int { kQFv = 0, kQFi, kQSv, kQSi, kQOvf, kQRing, kQCat = kQRing + kW };

// elements per thread for `tot` elements over the grid: the full kPer only when the input
// fills every workgroup's tiles (a small input on few workgroups would run kPer dependent
// element chains per thread in series)
__device__ __forceinline__ uint32_t tile_per(uint64_t tot) {
    const uint64_t per = (tot + (uint64_t)gridDim.x * kSB - 1) / ((uint64_t)gridDim.x * kSB);
    return (uint32_t)max<uint64_t>(1, min<uint64_t>(kPer, per));
}

struct Tile {
    uint32_t cnt[kQCat];
    uint32_t base[kQCat];
    unsigned long long ominb;
};

// One element's pushes: the frontier (with its light items) and the settled set (with its
// heavy items) for `take`; the ring slot or overflow for `far`.
struct Push {
    int32_t v;
    uint32_t nl, offi, nh, offs, offsv, offr;
    int8_t isv, q;   // q: -1 none, kQOvf, or kQRing + slot
    uint8_t take;
};

__device__ __forceinline__ void tile_begin(Tile &T) {
    for (int c = threadIdx.x; c < kQCat; c += kSB) T.cnt[c] = 0;
    if (threadIdx.x == 0) T.ominb = ~0ull;
    __syncthreads();
}

// Stage element v (distance d): frontier/settled when take, ring/overflow (bucket b) when far.
__device__ __forceinline__ void tile_stage(const SplitBufs &B, Tile &T, Push &P, bool take, bool far, int64_t v,
                                           unsigned long long d, int64_t b, int32_t epoch) {
    const SplitState *st = B.st;
    P.v = (int32_t)v;
    P.take = take;
    P.isv = 0;
    P.q = -1;
    P.nl = P.nh = 0;
    if (!take && !far) return;
    SRec r = B.srec[v];
    if (take) {
        B.lrel[v] = d;
        const VRec vr = B.vrec[v];
        P.nl = nchunks(vr.nl);
        atomicAdd(&T.cnt[kQFv], 1u);
        P.offi = atomicAdd(&T.cnt[kQFi], P.nl);
        if (r.sstamp != epoch || r.hmark >= st->epoch_round) {
            B.srec[v].sstamp = epoch;
            B.srec[v].hmark = 0;
            P.isv = 1;
            P.nh = nchunks(vr.nh);
            P.offsv = atomicAdd(&T.cnt[kQSv], 1u);
            P.offs = atomicAdd(&T.cnt[kQSi], P.nh);
        }
    }
    if (far) {
        if (b < st->win_base + kW) {
            const int32_t btag = (int32_t)(uint32_t)b + 1;
            if (r.bstamp != btag) {
                B.srec[v].bstamp = btag;
                P.q = (int8_t)(kQRing + (int)(b % kW));
                P.offr = atomicAdd(&T.cnt[P.q], 1u);
            }
        } else {
            // the bound counts every overflow vertex, also one already listed whose bucket dropped
            atomicMin(&T.ominb, (unsigned long long)b);
            if (r.ostamp != st->ostamp_tag) {
                B.srec[v].ostamp = st->ostamp_tag;
                P.q = kQOvf;
                P.offr = atomicAdd(&T.cnt[kQOvf], 1u);
            }
        }
    }
}

__device__ __forceinline__ uint32_t *tile_counter(SplitState *st, int c, int list) {
    switch (c) {
    case kQFv: return &st->fv[list];
    case kQFi: return &st->fi[list];
    case kQSv: return &st->sv;
    case kQSi: return &st->si;
    case kQOvf: return &st->ovf_cnt[st->oe];
    default: return &st->ring_cnt[c - kQRing];
    }
}

__device__ __forceinline__ void tile_reserve(SplitState *st, Tile &T, int list) {
    __syncthreads();
    for (int c = threadIdx.x; c < kQCat; c += kSB) T.base[c] = T.cnt[c] ? atomicAdd(tile_counter(st, c, list), T.cnt[c]) : 0u;
    if (threadIdx.x == 0 && T.ominb != ~0ull) atomicMin(&st->ovf_minb, T.ominb);
    __syncthreads();
}

__device__ __forceinline__ void tile_write(const SplitBufs &B, const Tile &T, const Push &P, int list) {
    const int64_t v = P.v;
    if (P.take)
        for (uint32_t j = 0; j < P.nl; j++) B.fitems[list][T.base[kQFi] + P.offi + j] = ((uint64_t)(uint32_t)v << 32) | j;
    if (P.isv) {
        const SplitState *st = B.st;
        const uint64_t iv = (uint64_t)T.base[kQSv] + P.offsv, is = (uint64_t)T.base[kQSi] + P.offs;
        if (iv - st->sv_done < st->sv_cap && is + P.nh - st->si_done <= st->si_cap) {
            B.sverts[iv % st->sv_cap] = (int32_t)v;
            for (uint32_t j = 0; j < P.nh; j++) B.sitems[(is + j) % st->si_cap] = ((uint64_t)(uint32_t)v << 32) | j;
        } else {
            atomicOr(&B.st->err, 1);
        }
    }
    if (P.q == kQOvf) B.ovf[B.st->oe][T.base[kQOvf] + P.offr] = (int32_t)v;
    else if (P.q >= kQRing) B.ring[(uint64_t)(P.q - kQRing) * (uint64_t)B.n + T.base[P.q] + P.offr] = (int32_t)v;
}

__global__ void k_split_start(SplitBufs B, int64_t src) {
    const int64_t i = (int64_t)blockIdx.x * kSB + threadIdx.x;
    for (int64_t v = i; v < B.n; v += (int64_t)gridDim.x * kSB) {
        B.dist[v] = v == src ? 0ull : kInf;
        B.lrel[v] = kInf;
        B.srec[v] = SRec{0, 0, 0, 0};
        B.qstamp[v] = 0;
    }
    for (int64_t v = i; v < B.v1 - B.v0; v += (int64_t)gridDim.x * kSB) B.istamp[v] = 0;
}

__global__ void k_split_seed(SplitBufs B, int64_t src, uint32_t pull_min, uint32_t fuse, uint32_t sv_cap,
                             uint64_t si_cap) {
    SplitState *st = B.st;
    if (threadIdx.x == 0) {
        memset(st, 0, sizeof(SplitState));
        st->sv_cap = sv_cap;
        st->si_cap = si_cap;
        st->epoch = 1;
        st->epoch_round = 1;
        st->ostamp_tag = 1;
        st->consume = -1;
        st->ovf_minb = ~0ull;
        st->pull_min = pull_min;
        st->fuse = fuse;
    }
    __syncthreads();
    // the source -> list 1 (the next frontier)
    __shared__ Tile T;
    tile_begin(T);
    Push P;
    tile_stage(B, T, P, threadIdx.x == 0, false, src, 0ull, 0, 1);
    tile_reserve(st, T, 1);
    tile_write(B, T, P, 1);
}

__device__ void k_split_plan_body(SplitState *st);

__global__ void k_split_plan(SplitState *st) {
    st->nimp = 0;
    if (st->done) {
        st->mode = kNone;
        return;
    }
    st->round++;
    k_split_plan_body(st);
    if (st->round <= 256) st->modelog[st->round - 1] = (int8_t)st->mode;
}

__device__ void k_split_plan_body(SplitState *st) {
    if (st->err || st->sv - st->sv_done > st->sv_cap || st->si - st->si_done > st->si_cap) {   // ring overrun
        st->err = 1;
        st->done = 1;
        st->mode = kNone;
        return;
    }
    if (st->consume >= 0) {
        for (int j = 0; j < st->consume_n; j++) st->ring_cnt[(st->consume + j) % kW] = 0;
        st->consume = -1;
    }
    const int nx = st->fc ^ 1;
    if (st->fv[nx] > 0) {   // the frontier queued last round
        st->mode = kLight;
        st->fc = nx;
        st->fv[nx ^ 1] = 0;
        st->fi[nx ^ 1] = 0;
        st->nmode[kLight]++;
        st->nitems[kLight] += st->fi[nx];
        return;
    }
    st->fv[nx] = st->fi[nx] = 0;
    if (st->sv > st->sv_done) {   // heavy edges of the vertices settled since the last time
        st->sb0 = st->sv_done;
        st->sb1 = st->sv;
        st->hs0 = st->si_done;
        st->hs1 = st->si;
        st->sv_done = st->sv;
        st->si_done = st->si;
        st->mode = st->pull_min && st->sb1 - st->sb0 >= st->pull_min ? kPull : kHeavy;
        st->smin = ~0ull;
        st->nmode[st->mode]++;
        st->nitems[kHeavy] += st->mode == kHeavy ? st->hs1 - st->hs0 : 0;
        return;
    }
    // open the next non-empty ring bucket, with the following ones while the vertices stay
    // within `fuse` (bucket fusion; any grouping reaches the same fixed point)
    const int64_t lim = st->win_base + kW;
    for (int64_t b = st->cur + 1; b < lim; b++) {
        const uint32_t c0 = st->ring_cnt[b % kW];
        if (c0 == 0) continue;
        uint32_t tot = c0;
        int64_t last = b;
        for (int64_t b2 = b + 1; b2 < lim; b2++) {
            const uint32_t c = st->ring_cnt[b2 % kW];
            if (tot + c > st->fuse) break;
            tot += c;
            last = b2;
        }
        st->mode = kAdvance;
        st->cur = last;
        st->slot0 = (int32_t)(b % kW);
        st->nslots = (int32_t)(last - b + 1);
        st->consume = st->slot0;
        st->consume_n = st->nslots;
        st->epoch++;
        st->epoch_round = st->round;
        st->sv = st->sv_done = st->si = st->si_done = 0;
        st->fc = nx;   // take fills list fc, apply the other
        st->fv[0] = st->fv[1] = st->fi[0] = st->fi[1] = 0;
        st->nmode[kAdvance]++;
        return;
    }
    const int src = st->oe;
    if (st->ovf_cnt[src] > 0) {   // new ring window from the overflow
        const int64_t mb = (int64_t)min(st->ovf_minb, 4000000000000000000ull);
        st->win_base = max(st->cur + 1, mb);
        st->cur = st->win_base - 1;
        st->oe = src ^ 1;
        st->ovf_cnt[st->oe] = 0;
        st->ovf_minb = ~0ull;
        st->ostamp_tag++;
        st->mode = kSplit;
        st->nmode[kSplit]++;
        return;
    }
    st->done = 1;
    st->mode = kNone;
}

// ADVANCE: the opened ring slots' still pending vertices -> this round's frontier;
// SPLIT: the old overflow -> ring slots of the new window / the new overflow;
// HEAVY / PULL: the settled batch's heavy edges are now relaxed (PULL: marked, and its
// smallest distance taken).
__global__ __launch_bounds__(kSB) void k_split_prep(SplitBufs B) {
    SplitState *st = B.st;
    const int32_t mode = st->mode;
    __shared__ Tile T;
    if (mode == kAdvance) {
        const int64_t cur = st->cur;
        const int32_t round = st->round, epoch = st->epoch, fc = st->fc;
        // the opened slots' entries as one index space
        uint32_t tot = 0;
        for (int j = 0; j < st->nslots; j++) tot += st->ring_cnt[(st->slot0 + j) % kW];
        const uint32_t per = tile_per(tot), tile = per * kSB;
        for (uint32_t t0 = blockIdx.x * tile; t0 < tot; t0 += gridDim.x * tile) {
            tile_begin(T);
            Push P[kPer];
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                uint32_t i = t0 + k * kSB + threadIdx.x;
                const bool valid = k < (int)per && i < tot;
                int32_t v = 0;
                if (valid) {
                    int j = 0;
                    uint32_t c = st->ring_cnt[st->slot0 % kW];
                    while (i >= c) {
                        i -= c;
                        j++;
                        c = st->ring_cnt[(st->slot0 + j) % kW];
                    }
                    v = B.ring[(uint64_t)((st->slot0 + j) % kW) * (uint64_t)B.n + i];
                }
                const unsigned long long d = valid ? B.dist[v] : kInf;
                bool now = valid && d < B.lrel[v] && sbucket(d, B.inv_delta) <= cur;
                if (now) now = B.qstamp[v] != round && atomicExch(&B.qstamp[v], round) != round;
                tile_stage(B, T, P[k], now, false, v, d, 0, epoch);
            }
            tile_reserve(st, T, fc);
#pragma unroll
            for (int k = 0; k < kPer; k++) tile_write(B, T, P[k], fc);
            __syncthreads();
        }
    } else if (mode == kSplit) {
        const int src = st->oe ^ 1;
        const uint32_t cnt = st->ovf_cnt[src];
        const uint32_t per = tile_per(cnt), tile = per * kSB;
        for (uint32_t t0 = blockIdx.x * tile; t0 < cnt; t0 += gridDim.x * tile) {
            tile_begin(T);
            Push P[kPer];
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                const uint32_t i = t0 + k * kSB + threadIdx.x;
                const bool valid = k < (int)per && i < cnt;
                const int32_t v = valid ? B.ovf[src][i] : 0;
                const unsigned long long d = valid ? B.dist[v] : kInf;
                const bool pend = valid && d < B.lrel[v];
                tile_stage(B, T, P[k], false, pend, v, d, pend ? sbucket(d, B.inv_delta) : 0, 0);
            }
            tile_reserve(st, T, 0);
#pragma unroll
            for (int k = 0; k < kPer; k++) tile_write(B, T, P[k], 0);
            __syncthreads();
        }
    } else if (mode == kHeavy || mode == kPull) {
        const int32_t round = st->round;
        unsigned long long m = ~0ull;
        for (uint32_t i = st->sb0 + blockIdx.x * kSB + threadIdx.x; i < st->sb1; i += gridDim.x * kSB) {
            const int32_t u = B.sverts[i % st->sv_cap];
            B.srec[u].hmark = round;
            if (mode == kPull) m = min(m, B.dist[u]);
        }
        if (mode == kPull) {
            for (int off = 32; off > 0; off >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, off, kWave));
            if ((threadIdx.x & (kWave - 1)) == 0 && m != ~0ull) atomicMin(&st->smin, m);
        }
    }
}

// LIGHT / ADVANCE: the frontier's light edges; HEAVY: the settled batch's heavy edges.  A wave
// takes up to 64 items (vertex, 256-edge chunk) and walks their concatenated edges 64 at a time,
// each lane finding its item by a shuffle binary search over the items' edge prefix -- a
// frontier of low-degree vertices fills the lanes.  PULL: a thread (a wave past kSmallDeg
// in-edges) per candidate, its heavy in-edges from the settled batch, minimum in registers.  Improved owned
// vertices are claimed once per round, staged in LDS and appended once per workgroup.
constexpr int kStageCap = 2048;

__global__ __launch_bounds__(kSB) void k_split_relax(SplitBufs B) {
    SplitState *st = B.st;
    const int32_t mode = st->mode;
    if (mode == kNone || mode == kSplit) return;
    __shared__ int32_t stage[kStageCap];
    __shared__ uint32_t scnt, sbase;
    if (threadIdx.x == 0) scnt = 0;
    __syncthreads();
    const int32_t round = st->round;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = (blockIdx.x * kSB + threadIdx.x) / kWave, nw = gridDim.x * (kSB / kWave);
    auto claim = [&](bool won, int32_t v) {   // every lane of the wave calls
        const uint64_t m = __ballot(won);
        if (!m) return;
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(&scnt, (uint32_t)__popcll(m));
        at = __shfl(at, 0, kWave) + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (won) {
            if (at < kStageCap) stage[at] = v;
            else B.imp[atomicAdd(&st->nimp, 1u)] = v;   // stage full: straight out
        }
    };
    if (mode == kPull) {
        // candidates found here: an owned vertex above fl(smin + delta) with heavy in-edges;
        // up to kSmallDeg of them a thread pulls at once, larger rows go to the workgroup's
        // LDS list for its waves (the loop trip count is uniform per wave)
        __shared__ int32_t bigs[kBigCap];
        __shared__ uint32_t nbig;
        if (threadIdx.x == 0) nbig = 0;
        __syncthreads();
        const unsigned long long lim =
            (unsigned long long)__double_as_longlong(__longlong_as_double((long long)st->smin) + B.delta);
        auto pull_row = [&](int64_t i) {
            unsigned long long best = kInf;
            for (int64_t e = B.orp[i]; e < B.orp[i + 1]; e++) {
                const int32_t u = B.oci[e];
                if (B.srec[u].hmark == round) {
                    const unsigned long long nd =
                        (unsigned long long)__double_as_longlong(__longlong_as_double((long long)B.dist[u]) + B.ow[e]);
                    best = min(best, nd);
                }
            }
            return best;
        };
        const int64_t own = B.v1 - B.v0;
        const int64_t nth = (int64_t)gridDim.x * kSB, span = (own + kWave - 1) / kWave * kWave;
        for (int64_t i = (int64_t)blockIdx.x * kSB + threadIdx.x; i < span; i += nth) {
            bool won = false;
            if (i < own) {
                const unsigned long long d = B.dist[B.v0 + i];
                const int64_t deg = d > lim ? B.orp[i + 1] - B.orp[i] : 0;
                bool listed = false;
                if (deg > kSmallDeg) {
                    const uint32_t at = atomicAdd(&nbig, 1u);
                    listed = at < (uint32_t)kBigCap;
                    if (listed) bigs[at] = (int32_t)i;
                }
                if (deg > 0 && !listed) {
                    // (a full list: the thread pulls the row itself)
                    const unsigned long long best = pull_row(i);
                    if (best < d) {
                        B.dist[B.v0 + i] = best;   // this thread alone writes the vertex this round
                        won = true;
                    }
                }
            }
            claim(won, (int32_t)(B.v0 + i));
        }
        __syncthreads();
        const uint32_t nb = min(nbig, (uint32_t)kBigCap);
        for (uint32_t it = threadIdx.x / kWave; it < nb; it += kSB / kWave) {
            const int64_t i = bigs[it];
            unsigned long long best = kInf;
            for (int64_t e = B.orp[i] + lane; e < B.orp[i + 1]; e += kWave) {
                const int32_t u = B.oci[e];
                if (B.srec[u].hmark == round) {
                    const unsigned long long nd =
                        (unsigned long long)__double_as_longlong(__longlong_as_double((long long)B.dist[u]) + B.ow[e]);
                    best = min(best, nd);
                }
            }
            for (int off = 32; off > 0; off >>= 1) best = min(best, (unsigned long long)__shfl_xor(best, off, kWave));
            bool won = false;
            if (lane == 0 && best < B.dist[B.v0 + i]) {
                B.dist[B.v0 + i] = best;   // this wave alone writes the vertex this round
                won = true;
            }
            claim(won, (int32_t)(B.v0 + i));
        }
    } else {
        const bool heavy = mode == kHeavy;
        const uint64_t *items = heavy ? B.sitems : B.fitems[st->fc];
        const uint32_t i0 = heavy ? st->hs0 : 0u, i1 = heavy ? st->hs1 : st->fi[st->fc];
        // G = ceil(items / waves) <= 64 items per wave: a short list (a hub's chunks) spreads
        // over as many waves as it has items instead of filling a few waves' lanes
        const uint32_t G = max(1u, min((uint32_t)kWave, (i1 - i0 + nw - 1) / nw));
        for (uint32_t g0 = i0 + wid * G; g0 < i1; g0 += nw * G) {
            // lane l < G: item g0 + l
            const uint32_t gi = g0 + lane;
            int64_t e0 = 0, len = 0;
            unsigned long long du = 0;
            if (lane < (int)G && gi < i1) {
                const uint64_t x = items[heavy ? gi % st->si_cap : gi];
                const int64_t u = (int64_t)(x >> 32), j = (int64_t)(x & 0xffffffffu);
                const VRec vr = B.vrec[u];
                const int64_t a = heavy ? vr.start + vr.nl : vr.start, b = a + (heavy ? vr.nh : vr.nl);
                e0 = a + j * kSChunk;
                len = max<int64_t>(0, min(b, e0 + kSChunk) - e0);
                du = B.dist[u];
            }
            // exclusive prefix of the items' lengths (<= 64 x 256: 32 bits)
            uint32_t x = (uint32_t)len;
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, kWave);
                if (lane >= off) x += y;
            }
            const uint32_t total = __shfl(x, kWave - 1, kWave);
            const uint32_t pre = x - (uint32_t)len;
            // four edges per lane and pass, each step issued for all four before any result is
            // used (the edge, target and claim loads of one edge are a dependent chain)
            constexpr int kQ = 4;
            for (uint32_t k0 = 0; k0 < total; k0 += kQ * kWave) {
                int32_t t[kQ];
                unsigned long long nd[kQ];
                bool live[kQ], won[kQ];
#pragma unroll
                for (int q = 0; q < kQ; q++) {
                    const uint32_t k = k0 + q * kWave + lane;
                    // the item holding edge k: the last lane whose prefix is <= k (lanes past
                    // the group have len 0 and prefix = total, never <= k < total)
                    int lo = 0;
#pragma unroll
                    for (int step = 32; step > 0; step >>= 1) {
                        const int c = lo + step;
                        const uint32_t pc = __shfl(pre, c < kWave ? c : kWave - 1, kWave);
                        if (c < kWave && pc <= k) lo = c;
                    }
                    const int64_t eo = __shfl(e0, lo, kWave);
                    const uint32_t po = __shfl(pre, lo, kWave);
                    const unsigned long long dbits = __shfl(du, lo, kWave);
                    live[q] = k < total;
                    t[q] = 0;
                    nd[q] = kInf;
                    if (live[q]) {
                        const int64_t e = eo + (int64_t)(k - po);
                        t[q] = B.sci[e];
                        nd[q] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)dbits) + B.sw[e]);
                    }
                }
                unsigned long long cur[kQ];
#pragma unroll
                for (int q = 0; q < kQ; q++)
                    cur[q] = live[q] ? __hip_atomic_load(&B.dist[B.v0 + t[q]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : 0ull;
                int32_t stamp[kQ];
#pragma unroll
                for (int q = 0; q < kQ; q++) {
                    won[q] = live[q] && nd[q] < cur[q];
                    // no return: the load decided that the vertex improves this round
                    if (won[q]) __hip_atomic_fetch_min(&B.dist[B.v0 + t[q]], nd[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    stamp[q] = won[q] ? B.istamp[t[q]] : round;
                }
#pragma unroll
                for (int q = 0; q < kQ; q++) {
                    won[q] = won[q] && stamp[q] != round && atomicExch(&B.istamp[t[q]], round) != round;
                    claim(won[q], (int32_t)(B.v0 + t[q]));
                }
            }
        }
    }
    __syncthreads();
    const uint32_t n_st = min(scnt, (uint32_t)kStageCap);
    if (threadIdx.x == 0) sbase = n_st ? atomicAdd(&st->nimp, n_st) : 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_st; i += kSB) B.imp[sbase + i] = stage[i];
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

// Every rank's pairs (rank r's at pairs + 2 r stride, their number at counts[2 r]), as one
// index space cut into tiles.
__global__ __launch_bounds__(kSB) void k_split_apply(SplitBufs B, const uint64_t *pairs, const uint64_t *counts,
                                                     int nranks, uint64_t stride) {
    SplitState *st = B.st;
    if (st->mode == kNone || st->mode == kSplit) return;
    const int64_t cur = st->cur;
    const int32_t epoch = st->epoch, nx = st->fc ^ 1;
    uint64_t tot = 0;
    if (!pairs) tot = st->nimp;
    else
        for (int r = 0; r < nranks; r++) tot += counts[2 * r];
    __shared__ Tile T;
    const uint32_t per = tile_per(tot), tile = per * kSB;
    for (uint64_t t0 = (uint64_t)blockIdx.x * tile; t0 < tot; t0 += (uint64_t)gridDim.x * tile) {
        tile_begin(T);
        Push P[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            uint64_t i = t0 + (uint64_t)k * kSB + threadIdx.x;
            const bool valid = k < (int)per && i < tot;
            int64_t v = 0;
            unsigned long long d = kInf;
            if (valid && !pairs) {   // this rank's own improved list (a single rank)
                v = B.imp[i];
                d = B.dist[v];
            } else if (valid) {
                int r = 0;
                while (i >= counts[2 * r]) {
                    i -= counts[2 * r];
                    r++;
                }
                const uint64_t *pr = pairs + 2 * ((uint64_t)r * stride + i);
                v = (int64_t)pr[0];
                d = pr[1];
                if (d < B.dist[v]) B.dist[v] = d;   // one pair per vertex and round
            }
            const int64_t b = valid ? sbucket(d, B.inv_delta) : 0;
            const bool near = valid && b <= cur;
            tile_stage(B, T, P[k], near, valid && !near, v, d, b, epoch);
        }
        tile_reserve(st, T, nx);
#pragma unroll
        for (int k = 0; k < kPer; k++) tile_write(B, T, P[k], nx);
        __syncthreads();
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

__global__ __launch_bounds__(kSB) void k_slice_vrec(const int64_t *__restrict__ srp, const int64_t *__restrict__ slend,
                                                    int64_t n, VRec *vrec) {
    for (int64_t u = (int64_t)blockIdx.x * kSB + threadIdx.x; u < n; u += (int64_t)gridDim.x * kSB)
        vrec[u] = VRec{srp[u], (uint32_t)(slend[u] - srp[u]), (uint32_t)(srp[u + 1] - slend[u])};
}

// PULL layout: the heavy entries (w >= delta) of the owned rows of A (an undirected graph's
// in-edges), row order kept.  Wave per row.
__global__ __launch_bounds__(kSB) void k_own_count(const int64_t *__restrict__ rp, const double *__restrict__ w,
                                                   int64_t v0, int64_t v1, double delta, int64_t *cnt) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (kSB / kWave), own = v1 - v0;
    for (int64_t i = ((int64_t)blockIdx.x * kSB + threadIdx.x) / kWave; i < own; i += nw) {
        uint32_t h = 0;
        for (int64_t e = rp[v0 + i] + lane; e < rp[v0 + i + 1]; e += kWave) h += !(w[e] < delta);
        for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off, kWave);
        if (lane == 0) cnt[i] = h;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[own] = 0;
}

__global__ __launch_bounds__(kSB) void k_own_scatter(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                     const double *__restrict__ w, int64_t v0, int64_t v1, double delta,
                                                     const int64_t *__restrict__ orp, int32_t *oci, double *ow) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (kSB / kWave), own = v1 - v0;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int64_t i = ((int64_t)blockIdx.x * kSB + threadIdx.x) / kWave; i < own; i += nw) {
        int64_t at = orp[i];
        const int64_t r0 = rp[v0 + i], r1 = rp[v0 + i + 1];
        for (int64_t eb = r0; eb < r1; eb += kWave) {
            const int64_t e = eb + lane;
            const bool hv = e < r1 && !(w[e] < delta);
            const uint64_t m = __ballot(hv);
            if (hv) {
                const int64_t q = at + __popcll(m & below);
                oci[q] = ci[e];
                ow[q] = w[e];
            }
            at += __popcll(m);
        }
    }
}

// Per-block partial sums of the weights in a fixed order (grid-stride per thread, butterfly per
// wave, waves in index order), so the bucket width derived from them is bitwise the same on
// every rank that holds the same graph: the ranks' scheduling decisions must agree.
__global__ __launch_bounds__(256) void k_split_sum_w(const double *__restrict__ w, int64_t m, double *part) {
    __shared__ double wsum[256 / kWave];
    double acc = 0.0;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < m; k += (int64_t)gridDim.x * 256) acc += w[k];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) wsum[threadIdx.x / kWave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < 256 / kWave; i++) t += wsum[i];
        part[blockIdx.x] = t;
    }
}

}  // namespace
}  // namespace gx

using namespace gx;

struct gx_sssp_split {
    gx_graph *g = nullptr;        // the graph the slice is built on (a single rank: its hub-first copy)
    gx_graph *caller = nullptr;   // the graph gx_sssp_split_create was given
    bool hub_checked = false;     // gx_sssp_split_run looked for the hub-first copy
    int rounds_hint = 0;          // rounds the last gx_sssp_split_run took
    int64_t n = 0, v0 = 0, v1 = 0, snnz = 0, onnz = 0;
    uint32_t sv_cap = 0;          // settled-list capacities (SplitState::sv_cap / si_cap)
    uint64_t si_cap = 0;
    double delta = 1.0;
    uint32_t pull_min = 0, fuse = 0;
    DBuf<VRec> vrec;
    DBuf<SRec> srec;
    DBuf<int64_t> orp;
    DBuf<int32_t> sci, oci;
    DBuf<double> sw, ow;
    DBuf<unsigned long long> dist, lrel;
    DBuf<int32_t> qstamp, istamp, sverts, ring, ovf0, ovf1, imp;
    DBuf<uint64_t> fitems0, fitems1, sitems, own_pairs, own_count;
    DBuf<SplitState> st;
    int32_t *h_done = nullptr;
    unsigned grid = 0;
    ~gx_sssp_split() {
        if (h_done) (void)hipHostFree(h_done);
    }
    SplitBufs bufs() {
        SplitBufs B;
        B.vrec = vrec.p;
        B.sci = sci.p;
        B.sw = sw.p;
        B.orp = orp.p;
        B.oci = oci.p;
        B.ow = ow.p;
        B.dist = dist.p;
        B.lrel = lrel.p;
        B.srec = srec.p;
        B.qstamp = qstamp.p;
        B.istamp = istamp.p;
        B.fitems[0] = fitems0.p;
        B.fitems[1] = fitems1.p;
        B.sitems = sitems.p;
        B.sverts = sverts.p;
        B.ring = ring.p;
        B.ovf[0] = ovf0.p;
        B.ovf[1] = ovf1.p;
        B.imp = imp.p;
        B.n = n;
        B.v0 = v0;
        B.v1 = v1;
        B.delta = delta;
        B.inv_delta = 1.0 / delta;
        B.st = st.p;
        return B;
    }
};

// as the other *_part_* steps (gx.h): NULL is the null (default) stream -- torch's -- so the
// steps order with the tensors and collectives issued there
static hipStream_t split_stream(gx_sssp_split *, void *stream) { return (hipStream_t)stream; }

// plan -> prep -> relax -> pairs (this rank's improved owned vertices; a single rank's device
// loop skips the pairs: its apply reads the improved list)
static int split_relax(gx_sssp_split *p, uint64_t *pairs, uint64_t *count, hipStream_t s) {
    const SplitBufs B = p->bufs();
    hipLaunchKernelGGL(k_split_plan, dim3(1), dim3(1), 0, s, B.st);
    hipLaunchKernelGGL(k_split_prep, dim3(p->grid), dim3(kSB), 0, s, B);
    hipLaunchKernelGGL(k_split_relax, dim3(p->grid), dim3(kSB), 0, s, B);
    if (pairs) hipLaunchKernelGGL(k_split_pairs, dim3(p->grid), dim3(kSB), 0, s, B, pairs, count);
    return check_launch("k_split_relax");
}

static int split_apply(gx_sssp_split *p, const uint64_t *pairs, const uint64_t *counts, int nranks, uint64_t stride,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_split_apply, dim3(p->grid), dim3(kSB), 0, s, p->bufs(), pairs, counts, nranks, stride);
    return check_launch("k_split_apply");
}

static int split_build(gx_sssp_split *p, gx_graph *g);

extern "C" int gx_sssp_split_create(gx_graph *g, uint64_t v0, uint64_t v1, gx_sssp_split **out) {
    if (!g || !out) return fail(GX_NULL_POINTER, "gx_sssp_split_create: null argument");
    if (!g->weighted) return fail(GX_INVALID_VALUE, "gx_sssp_split_create: graph has no edge weights");
    if (v0 > v1 || v1 > g->n) return fail(GX_INVALID_INDEX, "gx_sssp_split_create: bad vertex range");
    if (g->n >= (1ull << 31) / kW) return fail(GX_NOT_IMPLEMENTED, "gx_sssp_split_create: more than 2^26 vertices");
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    std::unique_ptr<gx_sssp_split> p(new gx_sssp_split());
    p->caller = g;
    p->v0 = (int64_t)v0;
    p->v1 = (int64_t)v1;
    GX_TRY(split_build(p.get(), g));
    *out = p.release();
    return GX_SUCCESS;
}

// The slice, the PULL layout and the work buffers of p for graph g (the caller's graph, or
// for gx_sssp_split_run its hub-first copy); earlier buffers are released.
static int split_build(gx_sssp_split *p, gx_graph *g) {
    hipStream_t s = g->ctx->stream;
    p->g = g;
    p->n = (int64_t)g->n;
    const int64_t n = p->n, own = p->v1 - p->v0;
    // bucket width: gx_sssp's rule (scale x mean weight / mean degree; GX_SSSP_DELTA and
    // GX_SSSP_DSCALE override) -- any positive value gives the same distances
    double mean = 1.0;
    if (g->nnz) {
        const unsigned sgrid = grid_for(g->nnz, 256, 4096);
        DBuf<double> part;
        GX_TRY(part.alloc(sgrid));
        hipLaunchKernelGGL(k_split_sum_w, dim3(sgrid), dim3(256), 0, s, g->A.w.p, (int64_t)g->nnz, part.p);
        GX_TRY(check_launch("k_split_sum_w"));
        std::vector<double> h(sgrid);
        GX_HIP_TRY(hipMemcpyAsync(h.data(), part.p, sgrid * sizeof(double), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        double t = 0.0;
        for (double x : h) t += x;   // block order: deterministic for a given graph
        mean = t / (double)g->nnz;
    }
    double scale = g->directed ? 0.5 : 3.0, delta = 0.0;   // SYN-8_5 N = 1: 9.3-9.4 ms at 3, 9.7 at 4
    if (const char *e = std::getenv("GX_SSSP_DSCALE")) scale = std::atof(e);
    if (const char *e = std::getenv("GX_SSSP_DELTA")) delta = std::atof(e);
    if (!(delta > 0.0)) delta = scale * mean / std::max(1.0, (double)g->nnz / std::max<double>(1.0, (double)n));
    if (!(delta > 0.0) || !std::isfinite(delta)) delta = 1.0;
    p->delta = delta;
    // the heavy phase is pulled (undirected graphs) once the settled batch holds 1/8 of the
    // vertices with edges (gx_sssp's rule; GX_SSSP_PULL = 0 never, 2 always); buckets are fused
    // while they hold at most n / 16 vertices (GX_SSSP_FUSE)
    int64_t nonisolated = n;
    GX_TRY(ensure_host_rp(g->ctx, g->A));
    if ((int64_t)g->A.h_rp.size() == n + 1) {
        nonisolated = 0;
        for (int64_t v = 0; v < n; v++) nonisolated += g->A.h_rp[v + 1] != g->A.h_rp[v];
    }
    const int pull_mode = std::getenv("GX_SSSP_PULL") ? std::atoi(std::getenv("GX_SSSP_PULL")) : 1;
    const bool can_pull = !g->directed && pull_mode != 0;
    p->pull_min = !can_pull ? 0u : pull_mode == 2 ? 1u : (uint32_t)std::max<int64_t>(1, nonisolated / 8);
    p->fuse = std::getenv("GX_SSSP_FUSE") ? (uint32_t)std::max(1, std::atoi(std::getenv("GX_SSSP_FUSE")))
                                          : (uint32_t)std::max<int64_t>(1024, n / 16);
    const unsigned wg_all = grid_for((uint64_t)std::max<int64_t>(n, 1) * kWave, kSB, 16384);
    // slice: count, scan, scatter
    GX_TRY(p->vrec.alloc(std::max<int64_t>(n, 1)));
    {
        DBuf<int64_t> lc, tc, srp, slend;
        GX_TRY(srp.alloc(n + 1));
        GX_TRY(slend.alloc(std::max<int64_t>(n, 1)));
        GX_TRY(lc.alloc(std::max<int64_t>(n, 1)));
        GX_TRY(tc.alloc(n + 1));
        if (n) {
            hipLaunchKernelGGL(k_slice_count, dim3(wg_all), dim3(kSB), 0, s, g->A.rp.p, g->A.ci.p, g->A.w.p, n, p->v0,
                               p->v1, delta, lc.p, tc.p);
            GX_TRY(check_launch("k_slice_count"));
        } else {
            GX_HIP_TRY(hipMemsetAsync(tc.p, 0, sizeof(int64_t), s));
        }
        GX_TRY(scan_exclusive_i64(tc.p, srp.p, (size_t)(n + 1), s));
        GX_HIP_TRY(hipMemcpyAsync(&p->snnz, srp.p + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        GX_TRY(p->sci.alloc(std::max<int64_t>(p->snnz, 1)));
        GX_TRY(p->sw.alloc(std::max<int64_t>(p->snnz, 1)));
        if (n) {
            hipLaunchKernelGGL(k_slice_scatter, dim3(wg_all), dim3(kSB), 0, s, g->A.rp.p, g->A.ci.p, g->A.w.p, n, p->v0,
                               p->v1, delta, srp.p, lc.p, slend.p, p->sci.p, p->sw.p);
            GX_TRY(check_launch("k_slice_scatter"));
            hipLaunchKernelGGL(k_slice_vrec, dim3(grid_for(n, kSB, 8192)), dim3(kSB), 0, s, srp.p, slend.p, n, p->vrec.p);
            GX_TRY(check_launch("k_slice_vrec"));
        }
        GX_HIP_TRY(hipStreamSynchronize(s));   // lc / tc die here
    }
    // owned rows' heavy in-edges (PULL)
    GX_TRY(p->orp.alloc(own + 1));
    if (can_pull) {
        DBuf<int64_t> cnt;
        GX_TRY(cnt.alloc(own + 1));
        const unsigned wg_own = grid_for((uint64_t)std::max<int64_t>(own, 1) * kWave, kSB, 16384);
        hipLaunchKernelGGL(k_own_count, dim3(wg_own), dim3(kSB), 0, s, g->A.rp.p, g->A.w.p, p->v0, p->v1, delta, cnt.p);
        GX_TRY(check_launch("k_own_count"));
        GX_TRY(scan_exclusive_i64(cnt.p, p->orp.p, (size_t)(own + 1), s));
        GX_HIP_TRY(hipMemcpyAsync(&p->onnz, p->orp.p + own, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        GX_TRY(p->oci.alloc(std::max<int64_t>(p->onnz, 1)));
        GX_TRY(p->ow.alloc(std::max<int64_t>(p->onnz, 1)));
        if (own) {
            hipLaunchKernelGGL(k_own_scatter, dim3(wg_own), dim3(kSB), 0, s, g->A.rp.p, g->A.ci.p, g->A.w.p, p->v0, p->v1,
                               delta, p->orp.p, p->oci.p, p->ow.p);
            GX_TRY(check_launch("k_own_scatter"));
        }
        GX_HIP_TRY(hipStreamSynchronize(s));
    } else {
        GX_HIP_TRY(hipMemset(p->orp.p, 0, (own + 1) * sizeof(int64_t)));
    }
    // state: item lists hold at most one item per vertex plus one per 256 slice entries
    const uint64_t icap = (uint64_t)n + (uint64_t)p->snnz / kSChunk + 64;
    const int64_t n1 = std::max<int64_t>(n, 1), own1 = std::max<int64_t>(own, 1);
    p->sv_cap = (uint32_t)n1;
    p->si_cap = icap;
    GX_TRY(p->dist.alloc(n1));
    GX_TRY(p->lrel.alloc(n1));
    for (DBuf<int32_t> *b : {&p->qstamp, &p->sverts, &p->ovf0, &p->ovf1}) GX_TRY(b->alloc(n1));
    GX_TRY(p->srec.alloc(n1));
    GX_TRY(p->ring.alloc((uint64_t)n1 * kW));
    GX_TRY(p->istamp.alloc(own1));
    GX_TRY(p->imp.alloc(own1));
    GX_TRY(p->fitems0.alloc(icap));
    GX_TRY(p->fitems1.alloc(icap));
    GX_TRY(p->sitems.alloc(icap));
    GX_TRY(p->own_pairs.alloc(2 * (uint64_t)own1));
    GX_TRY(p->own_count.alloc(2));
    GX_TRY(p->st.alloc(1));
    if (!p->h_done)
        GX_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&p->h_done), 2 * sizeof(int32_t), hipHostMallocDefault));
    p->grid = (unsigned)std::max(1, g->ctx->num_cus) * 8;
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
    if (p->g != p->caller) src = (uint64_t)p->caller->h_hub_perm[src];
    GX_HIP_TRY(hipSetDevice(p->g->ctx->device));
    hipStream_t s = split_stream(p, stream);
    const SplitBufs B = p->bufs();
    hipLaunchKernelGGL(k_split_start, dim3(grid_for(std::max<int64_t>(p->n, 1), kSB, 8192)), dim3(kSB), 0, s, B,
                       (int64_t)src);
    hipLaunchKernelGGL(k_split_seed, dim3(1), dim3(kSB), 0, s, B, (int64_t)src, p->pull_min, p->fuse, p->sv_cap,
                       p->si_cap);
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

// Fails when the run stopped on a full settled list (SplitState::err) instead of finishing.
int gx::sssp_split_check(gx_sssp_split *p, hipStream_t s) {
    int32_t err = 0;
    GX_HIP_TRY(hipMemcpyAsync(&err, &p->st.p->err, sizeof(err), hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    if (err) return fail(GX_OUT_OF_MEMORY, "gx_sssp_split: an epoch settled more vertices than the settled list holds");
    return GX_SUCCESS;
}

extern "C" int gx_sssp_split_distances(gx_sssp_split *p, double *dist, void *stream) {
    if (!p || !dist) return fail(GX_NULL_POINTER, "gx_sssp_split_distances: null argument");
    GX_HIP_TRY(hipSetDevice(p->g->ctx->device));
    hipStream_t s = split_stream(p, stream);
    GX_TRY(sssp_split_check(p, s));
    const void *res = nullptr;
    GX_TRY(remap_out(p->g, p->dist.p, 8, s, &res));   // hub-first copy -> the caller's order
    GX_HIP_TRY(hipMemcpyAsync(dist, res, (size_t)p->n * 8, hipMemcpyDeviceToDevice, s));
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
    if (!p->hub_checked) {
        // one rank owning every vertex: the hub-first copy of an undirected graph, as gx_sssp
        // runs from its second call (gx_runtime.hip hub_for; GX_HUB=0 keeps the caller's order)
        p->hub_checked = true;
        gx_graph *h = nullptr;
        GX_TRY(hub_for(p->caller, 2, &h, nullptr));
        if (h && h != p->g) GX_TRY(split_build(p, h));
    }
    GX_TRY(device_begin(ctx));
    GX_TRY(gx_sssp_split_start(p, src, s));
    // the first batch queues as many rounds as the last run took (+2), then batches of 8; a
    // round past the end is four launches that return at once
    int batch = p->rounds_hint > 0 ? std::min(p->rounds_hint + 2, 512) : 16;
    for (int64_t guard = 0;; guard++) {
        for (int k = 0; k < batch; k++) {
            GX_TRY(split_relax(p, nullptr, nullptr, s));
            GX_TRY(split_apply(p, nullptr, nullptr, 1, 0, s));
        }
        GX_HIP_TRY(hipMemcpyAsync(p->h_done, &p->st.p->done, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        if (p->h_done[0]) break;
        batch = 8;
        if (guard > 4 * (p->n + 16)) return fail(GX_DEVICE_ERROR, "gx_sssp_split_run: no fixed point");
    }
    {
        int32_t rounds = 0;
        GX_HIP_TRY(hipMemcpy(&rounds, &p->st.p->round, sizeof(int32_t), hipMemcpyDeviceToHost));
        p->rounds_hint = rounds;
    }
    GX_TRY(device_end(ctx));
    if (std::getenv("GX_SPLIT_VERBOSE")) {
        SplitState h;
        GX_HIP_TRY(hipMemcpy(&h, p->st.p, sizeof(h), hipMemcpyDeviceToHost));
        std::fprintf(stderr,
                     "[gx_sssp_split] delta %.4g rounds %d: light %u (items %llu), heavy push %u (items %llu), "
                     "pull %u, advance %u, split %u\n",
                     p->delta, h.round, h.nmode[kLight], h.nitems[kLight], h.nmode[kHeavy], h.nitems[kHeavy],
                     h.nmode[kPull], h.nmode[kAdvance], h.nmode[kSplit]);
        std::fprintf(stderr, "[gx_sssp_split] modes:");
        for (int i = 0; i < std::min(h.round, 256); i++) std::fprintf(stderr, " %d", (int)h.modelog[i]);
        std::fprintf(stderr, "\n");
    }
    GX_TRY(sssp_split_check(p, s));
    const void *res = nullptr;
    GX_TRY(remap_out(p->g, p->dist.p, 8, s, &res));   // hub-first copy -> the caller's order
    GX_HIP_TRY(hipStreamSynchronize(s));
    GX_HIP_TRY(hipMemcpy(dist_host, res, (size_t)p->n * 8, hipMemcpyDeviceToHost));
    return GX_SUCCESS;
}

GX_MODULE_WARMER(sssp_split)
