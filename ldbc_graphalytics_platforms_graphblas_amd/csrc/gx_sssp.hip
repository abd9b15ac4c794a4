// gx_sssp.hip -- single-source shortest paths by device-scheduled delta-stepping (min.plus).
//
// Replaces LA_SSSP -> diagonal fill + LAGraph_Cached_EMin + LAGr_SingleSourceShortestPath
// with delta = 2.5 (sssp.cpp:53-81).  The zero diagonal the reference inserts cannot change a
// distance and is not materialised.
// Distances are non-negative fp64 kept as their IEEE bit patterns, whose unsigned order is
// the numeric order, so a relaxation is one 64-bit atomicMin.  Every improvement re-queues
// its vertex, so the loop ends at the relaxation fixed point: the minimum over paths of the
// left-to-right fp64 path sum, the value Dijkstra produces -- bitwise equal to the oracle
// whatever delta or the relaxation order.
//
// Buckets (delta-stepping, Meyer & Sanders; GPU bucket ring after Davidson et al. and ADDS):
//   bucket(d) = floor(d / delta); `cur` is the bucket being settled.
//   near    : work items (vertex << 32 | 256-edge chunk) of vertices in buckets <= cur,
//             one wave per item, ping-ponged between rounds;
//   ring    : kRing vertex lists for the buckets cur+1 .. win_base+kRing-1 (deduplicated by
//             a per-vertex bucket stamp);
//   overflow: vertices beyond the ring window, split into a new window when the ring empties.
//   relaxed[v] = largest source distance any chunk of v was relaxed with since v was last
//             queued; a bucket entry whose distance equals it was already relaxed and is
//             skipped (removes the near/far double processing).
// Scheduling runs on the device: a one-thread plan kernel reads the queue counts and picks
// the next action (relax / open the next ring bucket / split the overflow / done), so the
// host launches plan -> advance -> relax triples in batches and syncs once per batch.
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

constexpr int kSsspBlock = 256;
constexpr int kChunk = 256;
constexpr int kRing = 32;
constexpr uint32_t kOob = 0x80000000u;   // buffer offset past every record: the lane is dropped
constexpr int64_t kMaxBufVertices = (int64_t)(kOob / 8u);   // dist[] must stay below kOob bytes

__device__ __forceinline__ unsigned long long dbits(double d) {
    return (unsigned long long)__double_as_longlong(d);
}
__device__ __forceinline__ double bitsd(unsigned long long b) { return __longlong_as_double((long long)b); }

__device__ __forceinline__ uint32_t chunks_of(int64_t deg) { return (uint32_t)((deg + kChunk - 1) / kChunk); }

__device__ __forceinline__ int64_t bucket_of(double d, double inv_delta) {
    const double q = d * inv_delta;
    return q < 4.0e18 ? (int64_t)q : (int64_t)4000000000000000000ll;
}

struct SsspState {
    int64_t cur;                  // bucket being settled
    int64_t win_base;             // ring window [win_base, win_base + kRing)
    unsigned long long ovf_minb;  // lower bound on the buckets in the overflow
    int32_t round;                // near queue q[round & 1] is relaxed this step
    int32_t done;
    int32_t epoch;                // relaxations append to overflow[epoch & 1]
    int32_t mode;                 // advance: 0 none, 1 open ring slot, 2 split overflow, 3 heavy items
    int32_t heavy;                // relax phase: 0 light edges, 1 heavy edges
    int32_t slot;                 // first ring slot opened (mode 1)
    int32_t nslots;               // ring slots opened together (bucket fusion, mode 1)
    int32_t consume;              // first ring slot to clear at the next plan, -1 none
    int32_t consume_n;            // ... and how many
    uint32_t fuse;                // bucket fusion: open further buckets while the entries stay <= fuse
    int32_t fuse_max;             // ... and at most fuse_max buckets (<= kRing)
    int32_t split_src;            // overflow list being split (mode 2)
    uint32_t qcnt[2];
    uint32_t ovf_cnt[2];
    uint32_t settled_cnt;         // vertices queued in the current bucket
    int32_t pull;                 // heavy phase pulled by the unsettled vertices (k_sssp_pull)
    uint32_t pull_min;            // settled-list size from which the heavy phase is pulled
    unsigned long long smin;      // smallest distance on the settled list (pull bound)
    int32_t bits_dirty;           // the settled bitmap holds a past pull's bits
    int32_t clear_bits;           // this step's advance clears the bitmap (all workgroups)
    uint32_t ring_cnt[kRing];
};

struct SsspBufs {
    const int64_t *rp;
    const int64_t *lend;          // light part of row v: [rp[v], lend[v]), heavy: [lend[v], rp[v+1])
    const int32_t *ci;            // light/heavy-partitioned rows (SsspLayout)
    const double *w;
    unsigned long long *dist;
    unsigned long long *relaxed;  // distance all edges of v were last relaxed with
    unsigned long long *nsw;      // (bucket a vertex was last put on the settled list for << 32) |
                                  // round it was last queued as near: one word, one exchange
    int32_t *bstamp;              // bucket a vertex was last put into a ring slot for
    int32_t *ostamp;              // overflow epoch a vertex was last put on the overflow
    uint32_t *sbits;              // pulled heavy phase: one bit per vertex on the settled list
    uint32_t nbits;               // words of sbits
    uint64_t *q[2];               // near work items
    int32_t *ring;                // kRing slots of ring_cap vertices
    int32_t *ovf[2];
    int32_t *settled;             // vertices of the current bucket (heavy edges pending)
    uint64_t ring_cap;
    double delta, inv_delta;
    SsspState *st;
    unsigned long long *stats;    // GX_SSSP_VERBOSE work counters, else null
    uint32_t dense_div;           // an opening of more than n / dense_div entries scans the stamps (0: never)
};

__device__ __forceinline__ unsigned long long nsw_pack(int64_t bucket, int32_t round) {
    return ((unsigned long long)(uint32_t)bucket << 32) | (uint32_t)round;
}

constexpr int kStatLanes = 256;
// stats slots: 0 items, 1 edges scanned, 2 relaxations tried, 3 improvements, 4 near pushes,
// 5 ring pushes, 6 overflow pushes, 7 bucket entries skipped as already relaxed
__device__ __forceinline__ void wave_count(unsigned long long *stats, int slot, unsigned long long x) {
    if (!stats) return;
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
    // spread over kStatLanes words per counter: one shared word would serialise the grid
    if ((threadIdx.x & (kWave - 1)) == 0 && x) atomicAdd(&stats[slot * kStatLanes + (blockIdx.x % kStatLanes)], x);
}

__device__ __forceinline__ void wave_min_to(unsigned long long m, unsigned long long *dst) {
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, kWave);
        m = o < m ? o : m;
    }
    // one shared word for the whole grid: only a wave that would lower it issues the atomic
    if ((threadIdx.x & (kWave - 1)) == 0 && m != ~0ull &&
        m < __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin(dst, m);
}

// Per-wave LDS staging of queue pushes.  The queue counters are a handful of words shared by
// the whole grid; device-scope atomics on one word serialise (about 20 ns apiece, measured:
// a relax round's time tracked its push count, not its edge count).  Pushes are therefore
// staged as (vertex, tag) in LDS and reserved in bulk: a flush counts the staged pushes per
// queue (near items, settled list, overflow, each ring slot), takes every queue's range with
// one atomic (the lanes of one instruction, one queue each) and then writes the entries.
// Mid-kernel flushes (a full stage) are per wave; the final one is per workgroup, so a launch
// costs at most one atomic per queue per workgroup plus one per full stage.
constexpr int kStage = 512;
constexpr int kTagNear = kRing, kTagOvf = kRing + 1;   // tags 0..kRing-1 are ring slots
constexpr int kCats = 3 + kRing;                       // near items, settled, overflow, ring slots

struct Stage {
    int32_t v[kStage];
    uint32_t tag[kStage];   // bits 0-6 queue, bit 7 settled-list push, bits 8.. chunk count
    uint32_t cnt[kCats];    // staged pushes per queue
    uint32_t base[kCats];   // next free entry per queue (reserved range)
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t *queue_counter(int cat, const SsspBufs &B, uint32_t *near_count,
                                                   uint32_t *ovf_count) {
    return cat == 0 ? near_count : cat == 1 ? &B.st->settled_cnt : cat == 2 ? ovf_count : &B.st->ring_cnt[cat - 3];
}

// pass 1: per-queue totals of the n staged pushes into sg.cnt
__device__ __forceinline__ void stage_count(Stage &sg, uint32_t n) {
    const int lane = threadIdx.x & (kWave - 1);
    if (lane < kCats) sg.cnt[lane] = 0;
    wave_lds_sync();
    uint32_t items = 0, nset = 0, novf = 0;
    for (uint32_t base = 0; base < n; base += kWave) {
        const uint32_t i = base + lane;
        if (i < n) {
            const uint32_t tag = sg.tag[i], q = tag & 0x7Fu;
            if (q == (uint32_t)kTagNear) {
                items += tag >> 8;
                nset += (tag >> 7) & 1u;
            } else if (q == (uint32_t)kTagOvf) {
                novf++;
            } else {
                atomicAdd(&sg.cnt[3 + q], 1u);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        items += __shfl_xor(items, off, kWave);
        nset += __shfl_xor(nset, off, kWave);
        novf += __shfl_xor(novf, off, kWave);
    }
    if (lane == 0) {
        sg.cnt[0] = items;
        sg.cnt[1] = nset;
        sg.cnt[2] = novf;
    }
    wave_lds_sync();
}

// pass 2: write the staged pushes into the ranges starting at sg.base
__device__ __forceinline__ void stage_write(Stage &sg, uint32_t n, const SsspBufs &B, uint64_t *near_out,
                                            int32_t *ovf) {
    const int lane = threadIdx.x & (kWave - 1);
    uint32_t r_items = sg.base[0], r_set = sg.base[1], r_ovf = sg.base[2];
    for (uint32_t base = 0; base < n; base += kWave) {
        const uint32_t i = base + lane;
        const bool valid = i < n;
        const int32_t v = valid ? sg.v[i] : 0;
        const uint32_t tag = valid ? sg.tag[i] : 0xFFu;
        const uint32_t q = tag & 0x7Fu;
        const bool near = valid && q == (uint32_t)kTagNear;
        const uint32_t k = near ? (tag >> 8) : 0u;
        uint32_t x = k;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const uint32_t y = __shfl_up(x, off, kWave);
            if (lane >= off) x += y;
        }
        const uint32_t at = r_items + x - k;
        for (uint32_t j = 0; j < k; j++) near_out[at + j] = ((uint64_t)(uint32_t)v << 32) | j;
        r_items += __shfl(x, kWave - 1, kWave);
        const uint64_t below = (1ull << lane) - 1;
        const bool set = near && (tag & 0x80u);
        const uint64_t ms = __ballot(set);
        if (set) B.settled[r_set + __popcll(ms & below)] = v;
        r_set += (uint32_t)__popcll(ms);
        const bool to_ovf = valid && q == (uint32_t)kTagOvf;
        const uint64_t mo = __ballot(to_ovf);
        if (to_ovf) ovf[r_ovf + __popcll(mo & below)] = v;
        r_ovf += (uint32_t)__popcll(mo);
        if (valid && q < (uint32_t)kRing) B.ring[(uint64_t)q * B.ring_cap + atomicAdd(&sg.base[3 + q], 1u)] = v;
    }
    wave_lds_sync();
}

// full stage mid-kernel: reserve for this wave alone
__device__ __forceinline__ void stage_flush(Stage &sg, uint32_t &n, const SsspBufs &B, uint64_t *near_out,
                                            uint32_t *near_count, int32_t *ovf, uint32_t *ovf_count) {
    wave_lds_sync();
    stage_count(sg, n);
    const int lane = threadIdx.x & (kWave - 1);
    if (lane < kCats) {
        const uint32_t c = sg.cnt[lane];
        sg.base[lane] = c ? atomicAdd(queue_counter(lane, B, near_count, ovf_count), c) : 0u;
    }
    wave_lds_sync();
    stage_write(sg, n, B, near_out, ovf);
    n = 0;
}

// end of the kernel: one reservation per queue for the whole workgroup.  Every thread of
// the workgroup must call it.
__device__ __forceinline__ void stage_final(Stage *stages, uint32_t &n, const SsspBufs &B, uint64_t *near_out,
                                            uint32_t *near_count, int32_t *ovf, uint32_t *ovf_count) {
    constexpr int kWaves = kSsspBlock / kWave;
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    Stage &sg = stages[wid];
    wave_lds_sync();
    stage_count(sg, n);
    __syncthreads();
    if (wid == 0 && lane < kCats) {
        uint32_t tot = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) {
            const uint32_t c = stages[w].cnt[lane];
            stages[w].base[lane] = tot;
            tot += c;
        }
        const uint32_t b = tot ? atomicAdd(queue_counter(lane, B, near_count, ovf_count), tot) : 0u;
#pragma unroll
        for (int w = 0; w < kWaves; w++) stages[w].base[lane] += b;
    }
    __syncthreads();
    if (n) stage_write(sg, n, B, near_out, ovf);
    n = 0;
}

// One thread: choose this step's action from the queue counts.
//   near non-empty           -> relax it (current phase)
//   light phase drained      -> heavy phase: relax the heavy edges of the bucket's vertices
//   heavy phase drained      -> open the next non-empty ring bucket, else split the overflow,
//                               else done
__global__ void k_sssp_plan(SsspState *st) {
    if (st->done) {
        st->mode = 0;
        return;
    }
    const int32_t r = ++st->round;
    st->clear_bits = 0;
    if (st->consume >= 0) {
        for (int j = 0; j < st->consume_n; j++) st->ring_cnt[(st->consume + j) % kRing] = 0;
        st->consume = -1;
    }
    const int qin = r & 1;
    st->qcnt[qin ^ 1] = 0;
    st->mode = 0;
    if (st->qcnt[qin] > 0) {
        if (st->bits_dirty) {
            st->clear_bits = 1;
            st->bits_dirty = 0;
        }
        return;
    }
    if (!st->heavy && st->settled_cnt > 0) {
        st->heavy = 1;
        st->mode = 3;
        st->pull = st->settled_cnt >= st->pull_min;
        st->smin = ~0ull;
        if (st->pull) st->bits_dirty = 1;   // this step's advance sets the bits (cleared before, below)
        return;
    }
    // any later step's advance clears a pull's bits (never the advance that sets them: a pull
    // is a mode-3 step, and the one after it is not)
    if (st->bits_dirty) {
        st->clear_bits = 1;
        st->bits_dirty = 0;
    }
    st->heavy = 0;
    st->settled_cnt = 0;
    const int64_t lim = st->win_base + kRing;
    for (int64_t b = st->cur + 1; b < lim; b++) {
        const int s = (int)(b % kRing);
        if (st->ring_cnt[s] > 0) {
            // bucket fusion: the later buckets of a sparse tail (SYN-8_5 from bucket ~20: ~40 K
            // entries, almost no light edges) cost a plan/advance/relax triple each, mostly
            // fixed cost; while the entries stay within `fuse`, the next buckets are opened
            // with it and settled as one.  Distances are the relaxation fixed point whatever
            // the grouping (a heavy edge landing inside the group goes past it, as always).
            uint32_t tot = st->ring_cnt[s];
            int64_t last = b;
            for (int64_t b2 = b + 1; b2 < lim && b2 < b + st->fuse_max; b2++) {
                const uint32_t c = st->ring_cnt[b2 % kRing];
                if (tot + c > st->fuse) break;
                tot += c;
                last = b2;
            }
            st->cur = last;
            st->mode = 1;
            st->slot = s;
            st->nslots = (int32_t)(last - b + 1);
            st->consume = s;
            st->consume_n = st->nslots;
            return;
        }
    }
    const int src = st->epoch & 1;
    if (st->ovf_cnt[src] > 0) {
        st->split_src = src;
        st->epoch++;
        st->ovf_cnt[st->epoch & 1] = 0;
        const int64_t mb = (int64_t)min(st->ovf_minb, 4000000000000000000ull);
        st->win_base = max(st->cur + 1, mb);
        st->cur = st->win_base - 1;
        st->ovf_minb = ~0ull;
        st->mode = 2;
        return;
    }
    st->done = 1;
}

// Mode 1: turn the opened ring bucket into near items (and settled-list entries);
// mode 2: split the overflow into the new ring window;
// mode 3: emit heavy-phase items for the bucket's settled list and record the distance
//         their edges are relaxed with.
// Ring / overflow entries whose edges were all relaxed at their current distance are dropped.
__global__ __launch_bounds__(kSsspBlock) void k_sssp_advance(SsspBufs B) {
    const SsspState *st = B.st;
    if (st->clear_bits) {   // a past pull's settled bitmap, cleared by the whole grid
        uint4 *w4 = reinterpret_cast<uint4 *>(B.sbits);
        for (uint32_t i = blockIdx.x * kSsspBlock + threadIdx.x; i < B.nbits / 4; i += gridDim.x * kSsspBlock)
            w4[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    const int mode = st->mode;
    if (mode == 0) return;
    const int32_t r = st->round;
    const int qin = r & 1;
    const int32_t *list;
    uint32_t count;
    int32_t fslot = 0, fn = 1;
    if (mode == 1) {
        fslot = st->slot;
        fn = st->nslots;
        list = B.ring + (uint64_t)fslot * B.ring_cap;
        count = 0;
        for (int j = 0; j < fn; j++) count += st->ring_cnt[(fslot + j) % kRing];
    } else if (mode == 2) {
        list = B.ovf[st->split_src];
        count = st->ovf_cnt[st->split_src];
    } else {
        list = B.settled;
        count = st->settled_cnt;
    }
    // dense opening: when the opened slots hold more than n / 16 entries (SYN-8_5's window
    // after its first pulled heavy phase: 3.4 M ring entries for 157 K live vertices, 419 us of
    // random reads), scan every vertex's bucket stamp instead -- a vertex is live in the opened
    // buckets exactly when its stamp names one of them (a push always stamps the bucket it
    // enters, every later push only lowers it, and opened buckets never receive pushes), so the
    // sequential 4 n bytes of stamps replace the entries' three random reads each
    const uint32_t dense_div = B.dense_div;
    const bool dense = mode == 1 && dense_div > 0 && (uint64_t)count * dense_div > B.ring_cap;
    const uint32_t dom = dense ? (uint32_t)B.ring_cap : count;
    if ((uint64_t)blockIdx.x * kSsspBlock >= dom) return;   // no entry for this workgroup
    __shared__ uint32_t fcnt[kRing];                            // fused slots' entry counts (mode 1)
    if (fn > 1 && (int)threadIdx.x < fn) fcnt[threadIdx.x] = st->ring_cnt[(fslot + threadIdx.x) % kRing];
    __syncthreads();
    const int64_t cur = st->cur, win_base = st->win_base, lim = win_base + kRing;
    const int32_t epoch = st->epoch;
    const bool pull = mode == 3 && st->pull;
    unsigned long long mymin = ~0ull, n_skip = 0;
    const uint32_t stride = gridDim.x * kSsspBlock;
    const uint32_t nround = (dom + stride - 1) / stride;
    const int32_t lo32 = (int32_t)(cur - (fn - 1));   // the first opened bucket (stamps are 32-bit)
    // pushes are staged per wave in LDS and flushed in bulk, as in k_sssp_relax
    __shared__ Stage stages[kSsspBlock / kWave];
    Stage &sg = stages[threadIdx.x / kWave];
    uint32_t staged = 0;
    const int lane = threadIdx.x & (kWave - 1);
    uint64_t *near_out = B.q[qin];
    uint32_t *near_count = &B.st->qcnt[qin];
    int32_t *ovf = B.ovf[epoch & 1];
    uint32_t *ovf_count = &B.st->ovf_cnt[epoch & 1];
    for (uint32_t it = 0; it < nround; it++) {
        const uint32_t f = it * stride + blockIdx.x * kSsspBlock + threadIdx.x;
        bool to_near = false, to_ring = false, to_ovf = false, to_set = false;
        int32_t v = 0;
        int slot = 0, fj = 0;
        uint32_t nch = 0;
        if (dense) {
            if (f < dom) {
                v = (int32_t)f;
                const uint32_t k = (uint32_t)B.bstamp[v] - (uint32_t)lo32;
                if (k < (uint32_t)fn) {
                    if (B.dist[v] == B.relaxed[v]) {
                        n_skip++;
                    } else {
                        B.nsw[v] = nsw_pack(cur, r);
                        to_near = to_set = true;
                        nch = chunks_of(B.lend[v] - B.rp[v]);
                    }
                }
            }
        } else if (f < count) {
            if (fn > 1) {   // entry f of the fused slots' concatenation
                uint32_t g = f;
                int j = 0;
                while (g >= fcnt[j]) g -= fcnt[j++];
                fj = j;
                v = B.ring[(uint64_t)((fslot + j) % kRing) * B.ring_cap + g];
            } else {
                v = list[f];
            }
            const unsigned long long db = B.dist[v];
            if (mode == 3) {
                B.relaxed[v] = db;   // heavy edges now, light edges already relaxed at db
                if (pull) {
                    mymin = min(mymin, db);
                    atomicOr(&B.sbits[(uint32_t)v >> 5], 1u << (v & 31));
                } else {
                    to_near = true;
                    nch = chunks_of(B.rp[v + 1] - B.lend[v]);
                }
            } else if (db == B.relaxed[v]) {
                n_skip++;
            } else if (mode == 1) {
                // entries are unique within a slot (plain stores); a vertex can sit in two
                // fused slots, so there the near stamp is claimed
                // a vertex pushed to several buckets of a fused group has one live entry, in the
                // slot of the bucket its bstamp names (later pushes only lower it): the others are
                // skipped without the exchange a claim would cost (3.4 M of them when SYN-8_5's
                // window opens whole)
                if (fn == 1 || B.bstamp[v] == (int32_t)(cur - (fn - 1) + fj)) {
                    B.nsw[v] = nsw_pack(cur, r);
                    to_near = to_set = true;
                    nch = chunks_of(B.lend[v] - B.rp[v]);
                }
            } else {
                const int64_t b = max(bucket_of(bitsd(db), B.inv_delta), win_base);
                if (b < lim) {
                    B.bstamp[v] = (int32_t)b;
                    slot = (int)(b % kRing);
                    to_ring = true;
                } else {
                    B.ostamp[v] = epoch;
                    to_ovf = true;
                    mymin = min(mymin, (unsigned long long)b);
                }
            }
        }
        const bool take = to_near | to_ring | to_ovf;
        const uint64_t mask = __ballot(take);
        if (mask == 0) continue;
        if (take) {
            const uint32_t pos = staged + (uint32_t)__popcll(mask & ((1ull << lane) - 1));
            sg.v[pos] = v;
            sg.tag[pos] = to_near ? ((uint32_t)kTagNear | (to_set ? 0x80u : 0u) | (nch << 8))
                                  : (to_ovf ? (uint32_t)kTagOvf : (uint32_t)slot);
        }
        staged += (uint32_t)__popcll(mask);
        if (staged > (uint32_t)(kStage - kWave)) stage_flush(sg, staged, B, near_out, near_count, ovf, ovf_count);
    }
    stage_final(stages, staged, B, near_out, near_count, ovf, ovf_count);
    if (mode == 2) wave_min_to(mymin, &B.st->ovf_minb);
    if (pull) wave_min_to(mymin, &B.st->smin);
    wave_count(B.stats, 7, n_skip);
}

// Heavy phase pulled by its targets (undirected graphs: the heavy edge (u, v, w) of a settled
// u is also the heavy edge (v, u, w) of v).  When the settled list holds a large share of the
// vertices -- the first buckets of a power-law graph hold most of the giant component --
// pushing its heavy edges scans far more edges than can improve anything: nearly all of them
// lead to vertices settled already.  Pulling skips every vertex whose distance is at most
// fl(smin + delta), the smallest value a heavy relaxation from this bucket can produce, and
// relaxes the heavy edges of the rest whose source is on the settled list (its bit in sbits),
// with the push's operands (dist[u] + w) and the push's strict-min test, so the distances
// are bit-identical.  Lanes take 64 consecutive vertices and walk their concatenated heavy
// edges as k_sssp_relax walks items; a vertex's candidates meet in an LDS min (its whole row
// is in the wave), so each improved vertex is written and queued once, by its own lane.
__device__ __forceinline__ void sssp_pull(const SsspBufs &B, Stage *stages, unsigned long long *vmin) {
    Stage &sg = stages[threadIdx.x / kWave];
    constexpr int kSlots = 4;
    const SsspState *st = B.st;
    const int64_t cur = st->cur, lim = st->win_base + kRing;
    const int32_t epoch = st->epoch;
    const unsigned long long bound = dbits(bitsd(st->smin) + B.delta);
    const uint64_t n = B.ring_cap;
    uint64_t *near_out = B.q[0];   // a pull never pushes near items
    uint32_t *near_count = &B.st->qcnt[0];
    int32_t *ovf = B.ovf[epoch & 1];
    uint32_t *ovf_count = &B.st->ovf_cnt[epoch & 1];
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t wave = (blockIdx.x * kSsspBlock + threadIdx.x) / kWave;
    const uint64_t nwaves = gridDim.x * (kSsspBlock / kWave);
    uint32_t staged = 0;
    unsigned long long mymin = ~0ull, c_items = 0, c_edges = 0, c_try = 0, c_impr = 0, c_ring = 0, c_ovf = 0;
    for (uint64_t base = wave * kWave; base < n; base += nwaves * kWave) {
        const uint64_t v0 = base + lane;
        int64_t rs = 0, sz = 0;
        unsigned long long dv = 0;
        if (v0 < n) {
            dv = B.dist[v0];
            if (dv > bound) {
                rs = B.lend[v0];
                sz = B.rp[v0 + 1] - rs;
                c_items += sz > 0;
            }
        }
        int64_t incl = sz;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int64_t y = __shfl_up(incl, off, kWave);
            if (lane >= off) incl += y;
        }
        const int64_t total = __shfl(incl, kWave - 1, kWave);
        if (total == 0) continue;
        const int64_t excl = incl - sz;
        vmin[lane] = dv;
        wave_lds_sync();
        for (int64_t e0 = 0; e0 < total; e0 += kWave * kSlots) {
            int64_t k[kSlots];
            int32_t u[kSlots], ss[kSlots], to[kSlots];
            unsigned long long tdv[kSlots], du[kSlots];
            double wk[kSlots];
            bool act[kSlots];
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                const int64_t e_raw = e0 + q * kWave + lane;
                act[q] = e_raw < total;
                const int64_t e = act[q] ? e_raw : total - 1;   // keep the loads in range
                int o = 0;
#pragma unroll
                for (int step = kWave / 2; step > 0; step >>= 1)
                    if (__shfl(incl, o + step - 1, kWave) <= e) o += step;
                k[q] = __shfl(rs, o, kWave) + (e - __shfl(excl, o, kWave));
                tdv[q] = __shfl(dv, o, kWave);
                to[q] = o;
            }
#pragma unroll
            for (int q = 0; q < kSlots; q++) u[q] = B.ci[k[q]];
#pragma unroll
            for (int q = 0; q < kSlots; q++) wk[q] = B.w[k[q]];
#pragma unroll
            for (int q = 0; q < kSlots; q++) ss[q] = (int32_t)((B.sbits[(uint32_t)u[q] >> 5] >> (u[q] & 31)) & 1u);
            // the settled sources' distances only: the 1 MB bitmap (SYN-8_5) stays in the XCD's L2
            // where a per-vertex stamp (32 MB) came from the Infinity Cache, and most in-edges of an
            // unsettled vertex start at unsettled ones
#pragma unroll
            for (int q = 0; q < kSlots; q++)
                du[q] = ss[q] ? __hip_atomic_load(&B.dist[u[q]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0ull;
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                c_edges += act[q];
                if (act[q] && ss[q]) {
                    c_try++;
                    const unsigned long long ndb = dbits(bitsd(du[q]) + wk[q]);
                    if (ndb < tdv[q]) atomicMin(&vmin[to[q]], ndb);
                }
            }
        }
        wave_lds_sync();
        const unsigned long long m = vmin[lane];
        wave_lds_sync();
        bool to_ring = false, to_ovf = false;
        int slot = 0;
        if (m < dv) {
            __hip_atomic_store(&B.dist[v0], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c_impr++;
            int64_t b = bucket_of(bitsd(m), B.inv_delta);
            if (b <= cur) b = cur + 1;
            // v0 is this lane's alone in a pull (its candidates met in LDS), so no other lane
            // pushes it in this launch: a plain test and store instead of a claim's exchange
            if (b < lim) {
                if (B.bstamp[v0] != (int32_t)b) {
                    B.bstamp[v0] = (int32_t)b;
                    to_ring = true;
                    slot = (int)(b % kRing);
                }
            } else {
                if (B.ostamp[v0] != epoch) {
                    B.ostamp[v0] = epoch;
                    to_ovf = true;
                }
                mymin = min(mymin, (unsigned long long)b);
            }
        }
        c_ring += to_ring;
        c_ovf += to_ovf;
        const bool take = to_ring | to_ovf;
        const uint64_t mask = __ballot(take);
        if (mask == 0) continue;
        if (take) {
            const uint32_t pos = staged + (uint32_t)__popcll(mask & ((1ull << lane) - 1));
            sg.v[pos] = (int32_t)v0;
            sg.tag[pos] = to_ovf ? (uint32_t)kTagOvf : (uint32_t)slot;
        }
        staged += (uint32_t)__popcll(mask);
        if (staged > (uint32_t)(kStage - kWave)) stage_flush(sg, staged, B, near_out, near_count, ovf, ovf_count);
    }
    stage_final(stages, staged, B, near_out, near_count, ovf, ovf_count);
    wave_min_to(mymin, &B.st->ovf_minb);
    if (B.stats) {
        wave_count(B.stats, 0, c_items);
        wave_count(B.stats, 1, c_edges);
        wave_count(B.stats, 2, c_try);
        wave_count(B.stats, 3, c_impr);
        wave_count(B.stats, 5, c_ring);
        wave_count(B.stats, 6, c_ovf);
    }
}

// Relax the light (w < delta) or, in the heavy phase, the heavy out-edges of every near item;
// improved targets go to the next near queue, a ring slot or the overflow by their new bucket.
// Heavy relaxations always land past the current bucket (forced there if rounding says
// otherwise), so the heavy phase is a single round per bucket.
// Load-balanced waves: a wave takes 64 items (one per lane), scans their edge counts and then
// walks the concatenated edge range 64 x kSlots edges at a time, every lane finding the item
// that owns its edge by a 6-step binary search over the scanned counts.  All lanes stay busy
// whatever the degrees, and each lane keeps kSlots independent gather chains in flight.
__global__ __launch_bounds__(kSsspBlock) void k_sssp_relax(SsspBufs B) {
    constexpr int kSlots = 4;
    const SsspState *st = B.st;
    const int32_t r = st->round;
    const int qin = r & 1;
    const uint32_t count = st->qcnt[qin];
    const bool heavy = st->heavy != 0;
    __shared__ Stage stages[kSsspBlock / kWave];
    Stage &sg = stages[threadIdx.x / kWave];
    if (heavy && st->pull) {
        __shared__ unsigned long long vmin[kSsspBlock];
        sssp_pull(B, stages, vmin + (threadIdx.x & ~(kWave - 1)));
        return;
    }
    if (count == 0) return;
    const int64_t cur = st->cur, lim = st->win_base + kRing;
    const int32_t epoch = st->epoch, rn = r + 1;
    const uint64_t *near_in = B.q[qin];
    uint64_t *near_out = B.q[qin ^ 1];
    uint32_t *near_count = &B.st->qcnt[qin ^ 1];
    int32_t *ovf = B.ovf[epoch & 1];
    uint32_t *ovf_count = &B.st->ovf_cnt[epoch & 1];
    const __amdgpu_buffer_rsrc_t dist_r =
        __builtin_amdgcn_make_buffer_rsrc(B.dist, (short)0, (int)(B.ring_cap * 8u), 0x00020000);
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = (blockIdx.x * kSsspBlock + threadIdx.x) / kWave;
    const uint32_t nwaves = gridDim.x * (kSsspBlock / kWave);
    uint32_t staged = 0;
    unsigned long long mymin = ~0ull, c_items = 0, c_edges = 0, c_try = 0, c_impr = 0, c_near = 0, c_ring = 0,
                       c_ovf = 0;
    // a wave takes up to 64 items, fewer when the queue is short, so that small rounds (a
    // hub's chunks) spread over all waves instead of serialising in a few
    const uint32_t ipw = min((uint32_t)kWave, max(1u, (count + nwaves - 1) / nwaves));
    if ((uint64_t)blockIdx.x * (kSsspBlock / kWave) * ipw >= count) return;   // no item for this workgroup
    for (uint64_t base = (uint64_t)wave * ipw; base < count; base += (uint64_t)nwaves * ipw) {
        const uint64_t idx = base + lane;
        int64_t rs = 0;
        int32_t sz = 0;
        double du = 0.0;
        if (lane < (int)ipw && idx < count) {
            const uint64_t item = near_in[idx];
            const int32_t u = (int32_t)(item >> 32);
            const int64_t lo = heavy ? B.lend[u] : B.rp[u], hi = heavy ? B.rp[u + 1] : B.lend[u];
            rs = lo + (int64_t)(uint32_t)item * kChunk;
            sz = (int32_t)min(hi - rs, (int64_t)kChunk);
            du = bitsd(__hip_atomic_load(&B.dist[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            c_items++;
        }
        int32_t incl = sz;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int32_t y = __shfl_up(incl, off, kWave);
            if (lane >= off) incl += y;
        }
        const int32_t total = __shfl(incl, kWave - 1, kWave);
        const int32_t excl = incl - sz;
        for (int32_t e0 = 0; e0 < total; e0 += kWave * kSlots) {
            int64_t k[kSlots];
            double dsrc[kSlots], wk[kSlots];
            int32_t v[kSlots];
            unsigned long long cd[kSlots];
            bool act[kSlots];
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                const int32_t e_raw = e0 + q * kWave + lane;
                act[q] = e_raw < total;
                const int32_t e = act[q] ? e_raw : total - 1;   // keep the loads in range
                int o = 0;
#pragma unroll
                for (int step = kWave / 2; step > 0; step >>= 1)
                    if (__shfl(incl, o + step - 1, kWave) <= e) o += step;
                k[q] = __shfl(rs, o, kWave) + (e - __shfl(excl, o, kWave));
                dsrc[q] = __shfl(du, o, kWave);
            }
#pragma unroll
            for (int q = 0; q < kSlots; q++) wk[q] = B.w[k[q]];
#pragma unroll
            for (int q = 0; q < kSlots; q++) v[q] = B.ci[k[q]];
            // idle slots get an out-of-range offset: the buffer load drops them without a
            // memory access or a branch.  A stale value only costs an extra atomicMin, it is
            // never below the true distance.
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                const bool in_class = act[q];
                cd[q] = __builtin_bit_cast(unsigned long long,
                                           __builtin_amdgcn_raw_buffer_load_b64(
                                               dist_r, in_class ? (uint32_t)v[q] * 8u : kOob, 0, 0));
            }
            // Improvements, then their dedup claims, each step issued for all slots before any
            // result is used: the claims are memory-side round trips, and chaining them slot by
            // slot serialised up to 4 x 2 of them per lane.
            int cls[kSlots];       // 0 nothing, 1 near, 2 ring slot, 3 overflow
            int32_t tag[kSlots];
            int32_t *stp[kSlots];  // ring slot / overflow stamp; near pushes claim nsw instead
            int slot[kSlots];
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                cls[q] = 0;
                tag[q] = 0;
                stp[q] = B.bstamp;
                slot[q] = 0;
                c_edges += act[q];
                if (act[q]) {
                    c_try++;
                    const double nd = dsrc[q] + wk[q];
                    const unsigned long long ndb = dbits(nd);
                    if (ndb < cd[q]) {
                        // no-return atomicMin: the pre-check decides the push.  If another lane
                        // lowered dist[v] further meanwhile, it pushes v as well: an extra push,
                        // never a missed one.
                        __hip_atomic_fetch_min(&B.dist[v[q]], ndb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        c_impr++;
                        int64_t b = bucket_of(nd, B.inv_delta);
                        if (heavy && b <= cur) b = cur + 1;
                        if (b <= cur) {
                            cls[q] = 1;
                            tag[q] = rn;
                        } else if (b < lim) {
                            cls[q] = 2;
                            stp[q] = B.bstamp + v[q];
                            tag[q] = (int32_t)b;
                            slot[q] = (int)(b % kRing);
                        } else {
                            cls[q] = 3;
                            stp[q] = B.ostamp + v[q];
                            tag[q] = epoch;
                            mymin = min(mymin, (unsigned long long)b);
                        }
                    }
                }
            }
            // claim = a plain load that filters repeats, then the exchange that settles races.  A
            // near push claims its round and its bucket's settled-list entry in one 64-bit word
            // (nsw): one exchange where two stamps took two
            int32_t seen[kSlots];
            unsigned long long nseen[kSlots];
            const unsigned long long ntag = nsw_pack(cur, rn);
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                nseen[q] = cls[q] == 1 ? __hip_atomic_load(&B.nsw[v[q]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ntag;
                seen[q] = cls[q] > 1 ? __hip_atomic_load(stp[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag[q];
            }
            bool won[kSlots], to_set[kSlots];
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                to_set[q] = false;
                if (cls[q] == 1) {
                    if ((uint32_t)nseen[q] != (uint32_t)rn) nseen[q] = atomicExch(&B.nsw[v[q]], ntag);
                    else nseen[q] = ntag;   // pushed this round already
                } else if (seen[q] != tag[q]) {
                    seen[q] = atomicExch(stp[q], tag[q]);
                }
            }
            int64_t rlo[kSlots], rhi[kSlots];
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                won[q] = cls[q] == 1 ? (uint32_t)nseen[q] != (uint32_t)rn : cls[q] != 0 && seen[q] != tag[q];
                // near pushes also join the settled list, once per bucket
                to_set[q] = cls[q] == 1 && won[q] && (uint32_t)(nseen[q] >> 32) != (uint32_t)cur;
                rlo[q] = rhi[q] = 0;
                if (won[q] && cls[q] == 1) {
                    rlo[q] = B.rp[v[q]];
                    rhi[q] = B.lend[v[q]];
                }
            }
#pragma unroll
            for (int q = 0; q < kSlots; q++) {
                const bool to_near = won[q] && cls[q] == 1, to_ring = won[q] && cls[q] == 2,
                           to_ovf = won[q] && cls[q] == 3;
                const uint32_t nch = to_near ? chunks_of(rhi[q] - rlo[q]) : 0u;
                c_near += to_near;
                c_ring += to_ring;
                c_ovf += to_ovf;
                const bool take = won[q];
                const uint64_t mask = __ballot(take);
                if (mask == 0) continue;
                if (take) {
                    const uint32_t pos = staged + (uint32_t)__popcll(mask & ((1ull << lane) - 1));
                    sg.v[pos] = v[q];
                    sg.tag[pos] = to_near ? ((uint32_t)kTagNear | (to_set[q] ? 0x80u : 0u) | (nch << 8))
                                          : (to_ovf ? (uint32_t)kTagOvf : (uint32_t)slot[q]);
                }
                staged += (uint32_t)__popcll(mask);
                if (staged > (uint32_t)(kStage - kWave)) stage_flush(sg, staged, B, near_out, near_count, ovf, ovf_count);
            }
        }
    }
    stage_final(stages, staged, B, near_out, near_count, ovf, ovf_count);
    wave_min_to(mymin, &B.st->ovf_minb);
    if (B.stats) {
        wave_count(B.stats, 0, c_items);
        wave_count(B.stats, 1, c_edges);
        wave_count(B.stats, 2, c_try);
        wave_count(B.stats, 3, c_impr);
        wave_count(B.stats, 4, c_near);
        wave_count(B.stats, 5, c_ring);
        wave_count(B.stats, 6, c_ovf);
    }
}

__global__ void k_sssp_init(unsigned long long *dist, unsigned long long *relaxed, unsigned long long *nsw,
                            int32_t *bstamp, int32_t *ostamp, int64_t n) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x) {
        dist[v] = 0x7FF0000000000000ull;   // +infinity
        relaxed[v] = ~0ull;                // never equal to a distance
        nsw[v] = ~0ull;                    // round -1, bucket -1
        bstamp[v] = -1;
        ostamp[v] = 0;
    }
}

__global__ void k_sssp_seed(SsspBufs B, int32_t src, uint32_t pull_min, uint32_t fuse, int32_t fuse_max) {
    SsspState *st = B.st;
    const uint32_t nch = chunks_of(B.lend[src] - B.rp[src]);
    for (uint32_t j = threadIdx.x; j < nch; j += blockDim.x) B.q[0][j] = ((uint64_t)(uint32_t)src << 32) | j;
    if (threadIdx.x < kRing) st->ring_cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        B.dist[src] = 0ull;
        B.nsw[src] = nsw_pack(0, 0);
        B.settled[0] = src;
        st->settled_cnt = 1;
        st->cur = 0;
        st->win_base = 0;
        st->ovf_minb = ~0ull;
        st->round = -1;   // the first plan makes it 0
        st->done = 0;
        st->epoch = 1;
        st->mode = 0;
        st->heavy = 0;
        st->pull = 0;
        st->pull_min = pull_min;
        st->bits_dirty = 1;   // a past run may have left bits: the first advance clears them
        st->clear_bits = 0;
        st->smin = ~0ull;
        st->slot = 0;
        st->nslots = 1;
        st->consume = -1;
        st->consume_n = 0;
        st->fuse = fuse;
        st->fuse_max = fuse_max;
        st->split_src = 0;
        st->qcnt[0] = nch;
        st->qcnt[1] = 0;
        st->ovf_cnt[0] = st->ovf_cnt[1] = 0;
    }
}

// ---- light/heavy edge layout (built once per graph and delta, no atomics) ----
// Entries are taken in 64-entry slabs: one ballot per slab gives its light mask, so the
// number of light entries before entry e is L(e) = cpre[e/64] + popc(mask[e/64] below e).
// A row's light entries go to rp[r] + L(e) - L(rp[r]), its heavy ones after lend[r] in order.
__global__ __launch_bounds__(256) void k_light_masks(const double *__restrict__ w, int64_t nnz, double delta,
                                                     uint64_t *mask, int32_t *cnt, int64_t nslabs) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);
    for (int64_t sl = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave; sl < nslabs; sl += nw) {
        const int64_t e = sl * kWave + lane;
        const bool light = e < nnz && w[e] < delta;
        const uint64_t m = __ballot(light);
        if (lane == 0) {
            mask[sl] = m;
            cnt[sl] = __popcll(m);
        }
    }
}

__device__ __forceinline__ int64_t light_before(const uint64_t *mask, const int64_t *cpre, int64_t e) {
    const int64_t sl = e / kWave;
    const int b = (int)(e % kWave);
    return cpre[sl] + (b ? __popcll(mask[sl] & ((1ull << b) - 1)) : 0);
}

__global__ __launch_bounds__(256) void k_light_rows(const int64_t *__restrict__ rp, const uint64_t *__restrict__ mask,
                                                    const int64_t *__restrict__ cpre, int64_t n, int64_t *Ls,
                                                    int64_t *lend) {
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n; v += (int64_t)gridDim.x * 256) {
        const int64_t a = light_before(mask, cpre, rp[v]), b = light_before(mask, cpre, rp[v + 1]);
        Ls[v] = a;
        lend[v] = rp[v] + (b - a);
    }
}

// One wave per slab; lane = entry.  The slab's rows lie in [r0, r1] (two uniform binary
// searches); when that range is at most 64 rows each lane finds its row by a 6-step shuffle
// search over rp[r0+1 .. r0+64], else by its own binary search.
__global__ __launch_bounds__(256) void k_light_scatter(const int64_t *__restrict__ rp, const int64_t *__restrict__ srow,
                                                       const int32_t *__restrict__ ci,
                                                       const double *__restrict__ w, const uint64_t *__restrict__ mask,
                                                       const int64_t *__restrict__ cpre, const int64_t *__restrict__ Ls,
                                                       const int64_t *__restrict__ lend, int64_t n, int64_t nnz,
                                                       int64_t nslabs, int32_t *ci2, double *w2) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);
    for (int64_t sl = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave; sl < nslabs; sl += nw) {
        const int64_t e0 = sl * kWave, e_last = min(e0 + kWave, nnz) - 1;
        const int64_t e = e0 + lane;
        const bool valid = e < nnz;
        const int64_t ee = valid ? e : e_last;
        const int64_t r = slab_row_of(rp, srow, n, sl, ee, lane);
        if (valid) {
            const uint64_t m = mask[sl];
            const bool light = (m >> lane) & 1ull;
            const int64_t lin = cpre[sl] + (lane ? __popcll(m & ((1ull << lane) - 1)) : 0) - Ls[r];
            const int64_t pos = light ? rp[r] + lin : lend[r] + ((e - rp[r]) - lin);
            ci2[pos] = ci[e];
            w2[pos] = w[e];
        }
    }
}

int ensure_sssp_layout(gx_graph *g, double delta, hipStream_t s) {
    if (g->sssp && g->sssp->delta == delta) return GX_SUCCESS;
    const int64_t n = (int64_t)g->n, nnz = (int64_t)g->nnz;
    auto L = std::make_unique<SsspLayout>();
    L->delta = delta;
    L->n_active = n;
    GX_TRY(ensure_host_rp(g->ctx, g->A));
    if ((int64_t)g->A.h_rp.size() == n + 1) {
        L->n_active = 0;
        for (int64_t v = 0; v < n; v++) L->n_active += g->A.h_rp[v + 1] != g->A.h_rp[v];
    }
    GX_TRY(L->ci.alloc(nnz, 16));
    GX_TRY(L->w.alloc(nnz, 16));
    GX_TRY(L->lend.alloc(n));
    const int64_t nslabs = (nnz + kWave - 1) / kWave;
    DBuf<uint64_t> mask;
    DBuf<int32_t> cnt;
    DBuf<int64_t> cpre, Ls;
    GX_TRY(mask.alloc(nslabs + 1));
    GX_TRY(cnt.alloc(nslabs + 1));
    GX_TRY(cpre.alloc(nslabs + 1));
    GX_TRY(Ls.alloc(n));
    GX_HIP_TRY(hipMemsetAsync(cnt.p + nslabs, 0, sizeof(int32_t), s));
    GX_HIP_TRY(hipMemsetAsync(mask.p + nslabs, 0, sizeof(uint64_t), s));
    const unsigned wgrid = grid_for((uint64_t)nslabs * kWave, 256, 16384);
    if (nslabs) {
        hipLaunchKernelGGL(k_light_masks, dim3(wgrid), dim3(256), 0, s, g->A.w.p, nnz, delta, mask.p, cnt.p, nslabs);
        GX_TRY(check_launch("k_light_masks"));
    }
    size_t tmp_bytes = 0;
    GX_HIP_TRY(rocprim::exclusive_scan(nullptr, tmp_bytes, cnt.p, cpre.p, (int64_t)0, (size_t)(nslabs + 1),
                                       rocprim::plus<int64_t>(), s));
    DBuf<char> tmp;
    GX_TRY(tmp.alloc(tmp_bytes));
    GX_HIP_TRY(rocprim::exclusive_scan(tmp.p, tmp_bytes, cnt.p, cpre.p, (int64_t)0, (size_t)(nslabs + 1),
                                       rocprim::plus<int64_t>(), s));
    if (n) {
        hipLaunchKernelGGL(k_light_rows, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, g->A.rp.p, mask.p, cpre.p, n,
                           Ls.p, L->lend.p);
        GX_TRY(check_launch("k_light_rows"));
    }
    if (nslabs) {
        DBuf<int64_t> srow;
        GX_TRY(srow.alloc(nslabs + 1));
        GX_TRY(slab_rows(g->A.rp.p, n, nslabs, srow.p, s));
        hipLaunchKernelGGL(k_light_scatter, dim3(wgrid), dim3(256), 0, s, g->A.rp.p, srow.p, g->A.ci.p, g->A.w.p, mask.p,
                           cpre.p, Ls.p, L->lend.p, n, nnz, nslabs, L->ci.p, L->w.p);
        GX_TRY(check_launch("k_light_scatter"));
    }
    GX_HIP_TRY(hipStreamSynchronize(s));   // the temporaries are freed on return
    delete g->sssp;
    g->sssp = L.release();
    return GX_SUCCESS;
}

// Work buffers of gx_sssp, kept with the graph's light/heavy layout so repeated runs reuse
// them, and the captured graph of kGraphSteps plan -> advance -> relax steps (its kernel
// arguments point into these buffers).  A run replays the graph, copying the done flag to
// pinned memory after each replay while the next one is already queued.
constexpr int kGraphSteps = 8;
inline uint32_t nbit_words(int64_t n) { return (uint32_t)(((n + 31) / 32 + 3) / 4 * 4); }
struct SsspWork {
    DBuf<unsigned long long> dist, relaxed;
    DBuf<unsigned long long> nsw;
    DBuf<int32_t> bstamp, ostamp, ring, ovf0, ovf1, settled;
    DBuf<uint32_t> sbits;          // settled bitmap of a pulled heavy phase (padded to 4 words)
    DBuf<uint64_t> q0, q1;
    DBuf<SsspState> st;
    int32_t *h_done = nullptr;     // round, done of the state (pinned)
    int replays_hint = 0;          // replays the last run needed (the next run queues as many)
    hipEvent_t ev = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    hipStream_t g_stream = nullptr;
    unsigned g_grid = 0;
    ~SsspWork() {
        if (gexec) (void)hipGraphExecDestroy(gexec);
        if (graph) (void)hipGraphDestroy(graph);
        if (ev) (void)hipEventDestroy(ev);
        if (h_done) (void)hipHostFree(h_done);
    }
    int alloc(int64_t n, uint64_t qcap) {
        GX_TRY(dist.alloc(n));
        GX_TRY(relaxed.alloc(n));
        GX_TRY(nsw.alloc(n));
        GX_TRY(bstamp.alloc(n));
        GX_TRY(ostamp.alloc(n));
        GX_TRY(sbits.alloc(nbit_words(n)));
        GX_HIP_TRY(hipMemset(sbits.p, 0, nbit_words(n) * 4));
        GX_TRY(settled.alloc(n));
        GX_TRY(ring.alloc((uint64_t)n * kRing));
        GX_TRY(ovf0.alloc(n));
        GX_TRY(ovf1.alloc(n));
        GX_TRY(q0.alloc(qcap));
        GX_TRY(q1.alloc(qcap));
        GX_TRY(st.alloc(1));
        GX_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h_done), 2 * sizeof(int32_t), hipHostMallocDefault));
        GX_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        return GX_SUCCESS;
    }
    int enqueue_steps(const SsspBufs &B, unsigned grid, int k, hipStream_t s) {
        for (int i = 0; i < k; i++) {
            hipLaunchKernelGGL(k_sssp_plan, dim3(1), dim3(1), 0, s, B.st);
            hipLaunchKernelGGL(k_sssp_advance, dim3(grid), dim3(kSsspBlock), 0, s, B);
            hipLaunchKernelGGL(k_sssp_relax, dim3(grid), dim3(kSsspBlock), 0, s, B);
        }
        return check_launch("k_sssp_relax");
    }
    int capture(const SsspBufs &B, unsigned grid, hipStream_t s) {
        if (gexec && g_stream == s && g_grid == grid) return GX_SUCCESS;
        if (gexec) (void)hipGraphExecDestroy(gexec);
        if (graph) (void)hipGraphDestroy(graph);
        gexec = nullptr;
        graph = nullptr;
        GX_HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        const int rc = enqueue_steps(B, grid, kGraphSteps, s);
        hipGraph_t gr = nullptr;
        const hipError_t e = hipStreamEndCapture(s, &gr);
        if (rc != GX_SUCCESS) {
            if (gr) (void)hipGraphDestroy(gr);
            return rc;
        }
        if (e != hipSuccess) return fail(GX_DEVICE_ERROR, std::string("gx_sssp capture: ") + hipGetErrorString(e));
        graph = gr;
        GX_HIP_TRY(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
        g_stream = s;
        g_grid = grid;
        return GX_SUCCESS;
    }
};

__global__ __launch_bounds__(256) void k_sum_weights(const double *__restrict__ w, int64_t m, double *sum) {
    double acc = 0.0;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < m; k += (int64_t)gridDim.x * 256) acc += w[k];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) atomicAdd(sum, acc);
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_sssp(gx_graph *g, uint64_t src, double *dist_out) {
    if (!g || !dist_out) return fail(GX_NULL_POINTER, "gx_sssp: null argument");
    if (!g->weighted) return fail(GX_INVALID_VALUE, "gx_sssp: graph has no edge weights");
    if (src >= g->n) return fail(GX_INVALID_INDEX, "gx_sssp: source out of range");
    if ((int64_t)g->n >= kMaxBufVertices)
        return fail(GX_NOT_IMPLEMENTED, "gx_sssp: more than 2^28 vertices (buffer-load offsets are 31-bit)");
    {
        gx_graph *h = nullptr;   // hub-first copy from the second call (gx_runtime.hip hub_for)
        GX_TRY(hub_for(g, ++g->sssp_calls, &h, &src));
        if (h) return gx_sssp(h, src, dist_out);
    }
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n;
    const uint64_t qcap = (uint64_t)n + g->nnz / kChunk + 64;
    // bucket width delta = scale * mean weight / mean degree (GX_SSSP_DELTA overrides); any
    // positive value gives the same distances, it only trades rounds for re-relaxations
    if (g->mean_w < 0.0) {
        double mean = 1.0;
        if (g->nnz) {
            DBuf<double> sum;
            GX_TRY(sum.alloc(1));
            GX_HIP_TRY(hipMemsetAsync(sum.p, 0, sizeof(double), s));
            hipLaunchKernelGGL(k_sum_weights, dim3(grid_for(g->nnz, 256, 4096)), dim3(256), 0, s, g->A.w.p,
                               (int64_t)g->nnz, sum.p);
            GX_TRY(check_launch("k_sum_weights"));
            double h = 0.0;
            GX_HIP_TRY(hipMemcpyAsync(&h, sum.p, sizeof(double), hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            mean = h / (double)g->nnz;
        }
        g->mean_w = mean;
    }
    // measured on the SYN stand-ins with bucket fusion: 2 for undirected graphs,
    // whose big early buckets are pulled (round 5 re-sweep after the dense opening,
    // profiles/r05_sssp_dscale_sweep.txt: against 3, SYN-8_5 5.88 -> 5.61 ms, SYN-g500-22
    // 3.56 -> 3.01, SYN-7_5 1.91 -> 1.80; round 3 had chosen 3 over 4), 0.5 for directed ones
    double delta = 0.0, scale = g->directed ? 0.5 : 2.0;
    if (const char *e = std::getenv("GX_SSSP_DELTA")) delta = std::atof(e);
    if (const char *e = std::getenv("GX_SSSP_DSCALE")) scale = std::atof(e);
    if (!(delta > 0.0)) {
        const double avg_deg = g->nnz ? (double)g->nnz / (double)n : 1.0;
        delta = scale * g->mean_w / std::max(1.0, avg_deg);
        if (!(delta > 0.0) || !std::isfinite(delta)) delta = 1.0;
    }
    const double inv_delta = 1.0 / delta;
    const bool verbose = std::getenv("GX_SSSP_VERBOSE") != nullptr;
    DBuf<unsigned long long> stats;
    if (verbose) {
        GX_TRY(stats.alloc(8 * kStatLanes));
        GX_HIP_TRY(hipMemsetAsync(stats.p, 0, 8 * kStatLanes * sizeof(unsigned long long), s));
    }
    GX_TRY(device_begin(ctx));
    {
        KTimer kt(ctx, "sssp_layout", s);
        GX_TRY(ensure_sssp_layout(g, delta, s));
    }
    SsspLayout &lay = *g->sssp;
    if (!lay.work) {
        auto w = std::make_shared<SsspWork>();
        GX_TRY(w->alloc(n, qcap));
        lay.work = w;
    }
    SsspWork &W = *static_cast<SsspWork *>(lay.work.get());
    auto &dist = W.dist, &relaxed = W.relaxed;
    auto &nsw = W.nsw;
    auto &bstamp = W.bstamp, &ostamp = W.ostamp;
    auto &st = W.st;
    SsspBufs B{g->A.rp.p,   lay.lend.p,   lay.ci.p,      lay.w.p,    dist.p,       relaxed.p,  nsw.p,
               bstamp.p,    ostamp.p,     W.sbits.p,     nbit_words(n), {W.q0.p, W.q1.p}, W.ring.p,
               {W.ovf0.p, W.ovf1.p},
               W.settled.p, (uint64_t)n,  delta,         inv_delta,  st.p,         stats.p, 16u};
    if (const char *e = std::getenv("GX_SSSP_DENSE")) B.dense_div = (uint32_t)std::strtoul(e, nullptr, 10);

    hipLaunchKernelGGL(k_sssp_init, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, dist.p, relaxed.p, nsw.p,
                       bstamp.p, ostamp.p, n);
    GX_TRY(check_launch("k_sssp_init"));
    // heavy phases whose settled list holds at least 1/GX_SSSP_PULL_FRAC (default 8) of the
    // non-isolated vertices are pulled (undirected graphs; GX_SSSP_PULL=0 never, 2 always).
    // 8 rather than 4: the same times at the default bucket width, and no cliff below it (a
    // scale of 2-2.5 left SYN-8_5's first bucket short of 1/4 and pushed it: 14.8 ms; 8.2 at 1/8)
    uint32_t pull_min = 0xFFFFFFFFu;
    {
        const char *e = std::getenv("GX_SSSP_PULL");
        const int mode = e ? std::atoi(e) : 1;
        const char *f = std::getenv("GX_SSSP_PULL_FRAC");
        const double frac = f ? std::atof(f) : 8.0;
        if (!g->directed && mode == 2) pull_min = 1;
        else if (!g->directed && mode == 1 && frac > 0.0)
            pull_min = (uint32_t)std::max<double>(1.0, std::ceil((double)lay.n_active / frac));
    }
    // bucket fusion bounds (GX_SSSP_FUSE entries, 0 = one bucket at a time; GX_SSSP_FUSE_MAX
    // buckets)
    uint32_t fuse = 0xFFFFFFFFu;
    int32_t fuse_max = kRing;
    if (const char *e = std::getenv("GX_SSSP_FUSE")) fuse = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GX_SSSP_FUSE_MAX")) fuse_max = std::max(1, std::min(kRing, std::atoi(e)));
    hipLaunchKernelGGL(k_sssp_seed, dim3(1), dim3(256), 0, s, B, (int32_t)src, pull_min, fuse, fuse_max);
    GX_TRY(check_launch("k_sssp_seed"));
    const unsigned grid = (unsigned)std::max(1, ctx->num_cus) * 8;
    // a bound every correct run stays far below: each step settles a vertex or a bucket
    const uint64_t max_steps = 8ull * (uint64_t)n + 4ull * (uint64_t)g->nnz + 1000000ull;
    uint64_t steps = 0;
    int batch = 4;
    int32_t done = 0;
    // GX_SSSP_VERBOSE=2: one step per batch, a line per step (bucket, phase, items, work, time)
    const bool per_step = verbose && std::atoi(std::getenv("GX_SSSP_VERBOSE")) >= 2;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    unsigned long long prev[8] = {};
    if (per_step) {
        batch = 1;
        GX_HIP_TRY(hipEventCreate(&ev0));
        GX_HIP_TRY(hipEventCreate(&ev1));
    }
    const void *res = nullptr;   // the distances to download (set once remapped)
    const char *ge = std::getenv("GX_SSSP_GRAPH");
    if (!verbose && !ctx->timing && !(ge && std::atoi(ge) == 0)) {
        // replayed step graph: one replay always queued behind the one whose done flag is read.
        // The first batch is as many replays as the last run on this layout needed; when that
        // was enough, the remap to the caller's order (hub-first copy) is queued behind it
        // instead of an idle replay, and runs while the host reads the flag.
        GX_TRY(W.capture(B, grid, s));
        // capped, so that one long run (a deep chain) cannot queue many idle replays for the next
        const int hint = std::min(W.replays_hint, 12);
        auto read_state = [&]() -> int {
            GX_HIP_TRY(hipMemcpyAsync(W.h_done, &st.p->round, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipEventRecord(W.ev, s));
            return GX_SUCCESS;
        };
        for (int i = 0; i < std::max(1, hint); i++) GX_HIP_TRY(hipGraphLaunch(W.gexec, s));
        steps += (uint64_t)std::max(1, hint) * kGraphSteps;
        GX_TRY(read_state());
        if (hint > 0) {
            GX_TRY(remap_out(g, dist.p, 8, s, &res));
        } else {
            GX_HIP_TRY(hipGraphLaunch(W.gexec, s));
            steps += kGraphSteps;
        }
        GX_HIP_TRY(hipEventSynchronize(W.ev));
        if (!W.h_done[1]) res = nullptr;
        while (!W.h_done[1]) {
            GX_TRY(read_state());
            GX_HIP_TRY(hipGraphLaunch(W.gexec, s));
            GX_HIP_TRY(hipEventSynchronize(W.ev));
            steps += kGraphSteps;
            if (steps > max_steps) return fail(GX_PANIC, "gx_sssp: delta-stepping did not converge");
        }
        W.replays_hint = (W.h_done[0] + kGraphSteps) / kGraphSteps;   // round + 1 plan steps ran
        done = 1;
    }
    while (!done) {
        if (per_step) {
            hipLaunchKernelGGL(k_sssp_plan, dim3(1), dim3(1), 0, s, st.p);
            SsspState h;
            GX_HIP_TRY(hipMemcpyAsync(&h, st.p, sizeof(h), hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipEventRecord(ev0, s));
            hipLaunchKernelGGL(k_sssp_advance, dim3(grid), dim3(kSsspBlock), 0, s, B);
            hipLaunchKernelGGL(k_sssp_relax, dim3(grid), dim3(kSsspBlock), 0, s, B);
            GX_HIP_TRY(hipEventRecord(ev1, s));
            std::vector<unsigned long long> raw(8 * kStatLanes);
            GX_HIP_TRY(hipMemcpyAsync(raw.data(), stats.p, raw.size() * sizeof(raw[0]), hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipMemcpyAsync(&done, &st.p->done, sizeof(int32_t), hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            float ms = 0.f;
            GX_HIP_TRY(hipEventElapsedTime(&ms, ev0, ev1));
            unsigned long long c[8] = {};
            for (int i = 0; i < 8 * kStatLanes; i++) c[i / kStatLanes] += raw[i];
            std::fprintf(stderr, "step %llu round %d bucket %lld mode %d heavy %d pull %d near %u settled %u | %.1f us "
                         "items %llu edges %llu improved %llu near %llu ring %llu\n",
                         (unsigned long long)steps, h.round, (long long)h.cur, h.mode, h.heavy, h.pull,
                         h.qcnt[h.round & 1], h.settled_cnt, ms * 1e3, c[0] - prev[0], c[1] - prev[1],
                         c[3] - prev[3], c[4] - prev[4], c[5] - prev[5]);
            std::memcpy(prev, c, sizeof(c));
            if (++steps > max_steps) return fail(GX_PANIC, "gx_sssp: delta-stepping did not converge");
            continue;
        }
        for (int i = 0; i < batch; i++) {
            hipLaunchKernelGGL(k_sssp_plan, dim3(1), dim3(1), 0, s, st.p);
            {
                KTimer kt(ctx, "sssp_advance", s);
                hipLaunchKernelGGL(k_sssp_advance, dim3(grid), dim3(kSsspBlock), 0, s, B);
            }
            {
                KTimer kt(ctx, "sssp_relax", s);
                hipLaunchKernelGGL(k_sssp_relax, dim3(grid), dim3(kSsspBlock), 0, s, B);
            }
        }
        GX_TRY(check_launch("k_sssp_relax"));
        steps += batch;
        GX_HIP_TRY(hipMemcpyAsync(&done, &st.p->done, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        if (steps > max_steps) return fail(GX_PANIC, "gx_sssp: delta-stepping did not converge");
        batch = std::min(batch * 2, 32);
    }
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (!res) GX_TRY(remap_out(g, dist.p, 8, s, &res));
    GX_TRY(device_end(ctx));
    if (verbose) {
        SsspState h;
        GX_HIP_TRY(hipMemcpy(&h, st.p, sizeof(h), hipMemcpyDeviceToHost));
        std::vector<unsigned long long> raw(8 * kStatLanes);
        GX_HIP_TRY(hipMemcpy(raw.data(), stats.p, raw.size() * sizeof(raw[0]), hipMemcpyDeviceToHost));
        unsigned long long c[8] = {};
        for (int i = 0; i < 8 * kStatLanes; i++) c[i / kStatLanes] += raw[i];
        std::fprintf(stderr,
                     "gx_sssp: delta %g rounds %d last bucket %lld epochs %d launched steps %llu | items %llu edges "
                     "%llu tried %llu improved %llu near %llu ring %llu ovf %llu skipped %llu\n",
                     delta, h.round, (long long)h.cur, h.epoch, (unsigned long long)steps, c[0], c[1], c[2], c[3],
                     c[4], c[5], c[6], c[7]);
    }
    GX_TRY(download(ctx, dist_out, res, (uint64_t)n, Xfer::Raw64));
    return GX_SUCCESS;
}

GX_MODULE_WARMER(sssp)
