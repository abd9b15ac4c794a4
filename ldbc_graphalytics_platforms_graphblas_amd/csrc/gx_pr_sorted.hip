// gx_pr_sorted.hip -- PageRank pull SpMV over column-sorted row blocks (k_pr_pull_units).
//
// Same iteration as k_pr_pull (gx_pr.hip; Graphalytics PR, LAGr_PageRankGX pr.cpp:61):
//     r(v) = teleport + sum_{u in in(v)} x(u);   x'(v) = r(v) / (outdeg(v)/d)
// but the x gathers are issued in column order.
//
// Why: gathering row by row, a 64-lane instruction covered 1.33 gathers per 128-B line of x on
// SYN-7_5 (44.7 M L2 requests per launch).  Sorting the entries of a block of rows by column
// puts equal and neighbouring columns into the same instruction, and each block sweeps x in
// increasing address order.
//
// Layout (built once per plan on the device by a radix sort of (block << 32 | column)):
//   spk[e]   uint32 : (column - group base) << 14 | row of the entry within its block
//   gbase[g] uint32 : base column of 64-entry group g; bit 31 set = escape: the group spans
//                     >= 2^18 columns and reads them from sci
//   sci[e]   int32  : the columns of the escape groups
// A block keeps the CSR range [rp[row_begin], rp[row_end]) of its rows and streams 4 B per
// entry, like the CSR column index.  Inside every full 64-entry group the entries are then
// permuted (k_sorted_laneperm) so that each LDS-add instruction hits distinct banks; the
// group's column set, hence its gathers' lines, is unchanged.
// Gathered values are added into LDS row accumulators (ds_add_f64) in wave-arrival order:
// scores agree with the row-order sum to ~1e-15 relative but are not bit-reproducible run to
// run (the parity bar is 1e-12 relative, tests/test_gpu_parity.py).
//
// Each sorted block is cut into interleaved units (one work item each, LDS accumulators for
// every row of the block); a multi-unit block's units combine through write-through slabs and
// an arrival ticket.  Items run one workgroup each, or, on launches of >= 2 items per CU, from
// a device work queue drained by one resident workgroup per CU (k_pr_pull_units QUEUE).  Rows longer than `long_nnz` take the LONG path (a workgroup per
// 8192-entry segment, in row order); their workgroups come first.  A block without any entry
// (isolated vertices: 29.5 % of SYN-7_5's rows) runs only the epilogue.  Its rows were also
// tried as 64 Ki-row blocks at the end of the grid: a CU streams one such block's epilogue at
// ~100 GB/s, ~15 us, which lengthened the launch (SYN-7_5 100-104 us against 85-86).
#include <algorithm>
#include <functional>
#include <queue>
#include <thread>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gx_pr.h"

namespace gx {
namespace {

constexpr int kRowBits = 14;     // packed entry: (column - group base) << kRowBits | row in block
constexpr int kBS = 1024;        // threads of a k_pr_pull_units workgroup (16 waves, one per CU)
constexpr int kCombRows = (1 << kRowBits) / kBS;   // rows per thread in a slab combine (16)
constexpr int kU = 8;            // entries per lane and round (two 16-B index loads)
constexpr int kRound = kBS * kU; // entries of one round of a workgroup
constexpr int kNSg = 512;        // codes of a narrow supergroup: one wave's 16-B load per lane
constexpr int kJunkRow = (1 << kRowBits) - kWave;   // accumulators [16320, 16384) absorb fillers
constexpr int kMaxBlockRows = kJunkRow;             // rows of a sorted block
static_assert(kMaxBlockRows == kPlanBlockRows, "gx_pr.h block rows");

struct SortedArgs {
    const RowBlock *blocks;
    const int32_t *ci;       // row-order columns (LONG rows)
    const int32_t *sci;      // block-sorted columns (escape groups)
    const uint32_t *spk;     // packed entries
    const uint32_t *gbase;   // per 64-entry group: base column, bit 31 = escape
    const int32_t *outdeg;
    const double *x_in;
    double *x_out;
    double *rank_out;
    int64_t chunk;
    int nranks;
    int zero_slot;
    int32_t zero_col;        // a padding slot of x that holds 0.0 (chunk - 2)
    double teleport0, damping_over_n, damping;
    const int32_t *long_first;
    const int32_t *long_nseg;
    double *long_part;
    uint32_t *long_ticket;
    uint32_t nlong, nlong_pad;
    // fused dangling sum: per block slot or -1, partials, ticket
    const int32_t *dslot;
    double *dpart;
    uint32_t *dticket;
    uint32_t ndblocks;
    // split blocks
    const SortedUnit *units;
    uint32_t nunits;
    double *uslab;
    uint32_t *uticket;
    uint64_t *utimes;        // debug (GX_PR_UNIT_TIMES): per workgroup start, gather end, end, XCC
    const uint16_t *npk;     // narrow codes
    const uint32_t *nbase;   // per narrow supergroup: the column before its first code
    uint32_t null_sg;        // all-padding supergroup (base = zero_col)
    uint32_t nt_col;         // CP bit 2: narrow supergroups from this column on gathered non-temporally
    double *xd;              // x of the rows past `live` (store_x, gx_pr.h)
    int64_t live;
    // paced sweep (PrPart::pace)
    const int32_t *pace_rounds;
    uint32_t *pace_prog;
    uint32_t pace_nw, pace_d, pace_polls, pace_ncus;
    // work queue (GX_PR_QUEUE): [0] next work item, [1] workgroups done (reset by the last)
    uint32_t *queue;
    // combine kernel (PrPart::comb_kernel): the units of multi-unit blocks only store their slabs
    int comb;
    const CombStripe *cstripes;
};

// Returns the row's score if the row is dangling (out-degree 0), else 0.
__device__ __forceinline__ double sorted_epilogue(const SortedArgs &a, int64_t row, double s, double teleport) {
    const double r = teleport + s;
    if (a.rank_out) a.rank_out[row] = r;
    const int32_t deg = a.outdeg[row];
    store_x(a.x_out, a.xd, a.live, row, deg > 0 ? r / ((double)deg / a.damping) : r);
    return deg > 0 ? 0.0 : r;
}

// The epilogue of rows [r0, r0 + nrows) of a block, thread tid taking rows tid, tid + kBS, ...:
// eight out-degree loads issued before any store, since the compiler cannot move a load of
// outdeg above a store to x_out (they might alias) and the row-by-row loop paid one memory
// latency per row a thread handles (16 for SYN-8_5's 16 320-row blocks).  acc null: sums 0.
// Returns the thread's dangling-score sum.
__device__ __forceinline__ double epilogue_rows(const SortedArgs &a, int64_t r0, int nrows, const double *acc,
                                                double teleport) {
    constexpr int kB = 8;
    double d = 0.0;
    for (int i0 = threadIdx.x; i0 < nrows; i0 += kB * kBS) {
        int32_t deg[kB];
#pragma unroll
        for (int q = 0; q < kB; q++) {
            const int i = i0 + q * kBS;
            deg[q] = i < nrows ? a.outdeg[r0 + i] : 1;
        }
#pragma unroll
        for (int q = 0; q < kB; q++) {
            const int i = i0 + q * kBS;
            if (i >= nrows) break;
            const double r = teleport + (acc ? acc[i] : 0.0);
            if (a.rank_out) a.rank_out[r0 + i] = r;
            store_x(a.x_out, a.xd, a.live, r0 + i, deg[q] > 0 ? r / ((double)deg[q] / a.damping) : r);
            if (deg[q] == 0) d += r;
        }
    }
    return d;
}

// Fused dangling sum: the block's dangling scores d (one value per thread) are reduced, the
// block publishes its partial in its slot (agent scope) and takes a ticket; the last of the
// ndblocks participants adds the partials up with the whole workgroup (thread t takes slots
// t, t + kBS, ...; fixed tree, so the order is fixed) into the chunk's last x slot.
template <int BS = kBS>
__device__ __forceinline__ void dangling_publish(const SortedArgs &a, int32_t slot, double d, double *wred, int *last) {
    const int tid = threadIdx.x;
    d = wave_sum(d);
    __syncthreads();   // wred may still be read by an earlier reduction
    if ((tid & (kWave - 1)) == 0) wred[tid / kWave] = d;
    __syncthreads();
    if (tid == 0) {
        double tot = 0.0;
#pragma unroll
        for (int w = 0; w < BS / kWave; w++) tot += wred[w];
        __hip_atomic_store(&a.dpart[slot], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t t = __hip_atomic_fetch_add(a.dticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last = t == a.ndblocks - 1;
    }
    __syncthreads();
    if (!*last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    double v = 0.0;
    for (uint32_t j = tid; j < a.ndblocks; j += BS) v += __hip_atomic_load(&a.dpart[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = wave_sum(v);
    __syncthreads();
    if ((tid & (kWave - 1)) == 0) wred[tid / kWave] = v;
    __syncthreads();
    if (tid == 0) {
        double all = 0.0;
#pragma unroll
        for (int w = 0; w < BS / kWave; w++) all += wred[w];
        __hip_atomic_store(a.dticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.x_out[a.chunk - 1] = all;
    }
}

// LONG: one segment of one long row (row order), a whole workgroup; segments of one row are
// combined by the last arriver (agent-scope release/acquire ticket).
__device__ __forceinline__ void long_segment(const SortedArgs &a, const RowBlock &b, double *wred, double teleport) {
    const int tid = threadIdx.x;
    const int64_t zb = b.nz_begin, ze = b.nz_end;
    double s0 = 0.0, s1 = 0.0;
    for (int64_t k0 = zb + tid; k0 < ze; k0 += (int64_t)kU * kBS) {
        int32_t c[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) c[u] = __builtin_nontemporal_load(a.ci + min(k0 + (int64_t)u * kBS, ze - 1));
        double g[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) g[u] = a.x_in[c[u]];
#pragma unroll
        for (int u = 0; u < kU; u++)
            if (k0 + (int64_t)u * kBS < ze) ((u & 1) ? s1 : s0) += g[u];
    }
    const double s = wave_sum(s0 + s1);
    if ((tid & (kWave - 1)) == 0) wred[tid / kWave] = s;
    __syncthreads();
    if (tid != 0) return;
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < kBS / kWave; w++) tot += wred[w];
    const int32_t sp = b.split;
    const int32_t nseg = a.long_nseg[sp];
    if (nseg == 1) {
        sorted_epilogue(a, b.row_begin, tot, teleport);
        return;
    }
    const int32_t first = a.long_first[sp];
    // publish the partial (agent scope), then take a ticket; the last arriver combines
    __hip_atomic_store(&a.long_part[first + b.seg], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(&a.long_ticket[sp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t != (uint32_t)(nseg - 1)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    double all = 0.0;
    for (int j = 0; j < nseg; j++)
        all += __hip_atomic_load(&a.long_part[first + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.long_ticket[sp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sorted_epilogue(a, b.row_begin, all, teleport);
}

// Adds x(column) of the sorted entries [lo, hi) of block b into the LDS row accumulators,
// taking every (step / kRound)-th round of kRound entries from the one holding lo (the
// interleaved units of a split block; lo - nz_begin is a multiple of kRound).
//
// Four entries per lane from one 16-B index load (X4): what bounds the launch is the CU's
// vector memory and LDS instruction stream (timing probes).  Wave w takes the
// kU / 4 256-entry supergroups [R + 256 (w kU/4 + v), +256) of round R; lane l holds entries
// 4l .. 4l+3 of each.  A supergroup has one base column, a scalar load, so a lane's columns are
// base + (entry >> 14) with no per-lane select.  Pipelined across rounds: round k+1's gathers
// are issued before round k's LDS adds, the index loads two rounds ahead, buffers A/B
// alternating (a copy of a pending load would wait for it).  Positions are block-relative
// 32-bit values.  An entry outside [lo, hi) gathers the zero padding slot x[zero_col] and adds
// 0.0 to whatever row its (clamped or neighbouring) index word names -- below 16 Ki, and the
// launch reserves 16 Ki accumulators -- so the hot path has no 64-bit compares or masks.  The
// columns of escape supergroups (spanning >= 2^18 ids) come from sci inside a uniform branch
// that consumes its loads there: a load merged into the columns after the branch made the
// compiler drain every outstanding load (s_waitcnt vmcnt(0)) each round.
//
// PROBE (diagnostic builds only, -DGX_PR_PROBES, tools/pr_probe.sh; wrong results by design):
// 1 no LDS adds (register sum), 2 no gathers, 3 neither, 4 gathers folded into x[c & 4095]
// (L1 hits), 5 no gathers + conflict-free LDS adds (acc[tid]), 6 gathers + conflict-free LDS
// adds, 7 no index loads (entries synthesised from the position, columns = the base),
// 8 gathers of columns >= 512 Ki folded into the first 512 Ki (the sparse tail as local as the
// hub lines), 9 every gather folded into the first 64 Ki columns, 10 no entries at all (the
// fixed costs: zeroing, epilogue, slabs), 11 as 3 (index loads and decode only).
// gather_narrow takes all but 7 (which runs it unchanged); 12 (gather_narrow only) reads the
// narrow entries' x from LDS (the accumulators at column mod 16 Ki): the launch if x came from
// LDS instead of the texture path; 13 (gather_narrow only) two 16-B loads per lane per 8
// entries (the instruction count of a layout loading each lane's column span once); 14
// (gather_narrow only) only the first entry of each column run gathers, the rest read 0; 15 as 14
// with the run's value handed on by ds_bpermute (correct results); 16 = the product kernel
// under the probes' launch (no queue), the baseline for 12-15; 17 the wide entries (gather_units:
// 4-byte packed entries and escapes) load and decode but do not gather (narrow unchanged), 18 no
// wide entries at all (gather_units skipped): the wide tail's share of the launch (round 6).
template <int PROBE, int CP>   // CP bit 0: index loads non-temporal (bit 2: gather_narrow)
__device__ __forceinline__ void gather_units(const SortedArgs &a, const RowBlock &b, int64_t lo64, int64_t hi64,
                                             double *acc, int64_t step64, int32_t k0 = 0, int32_t k1 = 0x7fffffff) {
    const int tid = threadIdx.x;
    const int64_t z0 = b.nz_begin;
    const int32_t lo = (int32_t)(lo64 - z0), hi = (int32_t)(hi64 - z0), step = (int32_t)step64;
    if (lo >= hi) return;
    const int32_t last = (int32_t)(b.nz_end - z0) - 1;
    const int32_t nsg = (last >> 8) + 1;   // supergroups of the block
    const uint32_t span = (uint32_t)(hi - lo);
    const uint32_t *spk = a.spk + z0;
    const int32_t *sci = a.sci + z0;
    const uint32_t *sgb = a.gbase + b.seg;
    const int32_t zc = a.zero_col;
    const char *xb = reinterpret_cast<const char *>(a.x_in);
    const int lane = tid & (kWave - 1);
    constexpr int V = kU / 4;
    const int wave = tid >> 6;
    struct Rd {
        uint4 q[V];
        uint32_t bq;   // lane l: the base of supergroup l mod V (a vector load, see below)
    };
    struct Gt {
        double g[kU];
        uint32_t r[kU];
    };
    // The supergroup bases come in through one vector load per round (lanes l mod V) read back
    // with v_readlane: a scalar load's wait (lgkmcnt) would also wait for the LDS adds in flight.
    auto load = [&](Rd &d, int32_t R) {
        const int32_t sg0 = R + wave * V * 256;
#pragma unroll
        for (int v = 0; v < V; v++) {
            const int32_t sg = sg0 + v * 256;
            if constexpr (PROBE == 7) {
                const uint32_t e0 = (uint32_t)(sg + 4 * lane) & 4095u;
                d.q[v] = make_uint4(e0, (e0 + 1) & 4095u, (e0 + 2) & 4095u, (e0 + 3) & 4095u);
            } else {
                // clamped into the block; spk's allocation slack covers the 3 entries past `last`;
                // the address is a CSR offset, only 4-B aligned (gx_u32x4)
                const gx_u32x4 *qa = reinterpret_cast<const gx_u32x4 *>(spk + min(sg + 4 * lane, last));
                const gx_u32x4 q4 = (CP & 1) ? __builtin_nontemporal_load(qa) : *qa;
                d.q[v] = make_uint4(q4.x, q4.y, q4.z, q4.w);
            }
        }
        d.bq = sgb[min((sg0 >> 8) + (lane & (V - 1)), nsg - 1)];
    };
    auto issue = [&](const Rd &d, int32_t R, Gt &t) {
        int32_t c[kU];
        uint32_t sb[V], esc = 0;
#pragma unroll
        for (int v = 0; v < V; v++) {
            sb[v] = __builtin_amdgcn_readlane(d.bq, v);
            esc |= sb[v];
        }
#pragma unroll
        for (int v = 0; v < V; v++) {
            const uint32_t w4[4] = {d.q[v].x, d.q[v].y, d.q[v].z, d.q[v].w};
            const int32_t d0 = R + (wave * V + v) * 256 + 4 * lane - lo;
            const uint32_t base = sb[v] & 0x7fffffffu;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int i = 4 * v + j;
                const bool ok = (uint32_t)(d0 + j) < span;
                t.r[i] = w4[j] & ((1u << kRowBits) - 1);
                // materialised here: sunk to the adds, the rows would keep this buffer's index
                // registers live past its reload, and the allocator copies at the loop latch
                asm volatile("" : "+v"(t.r[i]));
                if constexpr (PROBE == 7) c[i] = ok ? (int32_t)base : zc;
                else c[i] = ok ? (int32_t)(base + (w4[j] >> kRowBits)) : zc;
            }
        }
        if (PROBE != 7 && (esc & 0x80000000u)) {   // uniform: an escape supergroup in this round
#pragma unroll
            for (int v = 0; v < V; v++) {
                if (!(sb[v] & 0x80000000u)) continue;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int i = 4 * v + j;
                    const int32_t pos = R + (wave * V + v) * 256 + 4 * lane + j;
                    if ((uint32_t)(pos - lo) < span) c[i] = sci[pos];
                }
            }
            // consume the loads here: a column register still waiting on one at the branch's end
            // makes the compiler wait for every load in flight (vmcnt(0)) on both paths
            __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
        }
#pragma unroll
        for (int i = 0; i < kU; i++) {
            if constexpr (PROBE == 2 || PROBE == 3 || PROBE == 5 || PROBE == 11 || PROBE == 17) t.g[i] = (double)c[i];
            else if constexpr (PROBE == 4) t.g[i] = a.x_in[c[i] & 4095];
            else if constexpr (PROBE == 8) t.g[i] = a.x_in[c[i] >= (1 << 19) ? (c[i] & ((1 << 19) - 1)) : c[i]];
            else if constexpr (PROBE == 9) t.g[i] = a.x_in[c[i] & 65535];
            else t.g[i] = *reinterpret_cast<const double *>(xb + ((uint32_t)c[i] << 3));
        }
    };
    double rsum = 0.0;   // PROBE 1 / 3
    auto add = [&](const Gt &t) {
#pragma unroll
        for (int i = 0; i < kU; i++) {
            if constexpr (PROBE == 1 || PROBE == 3 || PROBE == 11) rsum += t.g[i];
            else if constexpr (PROBE == 5 || PROBE == 6) atomicAdd(&acc[tid], t.g[i]);
            else atomicAdd(&acc[t.r[i]], t.g[i]);
        }
    };
    // Two rounds per trip of a counted loop with a single exit.  The stages are fenced from
    // the scheduler and the exits are not shared: a load hoisted above the issue that still
    // reads its buffer, or one exit block adding "tA or tB", makes the register allocator copy
    // a buffer at the loop latch, and a copy waits for the loads in flight.
    // rounds [k0, k1) of this unit (a paced sweep's window; all of them by default)
    const int32_t nr = min((hi - lo + step - 1) / step, k1) - k0;
    if (nr <= 0) return;
    Rd dA, dB;
    Gt tA, tB;
    int32_t R = lo + k0 * step;
    load(dA, R);
    load(dB, R + step);
    issue(dA, R, tA);
    __builtin_amdgcn_sched_barrier(0);
    load(dA, R + 2 * step);
    int32_t k = 1;
    for (; k + 1 < nr; k += 2) {
        __builtin_amdgcn_sched_barrier(0);
        issue(dB, R + step, tB);
        __builtin_amdgcn_sched_barrier(0);
        load(dB, R + 3 * step);
        __builtin_amdgcn_sched_barrier(0);
        add(tA);
        __builtin_amdgcn_sched_barrier(0);
        issue(dA, R + 2 * step, tA);
        __builtin_amdgcn_sched_barrier(0);
        load(dA, R + 4 * step);
        __builtin_amdgcn_sched_barrier(0);
        add(tB);
        R += 2 * step;
    }
    if (k < nr) {
        issue(dB, R + step, tB);
        add(tA);
        add(tB);
    } else {
        add(tA);
    }
    if constexpr (PROBE == 1 || PROBE == 3 || PROBE == 11) atomicAdd(&acc[tid], rsum);
}

// Inclusive prefix sum over the 64 lanes by DPP moves (row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast:15 and row_bcast:31 across rows); lanes whose source is out of range or
// whose row is masked add the `old` operand, 0.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}

// The narrow prefix of a block: 2-byte codes (delta << 14) | row, delta = the column step from
// the previous code (0..3; a larger step is split by filler codes of step 3 whose rows are
// junk accumulators >= kJunkRow).  A narrow supergroup of 512 codes is one wave-load of 16 B
// per lane (lane l: codes l + 64 k, stored lane-major), decoded by two packed DPP scans (issue
// below).  Round i of the unit is
// the workgroup's 16 supergroups (j + i k) * 16 + wave; a supergroup past the block reads the
// null supergroup (padding codes, base = x's zero slot), so the loop has no range checks.
// Same pipeline as gather_units: round i+1's gathers issue before round i's LDS adds, the
// loads two rounds ahead, buffers A/B alternating.
template <int CP, int PROBE = 0>
__device__ __forceinline__ void gather_narrow(const SortedArgs &a, const SortedUnit &u, double *acc, int32_t i0 = 0,
                                              int32_t i1 = 0x7fffffff) {
    constexpr int W = kBS / kWave;   // supergroups per round
    const int32_t nrounds = (u.nsg + W - 1) / W;
    if (u.unit >= nrounds) return;
    // rounds [i0, i1) of this unit (a paced sweep's window; all of them by default)
    const int32_t nr = min((nrounds - u.unit + u.nunits - 1) / u.nunits, i1) - i0;
    if (nr <= 0) return;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid >> 6;
    const uint32_t sg0 = (uint32_t)(u.nbeg / kNSg);
    const char *xb = reinterpret_cast<const char *>(a.x_in);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // 16-B aligned (512-code runs)
    struct Rd {
        u32x4 q;
        uint32_t base;
    };
    struct Gt {
        double g[kU];
        uint32_t r[kU];
        uint64_t m[kU];   // PROBE 15: the leader mask of instruction k
    };
    auto load = [&](Rd &d, int32_t i) {
        const int32_t sg = (u.unit + (i + i0) * u.nunits) * W + wave;
        const uint32_t g = sg < u.nsg ? sg0 + (uint32_t)sg : a.null_sg;
        const u32x4 *qa = reinterpret_cast<const u32x4 *>(a.npk + (size_t)g * kNSg) + lane;
        d.q = (CP & 1) ? __builtin_nontemporal_load(qa) : *qa;
        d.base = a.nbase[g];
    };
    // Lane l holds the codes of entries l + 64 k (k < 8) of the supergroup, so instruction k
    // gathers 64 consecutive sorted entries (3x fewer distinct lines per instruction than 8
    // consecutive entries per lane on SYN-8_5).  The eight lane scans run packed, four 8-bit
    // fields per register (a field's sum is at most 64 x 3), in two DPP scans; entry 64 k + l
    // sits at base + (the column steps of instructions < k) + field k of the scan.
    auto issue = [&](const Rd &d, Gt &t) {
        const uint32_t w[4] = {d.q.x, d.q.y, d.q.z, d.q.w};
        uint32_t pk[2] = {0u, 0u};
#pragma unroll
        for (int k = 0; k < kU; k++) {
            const uint32_t c = (k & 1) ? (w[k >> 1] >> 16) : (w[k >> 1] & 0xffffu);
            pk[k >> 2] |= (c >> kRowBits) << (8 * (k & 3));
            t.r[k] = c & ((1u << kRowBits) - 1);
            asm volatile("" : "+v"(t.r[k]));
        }
        const uint32_t s0 = wave_scan_incl(pk[0]), s1 = wave_scan_incl(pk[1]);
        const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)s0, kWave - 1);
        const uint32_t t1 = (uint32_t)__builtin_amdgcn_readlane((int)s1, kWave - 1);
        uint32_t bk = (uint32_t)__builtin_amdgcn_readfirstlane((int)d.base);
        const uint32_t b0 = bk;
        uint32_t col[kU];
#pragma unroll
        for (int k = 0; k < kU; k++) {
            const uint32_t sk = k < 4 ? s0 : s1, tk = k < 4 ? t0 : t1;
            col[k] = bk + ((sk >> (8 * (k & 3))) & 255u);
            bk += (tk >> (8 * (k & 3))) & 255u;
        }
        if constexpr (PROBE == 14 || PROBE == 15) {
            // only the first entry of each column run gathers (a zero step repeats the previous
            // sorted entry's column, lane 0 always loads): 14 leaves the others at 0, 15 hands the
            // leader's value to them by ds_bpermute in the add stage (correct results)
            const bool ntl = (CP & 4) && b0 >= a.nt_col;
#pragma unroll
            for (int k = 0; k < kU; k++) {
                const uint32_t st = ((k < 4 ? pk[0] : pk[1]) >> (8 * (k & 3))) & 255u;
                const bool lead = st != 0u || lane == 0;
                if constexpr (PROBE == 15) t.m[k] = __builtin_amdgcn_ballot_w64(lead);
                double v = 0.0;
                if (lead) {
                    const double *xp = reinterpret_cast<const double *>(xb + (col[k] << 3));
                    v = ntl ? __builtin_nontemporal_load(xp) : *xp;
                }
                t.g[k] = v;
            }
        } else if constexpr (PROBE == 13) {
            // two 16-B loads per lane instead of eight 8-B gathers: the instruction count of a
            // layout whose lane loads its entries' column span once
            typedef double d2 __attribute__((ext_vector_type(2)));
            const d2 *x2 = reinterpret_cast<const d2 *>(a.x_in);
            const uint32_t p0 = col[0] >> 1;
            const d2 A = x2[p0], B = x2[p0 + 1];
#pragma unroll
            for (int k = 0; k < kU; k++) t.g[k] = (k & 3) == 0 ? A.x : (k & 3) == 1 ? A.y : (k & 3) == 2 ? B.x : B.y;
            (void)b0;
        } else if constexpr (PROBE == 2 || PROBE == 3 || PROBE == 5 || PROBE == 11 || PROBE == 4 || PROBE == 8 || PROBE == 9 ||
                      PROBE == 12) {
#pragma unroll
            for (int k = 0; k < kU; k++) {
                const uint32_t c = col[k];
                if constexpr (PROBE == 2 || PROBE == 3 || PROBE == 5 || PROBE == 11) t.g[k] = (double)c;
                else if constexpr (PROBE == 12) t.g[k] = acc[c & ((1u << kRowBits) - 1)];   // x from LDS
                else if constexpr (PROBE == 4) t.g[k] = a.x_in[c & 4095u];
                else if constexpr (PROBE == 8) t.g[k] = a.x_in[c >= (1u << 19) ? (c & ((1u << 19) - 1)) : c];
                else t.g[k] = a.x_in[c & 65535u];
            }
            (void)b0;
        } else if ((CP & 4) && b0 >= a.nt_col) {   // past the hub lines: streamed (GX_PR_CP bit 2)
#pragma unroll
            for (int k = 0; k < kU; k++) t.g[k] = __builtin_nontemporal_load(reinterpret_cast<const double *>(xb + (col[k] << 3)));
        } else {
#pragma unroll
            for (int k = 0; k < kU; k++) t.g[k] = *reinterpret_cast<const double *>(xb + (col[k] << 3));
        }
    };
    double rsum = 0.0;   // PROBE 1 / 3 / 11: register sum instead of the LDS adds
    const uint64_t lane_le = (2ull << lane) - 1;   // PROBE 15: lanes 0..lane
    auto add = [&](const Gt &t) {
#pragma unroll
        for (int k = 0; k < kU; k++) {
            if constexpr (PROBE == 15) {
                const int src = 63 - __builtin_clzll(t.m[k] & lane_le);   // bit 0 is always set
                const uint64_t b = __builtin_bit_cast(uint64_t, t.g[k]);
                const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)b);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)(b >> 32));
                atomicAdd(&acc[t.r[k]], __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo));
            } else if constexpr (PROBE == 1 || PROBE == 3 || PROBE == 11) rsum += t.g[k];
            else if constexpr (PROBE == 5 || PROBE == 6) atomicAdd(&acc[threadIdx.x], t.g[k]);
            else atomicAdd(&acc[t.r[k]], t.g[k]);
        }
    };
    Rd dA, dB;
    Gt tA, tB;
    load(dA, 0);
    load(dB, 1);
    issue(dA, tA);
    __builtin_amdgcn_sched_barrier(0);
    load(dA, 2);
    int32_t k = 1;
    for (; k + 1 < nr; k += 2) {
        __builtin_amdgcn_sched_barrier(0);
        issue(dB, tB);
        __builtin_amdgcn_sched_barrier(0);
        load(dB, k + 2);
        __builtin_amdgcn_sched_barrier(0);
        add(tA);
        __builtin_amdgcn_sched_barrier(0);
        issue(dA, tA);
        __builtin_amdgcn_sched_barrier(0);
        load(dA, k + 3);
        __builtin_amdgcn_sched_barrier(0);
        add(tB);
    }
    if (k < nr) {
        issue(dB, tB);
        add(tA);
        add(tB);
    } else {
        add(tA);
    }
    if constexpr (PROBE == 1 || PROBE == 3 || PROBE == 11) atomicAdd(&acc[threadIdx.x], rsum);
}

// Paced sweep (PrPart::pace): the CU slot of this workgroup inside its XCD (SE, SH, CU ids of
// HW_REG_HW_ID bits 8..15) and the XCD's progress words (HW_REG_XCC_ID).  Placement is read,
// not assumed; it only steers speed (cdna_hip_programming.md §1: never correctness).
__device__ __forceinline__ uint32_t *pace_slot(const SortedArgs &a) {
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;         // HW_REG_XCC_ID[3:0]
    const uint32_t cu = (uint32_t)__builtin_amdgcn_s_getreg((7 << 11) | (8 << 6) | 4) & 255u;   // HW_REG_HW_ID[15:8]
    return a.pace_prog + xcc * 256u + cu;
}

// Entering window `win` of generation `gen`: publish it, then wait (bounded: pace_polls polls)
// until no unit of the same generation on this XCD is more than pace_d windows behind.  The
// whole workgroup waits at the barriers; wave 0 polls the XCD's 256 slots with L1-bypassing
// 16-B loads (L2-served; the slots are written with plain stores, which stay in L2).
__device__ __forceinline__ void pace_wait(const SortedArgs &a, uint32_t *slot, uint32_t gen, uint32_t win) {
    __syncthreads();
    if (threadIdx.x < kWave) {
        const uint32_t me = (gen << 16) | (win + 1);
        if (threadIdx.x == 0) *reinterpret_cast<volatile uint32_t *>(slot) = me;
        const gx_u32x4 *base = reinterpret_cast<const gx_u32x4 *>(a.pace_prog + (size_t)(slot - a.pace_prog) / 256 * 256);
        for (uint32_t p = 0; p < a.pace_polls; p++) {
            const gx_u32x4 q = __builtin_nontemporal_load(base + threadIdx.x);
            const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
            uint32_t lo = 0xffffu;
#pragma unroll
            for (int j = 0; j < 4; j++)
                if ((w4[j] >> 16) == gen && (w4[j] & 0xffffu)) lo = min(lo, w4[j] & 0xffffu);
            for (int off = 32; off > 0; off >>= 1) lo = min(lo, (uint32_t)__shfl_xor((int)lo, off, kWave));
            if (win + 1 <= lo + a.pace_d) break;
            __builtin_amdgcn_s_sleep(4);
        }
    }
    __syncthreads();
}

// One iteration's SpMV over split blocks.  Work items: [0, nlong_pad) LONG row segments (padded
// to a multiple of 8), then the units (largest first; the blocks of rows without entries last).  A multi-unit block's units store their row sums write-through (sc1) to
// their own slab, drain them (vmcnt(0)) and take a ticket; the last arriver adds the slabs in
// unit order with sc1 loads and runs the epilogue (MI355X_MICROARCH.md "Valid forms": sc1 stores
// drained before the counter add, sc1 loads by the workgroup whose add came last).
// TIMES: debug build with per-workgroup timestamps (GX_PR_UNIT_TIMES).
template <bool TIMES, int PROBE, int CP, bool PACE>
__device__ __forceinline__ void pull_item(const SortedArgs &a, const uint32_t w, double *acc, double *wred, int &last,
                                          const double teleport) {
    const int tid = threadIdx.x;
    __shared__ uint64_t ts[2];   // TIMES: start, gather end (LDS, so no registers are held)
    if (TIMES && tid == 0) ts[0] = __builtin_amdgcn_s_memrealtime();
    auto stamp = [&]() {
        if (TIMES && tid == 0) {
            a.utimes[4 * w + 0] = ts[0];
            a.utimes[4 * w + 1] = ts[1];
            a.utimes[4 * w + 2] = __builtin_amdgcn_s_memrealtime();
            a.utimes[4 * w + 3] = (uint64_t)__builtin_amdgcn_s_getreg((3 << 11) | 20);   // HW_REG_XCC_ID[3:0]
        }
    };
    if (a.zero_slot && w == 0 && tid == 0) a.x_out[a.chunk - 1] = 0.0;
    if (w < a.nlong_pad) {
        if (w < a.nlong) long_segment(a, a.blocks[w], wred, teleport);
        stamp();
        return;
    }
    const SortedUnit u = a.units[w - a.nlong_pad];
    const RowBlock b = {u.z0, u.z1, u.r0, u.r1, -1, u.seg};
    const int nrows = b.row_end - b.row_begin;
    // a block without entries (the isolated vertices a hub-first undirected graph puts last):
    // r = teleport, no accumulators, no gathers
    const bool empty = b.nz_begin == b.nz_end;
    if (!empty) {
        for (int i = tid; i < nrows; i += kBS) acc[i] = 0.0;
        __syncthreads();
        if constexpr (PACE) {
            // window by window: the narrow rounds, then the wide rounds starting in it
            const uint32_t nw = a.pace_nw;
            const int32_t *pr = a.pace_rounds + (size_t)(w - a.nlong_pad) * 2 * (nw + 1);
            uint32_t *slot = pace_slot(a);
            const uint32_t gen = (w - a.nlong_pad) / a.pace_ncus;
            for (uint32_t win = 0; win < nw; win++) {
                const int32_t n0 = pr[win], n1 = pr[win + 1], w0 = pr[nw + 1 + win], w1 = pr[nw + 2 + win];
                if (n0 == n1 && w0 == w1) continue;
                pace_wait(a, slot, gen, win);
                if (n1 > n0) gather_narrow<CP, PROBE>(a, u, acc, n0, n1);
                if (w1 > w0) gather_units<PROBE, CP>(a, b, u.lo, u.hi, acc, u.step, w0, w1);
            }
            __syncthreads();
            if (tid == 0) *reinterpret_cast<volatile uint32_t *>(slot) = 0u;   // this CU's sweep is over
        } else if constexpr (PROBE != 10) {   // probe 10: no entries at all (the fixed costs)
            gather_narrow<CP, PROBE>(a, u, acc);
            if constexpr (PROBE != 18) gather_units<PROBE, CP>(a, b, u.lo, u.hi, acc, u.step);
        }
        __syncthreads();
    }
    if (TIMES && tid == 0) ts[1] = __builtin_amdgcn_s_memrealtime();
    if (u.nunits > 1 && a.comb) {
        // the combine kernel adds the slabs after this launch (the launch boundary orders them)
        double *mine = a.uslab + u.slab + (int64_t)u.unit * nrows;
        for (int i = tid; i < nrows; i += kBS) mine[i] = acc[i];
        stamp();
        return;
    }
    if (u.nunits > 1) {
        double *mine = a.uslab + u.slab + (int64_t)u.unit * nrows;
        for (int i = tid; i < nrows; i += kBS)
            __hip_atomic_store(&mine[i], acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const uint32_t t = __hip_atomic_fetch_add(&a.uticket[u.part], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = t == (uint32_t)(u.nunits - 1);
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&a.uticket[u.part], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (!last) {
            stamp();
            return;
        }
        // after tid 0's acquire (this CU's L1 invalidated) and the barrier, plain loads see the
        // other units' slabs.  All kCombRows rows of a thread at once (a block's 16 Ki rows in
        // one pass), so a slab costs one round trip: the slabs live beyond this XCD's L2, and
        // four rows at a time made the combine of 5 slabs ~30 us of a 1/8 piece's 80
        // (tools/unit_times.py).  The adds keep unit order.
        const double *slabs = a.uslab + u.slab;
        if (2 * nrows <= kBS) {
            // few rows (the longest rows' blocks, split into up to 256 units): S threads per
            // row, thread g summing slabs g, g + S, ... 16 loads at a time, then the S partials
            // added in group order through LDS above the block's rows -- a row-per-thread loop
            // would take one round trip per slab (256 on a 1/8 piece's first block)
            int S = 2;
            while (4 * S * nrows <= 2 * kBS && S < u.nunits) S *= 2;
            double *part = acc + (1 << (kRowBits - 1));
            const int r = tid % nrows, g = tid / nrows;
            if (g < S) {
                double s = 0.0;
                for (int j0 = g; j0 < u.nunits; j0 += kCombRows * S) {
                    double v[kCombRows];
#pragma unroll
                    for (int q = 0; q < kCombRows; q++) {
                        const int j = j0 + q * S;
                        v[q] = j < u.nunits ? slabs[(int64_t)j * nrows + r] : 0.0;
                    }
#pragma unroll
                    for (int q = 0; q < kCombRows; q++) s += v[q];
                }
                part[g * nrows + r] = s;
            }
            __syncthreads();
            if (tid < nrows) {
                double s = 0.0;
                for (int q = 0; q < S; q++) s += part[q * nrows + tid];
                acc[tid] = s;
            }
        } else
        for (int i0 = tid; i0 < nrows; i0 += kCombRows * kBS) {
            double s[kCombRows];
#pragma unroll
            for (int q = 0; q < kCombRows; q++) s[q] = 0.0;
            for (int j = 0; j < u.nunits; j++) {
                const double *sl = slabs + (int64_t)j * nrows;
                double v[kCombRows];
#pragma unroll
                for (int q = 0; q < kCombRows; q++) v[q] = i0 + q * kBS < nrows ? sl[i0 + q * kBS] : 0.0;
#pragma unroll
                for (int q = 0; q < kCombRows; q++) s[q] += v[q];
            }
#pragma unroll
            for (int q = 0; q < kCombRows; q++)
                if (i0 + q * kBS < nrows) acc[i0 + q * kBS] = s[q];
        }
        // each thread reads back only the acc entries it wrote: no barrier needed
    }
    double d = 0.0;
    if (empty)
        d = epilogue_rows(a, b.row_begin, nrows, nullptr, teleport);
    else
        d = epilogue_rows(a, b.row_begin, nrows, acc, teleport);
    if (a.dslot) {
        const int32_t slot = a.dslot[u.blk];
        if (slot >= 0) dangling_publish(a, slot, d, wred, &last);
    }
    stamp();
}

// The slabs of the multi-unit blocks (GX_PR_COMBINE=1), one workgroup per row stripe of at
// most kCombBS rows: S threads per row (S = 1 for full stripes, up to kCombBS / rows for the
// few-row blocks of the longest rows), thread g adding slabs g, g + S, ... in order, 16 loads in
// flight, then the S partials in group order; the row's epilogue; the stripe's dangling partial.
// Spread over the chip instead of one last-arriving workgroup per block, whose k round trips to
// the slabs (a 1/8 piece's 33 Mi-entry block: 75 units of 9 Ki rows) outlasted the launch.
constexpr int kCombBS = 256;
__global__ __launch_bounds__(kCombBS) void k_pr_combine(SortedArgs a) {
    __shared__ double part[kCombBS];
    __shared__ double wred[kCombBS / kWave];
    __shared__ int last;
    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    const CombStripe c = a.cstripes[blockIdx.x];
    const int rows = c.s1 - c.s0;
    int S = 1;
    while (2 * S * rows <= kCombBS && S < c.k) S *= 2;
    const int tid = threadIdx.x, r = tid % rows, g = tid / rows;
    double s = 0.0;
    if (g < S) {
        const double *sl = a.uslab + c.slab + c.s0 + r;
        for (int j0 = g; j0 < c.k; j0 += 16 * S) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const int j = j0 + q * S;
                v[q] = j < c.k ? sl[(int64_t)j * c.nrows] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < 16; q++) s += v[q];
        }
    }
    if (S > 1) {
        if (g < S) part[g * rows + r] = s;
        __syncthreads();
        if (tid < rows) {
            s = 0.0;
            for (int q = 0; q < S; q++) s += part[q * rows + tid];
        }
    }
    double d = 0.0;
    if (tid < rows) d = sorted_epilogue(a, (int64_t)c.r0 + c.s0 + tid, s, teleport);
    if (c.dslot >= 0) dangling_publish<kCombBS>(a, c.dslot, d, wred, &last);
}

// The next work item for the whole workgroup, with no divergent branch anywhere: wave 0 takes
// it (a scalar branch: readfirstlane of the thread id) by an add in which lane 0 adds 1 and the
// other lanes 0, so lane 0's return value is the item; readfirstlane makes it a scalar, which
// wave 0 stores to LDS and every wave reads back through readfirstlane again.  The caller's
// `w >= total` loop exit is therefore a uniform scalar branch.  Round 4's version took the item
// under `threadIdx.x == 0`, a divergent branch: inlined, the compiler turned that branch into
// the exit of an inner loop which the other lanes of wave 0 kept running, barriers and all,
// while lane 0 waited to fetch, and the launch never ended (a __noinline__ hid it; reading the
// slot through readfirstlane alone did not: the divergent branch was still there).
__device__ __forceinline__ uint32_t queue_fetch(uint32_t *q, uint32_t *slot) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) < (uint32_t)kWave) {
        const uint32_t v = __hip_atomic_fetch_add(q, (threadIdx.x & (kWave - 1)) == 0 ? 1u : 0u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        *slot = __builtin_amdgcn_readfirstlane(v);
    }
    __syncthreads();
    const uint32_t w = __builtin_amdgcn_readfirstlane(*slot);
    __syncthreads();   // every wave has read the slot before the next fetch rewrites it
    return w;
}

// One workgroup per work item, or (QUEUE, GX_PR_QUEUE=1) one resident workgroup per CU taking
// items from a device counter in the same order: the dispatcher deals workgroups to the XCDs
// round-robin, so an item whose XCD has no free CU waits even while other XCDs idle; from a
// queue every CU takes the next item the moment it is free.
template <bool TIMES, int PROBE = 0, int CP = 0, bool PACE = false, bool QUEUE = false>
__global__ __launch_bounds__(kBS, TIMES ? 1 : 4) void k_pr_pull_units(SortedArgs a) {
    extern __shared__ double acc[];
    __shared__ double wred[kBS / kWave];
    __shared__ int last;
    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    if constexpr (!QUEUE) {
        pull_item<TIMES, PROBE, CP, PACE>(a, blockIdx.x, acc, wred, last, teleport);
    } else {
        __shared__ uint32_t item;
        const uint32_t total = a.nlong_pad + a.nunits;
        for (;;) {
            const uint32_t w = queue_fetch(a.queue, &item);   // (its barriers: the last item's LDS is free)
            if (w >= total) break;
            pull_item<TIMES, PROBE, CP, PACE>(a, w, acc, wred, last, teleport);
        }
        if (threadIdx.x == 0 &&
            __hip_atomic_fetch_add(&a.queue[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            __hip_atomic_store(&a.queue[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.queue[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The plan's one radix sort.  The rows are cut into segments, in row order: the sorted blocks
// and each LONG row (a sorted block's rows, or one LONG row).  Entry e of local row i gets key
// (segment << colbits) | column and value i - (its segment's first row); sorted, every
// segment's entries keep its CSR range [rp[row_begin], rp[row_end]) and come out in column
// order.  Local row i is row order[i] of the source CSR with columns renamed perm[c]
// (gx_pagerank's hub-first relabelling, never materialised), or row i itself (order / perm
// null).  Sixteen entries per thread, the row found once by a binary search of the row
// pointers.
struct KeySrc {
    const int64_t *rp;          // local row pointers (the plan's, row order)
    int64_t rows;
    const int64_t *srp;         // source CSR
    const int32_t *sci;
    const int32_t *order;       // null: identity
    const int32_t *perm;        // null: columns as stored
    const int32_t *seg_row;     // nseg + 1 segment row starts
    int32_t nseg;
    int colbits;
    int32_t segmask;            // segment bits kept in the key (its sort group's share)
};

// The segment of every local row (one workgroup per segment; rows of skipped empty blocks fall
// in the segment before them and are never looked up: they hold no entry).
__global__ __launch_bounds__(256) void k_row_seg(const int32_t *__restrict__ seg_row, int32_t nseg, int32_t *rowseg) {
    for (int32_t sg = blockIdx.x; sg < nseg; sg += gridDim.x)
        for (int32_t r = seg_row[sg] + threadIdx.x; r < seg_row[sg + 1]; r += 256) rowseg[r] = sg;
}

// One wave per kKeyU 64-entry slabs of the plan's rows, lane = entry (coalesced key / row writes
// and row-contiguous column reads; the row by the slab shuffle search, gx_device.h
// slab_row_of, the segment from rowseg).  The slabs' chains (row -> source row -> column ->
// renamed column) are issued side by side: one slab at a time this kernel was a chain of
// ~15 dependent loads per slab (a binary search of the segments among them), ~10 ms on SYN-8_5.
constexpr int kKeyU = 4;

template <typename K>
__global__ __launch_bounds__(256) void k_sorted_keys(KeySrc k, int64_t nnz, const int64_t *__restrict__ srow,
                                                     int64_t nslabs, const int32_t *__restrict__ rowseg,
                                                     K *__restrict__ keys, uint16_t *__restrict__ vals) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);
    const int64_t nch = (nslabs + kKeyU - 1) / kKeyU;
    for (int64_t ch = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave; ch < nch; ch += nw) {
        int32_t i[kKeyU], sg[kKeyU], c0[kKeyU];
        int64_t rpi[kKeyU], sp[kKeyU];
        const int64_t e0 = ch * kKeyU * kWave + lane;   // lane's entry of slab u: e0 + u * kWave
#pragma unroll
        for (int u = 0; u < kKeyU; u++) {
            const int64_t sl = min(ch * kKeyU + u, nslabs - 1);
            i[u] = (int32_t)slab_row_of(k.rp, srow, k.rows, sl, min(e0 + u * kWave, nnz - 1), lane);
        }
#pragma unroll
        for (int u = 0; u < kKeyU; u++) {
            sg[u] = rowseg[i[u]];
            rpi[u] = k.rp[i[u]];
            sp[u] = k.srp[k.order ? k.order[i[u]] : i[u]];
        }
#pragma unroll
        for (int u = 0; u < kKeyU; u++) c0[u] = k.sci[sp[u] + (min(e0 + u * kWave, nnz - 1) - rpi[u])];
#pragma unroll
        for (int u = 0; u < kKeyU; u++) {
            const uint32_t c = (uint32_t)(k.perm ? k.perm[c0[u]] : c0[u]);
            const int64_t e = e0 + u * kWave;
            if (e < nnz) {
                keys[e] = ((K)(sg[u] & k.segmask) << k.colbits) | (K)c;
                vals[e] = (uint16_t)(i[u] - k.seg_row[sg[u]]);
            }
        }
    }
}

// The key pass from the source side (PrPart::job): the source entries [e0, e1) of one uploaded
// chunk, one wave per 64-entry slab of the SOURCE CSR, lane = entry.  Source row u is local row
// perm[u] (the single plan's hub-first relabelling: order and perm are inverse), so entry e of
// row u lands at local position rp[perm[u]] + (e - srp[u]), the position the gather pass
// (k_sorted_keys) gives it: the sort that follows sees the same keys in the same places.  Each
// chunk runs as soon as its copy has landed, under the copies of the later chunks.
template <typename K>
__global__ __launch_bounds__(256) void k_scatter_keys(KeySrc k, int64_t n_src, const int64_t *__restrict__ ssrow,
                                                      int64_t sl0, int64_t sl1, int64_t nnz,
                                                      const int32_t *__restrict__ rowseg, K *__restrict__ keys,
                                                      uint16_t *__restrict__ vals) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (256 / kWave);
    const int64_t nslabs_src = (nnz + kWave - 1) / kWave;
    for (int64_t sl = sl0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave; sl < sl1; sl += nw) {
        const int64_t e = sl * kWave + lane;
        const int64_t ee = min(e, nnz - 1);
        const int64_t u = slab_row_of(k.srp, ssrow, n_src, min(sl, nslabs_src - 1), ee, lane);
        const int32_t i = k.perm[u];
        const int32_t sg = rowseg[i];
        const int64_t dst = k.rp[i] + (ee - k.srp[u]);
        const uint32_t c = (uint32_t)k.perm[k.sci[ee]];
        if (e < nnz) {
            keys[dst] = ((K)(sg & k.segmask) << k.colbits) | (K)c;
            vals[dst] = (uint16_t)(i - k.seg_row[sg]);
        }
    }
}

// sci / spk / gbase from the sorted (key, row) pairs: every entry's column into sci (the LONG
// path and the escape supergroups read it), and for the sorted blocks (segments with gseg >= 0)
// the packed entries and the base column of each 256-entry supergroup, aligned to the block's
// first entry (the kernel's rounds).
struct SegDesc {
    int64_t z0, z1;
    int32_t gseg;   // the block's first supergroup in gbase, -1 for a LONG row
    int32_t pad;
};

// A workgroup per kPackChunk entries of one segment (host-built list: no search per entry); the
// chunks start on the segment's 256-entry supergroups, so each of a thread's 16 entries lies in
// one supergroup whose base / last keys every thread of the workgroup reads alike.
constexpr int64_t kPackChunk = 4096;
struct PackChunk {
    int64_t z0;
    int32_t seg;
    int32_t pad;
};

template <typename K>
__global__ __launch_bounds__(256) void k_sorted_pack(const SegDesc *__restrict__ segs, const PackChunk *__restrict__ chunks,
                                                     int64_t nchunks, const K *__restrict__ keys,
                                                     const uint16_t *__restrict__ vals, uint32_t colmask,
                                                     int32_t *__restrict__ sci, uint32_t *__restrict__ spk,
                                                     uint32_t *__restrict__ gbase) {
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const PackChunk pc = chunks[c];
        const SegDesc sg = segs[pc.seg];
        const int64_t z1 = min(pc.z0 + kPackChunk, sg.z1);
#pragma unroll 4
        for (int64_t g0 = pc.z0; g0 < z1; g0 += 256) {
            const int64_t e = g0 + threadIdx.x;
            const bool in = e < z1;
            const uint32_t col = in ? (uint32_t)keys[e] & colmask : 0u;
            if (in) sci[e] = (int32_t)col;
            if (sg.gseg < 0 || !in) continue;
            const int64_t q = (g0 - sg.z0) >> 8;
            const uint32_t base = (uint32_t)keys[g0] & colmask;
            const uint32_t lastc = (uint32_t)keys[min(g0 + 255, sg.z1 - 1)] & colmask;
            const bool esc = lastc - base >= (1u << (32 - kRowBits));
            const uint32_t row = vals[e];
            spk[e] = esc ? row : ((col - base) << kRowBits) | row;
            if (threadIdx.x == 0) gbase[sg.gseg + q] = esc ? (base | 0x80000000u) : base;
        }
    }
}

// LDS bank spreading: inside every full 64-entry group of a sorted block, the 64 entries are
// permuted so that each of the four LDS-add wave-instructions of the X4 layout (instruction j
// adds the entries at positions 4s + j, s < 16, of the group: one per lane of the group's 16
// lanes) gets entries whose rows differ mod 16 wherever possible -- the banks of a 64-bit LDS
// address a are (a/4) mod 32, so rows r and r' collide on a 16-lane group iff r = r' mod 16.
// The entries are ranked by (row mod 16, bit 4 of the row, position) and entry k of that order
// goes to instruction k mod 4, slot k / 4: a residue held by m <= 4 entries lands in m
// different instructions.  The group keeps its column set, so its gathers touch the same lines.
// One wave per group.
// Only the wide part of the block (from its narrow prefix nsplit[block] supergroups on).
__global__ __launch_bounds__(256) void k_sorted_laneperm(const RowBlock *__restrict__ blocks, const uint32_t *__restrict__ nsplit,
                                                         uint32_t *spk, int32_t *sci) {
    const RowBlock b = blocks[blockIdx.y];
    const int64_t z0 = b.nz_begin + 256 * (int64_t)nsplit[blockIdx.y], ngroups = (b.nz_end - z0) >> 6;   // full groups only
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    const int64_t waves = (int64_t)gridDim.x * blockDim.x / kWave;
    for (int64_t g = wave; g < ngroups; g += waves) {
        const int64_t e = z0 + (g << 6) + lane;
        const uint32_t p = spk[e];
        const int32_t c = sci[e];
        const uint32_t row = p & ((1u << kRowBits) - 1);
        const uint32_t key = ((row & 15u) << 1) | ((row >> 4) & 1u);
        // rank = entries with a smaller key + entries with my key at a lower lane
        uint32_t rank = 0;
        for (uint32_t k = 0; k < 32; k++) {
            const uint64_t m = __ballot(key == k);
            if (k < key) rank += (uint32_t)__popcll(m);
            else if (k == key) rank += (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        }
        const int64_t dst = z0 + (g << 6) + 4 * (rank >> 2) + (rank & 3);
        spk[dst] = p;
        sci[dst] = c;
    }
}

// ---- narrow codes (gather_narrow).  A sorted block's entries are column-sorted; its prefix of
// supergroups where 2-byte codes (fillers included) take fewer bytes than the 4-byte entries is
// recoded, chosen per block to minimise the index bytes: supergroup g costs 2 (n_g + D_g) bytes
// narrow against 4 n_g wide, D_g = the fillers its column steps need (a step s > 3 takes
// ceil(s / 3) - 1).  SYN-8_5: 95 % of the entries, 2.5 % fillers, index bytes 2.51 -> 1.35 GB.

// fillers of the step from the previous entry of the block to entry e (0 for its first)
__device__ __forceinline__ uint32_t narrow_fillers(const int32_t *sci, int64_t z0, int64_t e, uint32_t *step) {
    const uint32_t c = (uint32_t)sci[e];
    const uint32_t s0 = e > z0 ? c - (uint32_t)sci[e - 1] : 0u;
    *step = s0;
    return s0 > 3 ? (s0 + 2) / 3 - 1 : 0u;
}

__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(v), kWave - 1);
}

// D_g of every 256-entry supergroup of every sorted block (grid.y = block), one wave each.
__global__ __launch_bounds__(256) void k_narrow_cost(const RowBlock *__restrict__ blocks, const int32_t *__restrict__ sci,
                                                     uint32_t *__restrict__ fill) {
    const RowBlock b = blocks[blockIdx.y];
    const int64_t z0 = b.nz_begin, N = b.nz_end - z0, ng = (N + 255) >> 8;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t waves = (int64_t)gridDim.x * blockDim.x / kWave;
    for (int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; g < ng; g += waves) {
        uint32_t d = 0, st;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e = (g << 8) + 4 * lane + j;
            if (e < N) d += narrow_fillers(sci, z0, z0 + e, &st);
        }
        d = wave_total(d);
        if (lane == 0) fill[b.seg + g] = d;
    }
}

// Per block (one 1024-thread workgroup): the narrow prefix P (supergroups) maximising
// sum_{g<P} (n_g - D_g) (0 when `enable` is off), the code offset of every supergroup inside
// the block's narrow run (exclusive prefix of n_g + D_g), and the block's code count.
__global__ __launch_bounds__(1024) void k_narrow_split(const RowBlock *__restrict__ blocks, const uint32_t *__restrict__ fill,
                                                       int enable, int64_t min_entries, uint32_t *__restrict__ nsplit,
                                                       uint32_t *__restrict__ ncode,
                                                       uint32_t *__restrict__ noff) {
    __shared__ int64_t sben[1024], scod[1024];
    __shared__ int64_t bestv[1024];
    __shared__ int32_t besti[1024];
    const RowBlock b = blocks[blockIdx.x];
    const int64_t N = b.nz_end - b.nz_begin, ng = (N + 255) >> 8;
    const int t = threadIdx.x;
    const int64_t per = (ng + 1023) / 1024, g0 = min(ng, t * per), g1 = min(ng, g0 + per);
    auto cnt = [&](int64_t g) { return min<int64_t>(256, N - (g << 8)); };
    int64_t ben = 0, cod = 0;
    for (int64_t g = g0; g < g1; g++) {
        ben += cnt(g) - (int64_t)fill[b.seg + g];
        cod += cnt(g) + (int64_t)fill[b.seg + g];
    }
    sben[t] = ben;
    scod[t] = cod;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {   // inclusive scans (Hillis-Steele)
        const int64_t a1 = t >= o ? sben[t - o] : 0, a2 = t >= o ? scod[t - o] : 0;
        __syncthreads();
        sben[t] += a1;
        scod[t] += a2;
        __syncthreads();
    }
    int64_t pb = sben[t] - ben, pc = scod[t] - cod;
    int64_t bv = 0;
    int32_t bi = 0;   // P = 0 is always allowed
    for (int64_t g = g0; g < g1; g++) {
        noff[b.seg + g] = (uint32_t)pc;
        pb += cnt(g) - (int64_t)fill[b.seg + g];
        pc += cnt(g) + (int64_t)fill[b.seg + g];
        if (pb > bv) {
            bv = pb;
            bi = (int32_t)(g + 1);
        }
    }
    bestv[t] = bv;
    besti[t] = bi;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {   // max value, then the smallest prefix
        if (t < o) {
            const int64_t v2 = bestv[t + o];
            const int32_t i2 = besti[t + o];
            if (v2 > bestv[t] || (v2 == bestv[t] && i2 < besti[t])) {
                bestv[t] = v2;
                besti[t] = i2;
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        const int32_t P = (enable && N >= min_entries) ? besti[0] : 0;
        nsplit[blockIdx.x] = (uint32_t)P;
        // codes of the prefix: the offset of supergroup P, or all of them
        ncode[blockIdx.x] = P == 0 ? 0u : (uint32_t)(P < ng ? noff[b.seg + P] : (uint32_t)scod[1023]);
    }
}

// Padding codes everywhere (step 0, a junk row by lane) and the null supergroup's base.
__global__ void k_narrow_fill(uint16_t *__restrict__ npk, uint64_t ncodes, uint32_t *__restrict__ nbase, uint32_t null_sg,
                              uint32_t zero_col) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < ncodes; p += (uint64_t)gridDim.x * blockDim.x)
        npk[p] = (uint16_t)(kJunkRow + ((p >> 3) & (kWave - 1)));
    if (blockIdx.x == 0 && threadIdx.x == 0) nbase[null_sg] = zero_col;
}

// The codes of the narrow prefix: one wave per 256-entry supergroup g < P of each block; lane
// l emits entries 4l .. 4l+3, each preceded by its fillers, at the block's run + noff[g] + the
// lane's exclusive scan of code counts.  Whoever emits the last code of a 512-code supergroup
// stores the next one's base (the column reached); the block's first base is its first column.
__global__ __launch_bounds__(256) void k_narrow_emit(const RowBlock *__restrict__ blocks, const int32_t *__restrict__ sci,
                                                     const uint32_t *__restrict__ spk, const uint32_t *__restrict__ nsplit,
                                                     const uint32_t *__restrict__ ncode, const uint32_t *__restrict__ noff,
                                                     const int64_t *__restrict__ nbeg, uint16_t *__restrict__ npk,
                                                     uint32_t *__restrict__ nbase) {
    const RowBlock b = blocks[blockIdx.y];
    const int64_t z0 = b.nz_begin, N = b.nz_end - z0, P = nsplit[blockIdx.y];
    const int64_t nb = nbeg[blockIdx.y], C = ncode[blockIdx.y];
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t waves = (int64_t)gridDim.x * blockDim.x / kWave;
    if (P > 0 && blockIdx.x == 0 && threadIdx.x == 0) nbase[nb / kNSg] = (uint32_t)sci[z0];
    for (int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; g < P; g += waves) {
        uint32_t fl[4], st[4], n = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e = (g << 8) + 4 * lane + j;
            fl[j] = e < N ? narrow_fillers(sci, z0, z0 + e, &st[j]) : 0u;
            n += e < N ? fl[j] + 1 : 0u;
        }
        int64_t pos = nb + noff[b.seg + g] + (wave_scan_incl(n) - n);   // absolute code index
        // stored lane-major inside the 512-code supergroup: code e of it at (e mod 64) * 8 + e / 64
        auto put = [&](uint32_t step, uint32_t row, uint32_t col_after) {
            npk[(pos & ~(int64_t)(kNSg - 1)) + (pos & (kWave - 1)) * 8 + ((pos >> 6) & 7)] = (uint16_t)((step << kRowBits) | row);
            const int64_t rel = pos - nb + 1;   // codes of the block up to and including this one
            if ((rel & (kNSg - 1)) == 0 && rel < C) nbase[(pos + 1) / kNSg] = col_after;
            pos++;
        };
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e = (g << 8) + 4 * lane + j;
            if (e >= N) continue;
            const uint32_t c = (uint32_t)sci[z0 + e];
            uint32_t at = c - st[j];
            for (uint32_t f = 0; f < fl[j]; f++) {
                at += 3;
                put(3u, (uint32_t)(kJunkRow + (pos & (kWave - 1))), at);   // the lane's own junk row
            }
            put(c - at, spk[z0 + e] & ((1u << kRowBits) - 1), c);
        }
    }
}

// Paced sweep plan: per unit, the first narrow round and the first wide round whose column is
// in window w (window 0: columns below h; window w >= 1 from h + (w - 1) 2^wshift), w = 0..nw,
// by binary searches over the unit's rounds (their first columns ascend).  One workgroup per unit.
__global__ __launch_bounds__(64) void k_pace_rounds(const SortedUnit *__restrict__ units, uint32_t nunits,
                                                    const uint32_t *__restrict__ nbase, const int32_t *__restrict__ sci,
                                                    uint32_t nw, uint32_t h, uint32_t wshift, int32_t *__restrict__ out) {
    const uint32_t ui = blockIdx.x;
    if (ui >= nunits) return;
    const SortedUnit u = units[ui];
    int32_t *o = out + (size_t)ui * 2 * (nw + 1);
    constexpr int W = kBS / kWave;
    const int32_t nrounds = (u.nsg + W - 1) / W;
    const int32_t nrn = u.unit >= nrounds ? 0 : (nrounds - u.unit + u.nunits - 1) / u.nunits;
    const int32_t nrw = u.lo < u.hi ? (int32_t)((u.hi - u.lo + u.step - 1) / u.step) : 0;
    const uint32_t sg0 = (uint32_t)(u.nbeg / kNSg);
    for (uint32_t w = threadIdx.x; w <= nw; w += blockDim.x) {
        int32_t rn = 0, rw = 0;
        if (w == nw) {
            rn = nrn;
            rw = nrw;
        } else if (w > 0) {
            const uint64_t start = (uint64_t)h + ((uint64_t)(w - 1) << wshift);
            int32_t L = 0, H = nrn;
            while (L < H) {
                const int32_t mid = (L + H) >> 1;
                if ((uint64_t)nbase[sg0 + (uint32_t)((u.unit + mid * u.nunits) * W)] >= start) H = mid;
                else L = mid + 1;
            }
            rn = L;
            L = 0;
            H = nrw;
            while (L < H) {
                const int32_t mid = (L + H) >> 1;
                if ((uint64_t)(uint32_t)sci[u.lo + (int64_t)mid * u.step] >= start) H = mid;
                else L = mid + 1;
            }
            rw = L;
        }
        o[w] = rn;
        o[nw + 1 + w] = rw;
    }
}

int env_int(const char *name, int dflt, int lo, int hi) {
    if (const char *e = std::getenv(name)) {
        const int v = std::atoi(e);
        if (v >= lo && v <= hi) return v;
    }
    return dflt;
}

// Simulated duration (us) of one k_pr_pull_units launch: the units of every sorted block
// (entries ents[i], rows rws[i]) cut at unit size t, and the LONG segments (lsegs), dealt
// largest first to one workgroup slot per CU, each slot taking the next unit when it frees
// (list scheduling; the grid is issued in that order).  Per-unit cost from the per-workgroup
// timestamps (tools/unit_times.py on SYN-7_5): ~2,900 entries/us of gathers, ~2 ns per row
// (zeroing, epilogue, slab store), ~1.5 us fixed, and the last arriver's slab reads.  It
// picks the unit size on large graphs, so that the units of the large blocks land in as few
// waves as the CUs allow.
struct UnitCost {
    // entries per us, us per row, us fixed, us per row and slab (GX_PR_SIM_RATE, GX_PR_SIM_ROW_PS,
    // GX_PR_SIM_SLAB_PS override: entries / us and ps)
    double rate = 2900.0, row = 0.002, fixed = 1.5, slab = 0.0005;
    // model 1 (GX_PR_SIM_MODEL=1): a multi-unit block's units each store their slab (slab per
    // row), and only the last arriver pays the combine, one round trip (rt us, GX_PR_SIM_RT_NS)
    // per 16 Ki slab entries
    int model = 0;
    double rt = 2.0;
};

double pr_unit_makespan(const std::vector<int64_t> &ents, const std::vector<int64_t> &effs, const std::vector<int64_t> &rws,
                        const std::vector<int64_t> &lsegs, int64_t t, int cus, bool by_cost, const UnitCost &uc) {
    const double kRate = uc.rate, kRow = uc.row, kFixed = uc.fixed, kSlab = uc.slab;
    std::vector<double> cost;
    for (size_t i = 0; i < ents.size(); i++) {
        const int64_t E = ents[i];
        // units by cost, not entries: a block of mostly wide (sparse-tail) entries runs at about
        // half the hub blocks' entry rate, so it is cut into more units (pr_unit_count)
        const int64_t k = std::max<int64_t>(1, std::min((E + kRound - 1) / kRound, ((by_cost ? effs[i] : E) + t - 1) / t));
        if (uc.model == 1) {
            const double c = (double)effs[i] / (double)k / kRate + kRow * (double)rws[i] + kFixed +
                             (k > 1 ? kSlab * (double)rws[i] : 0.0);
            for (int64_t j = 0; j + 1 < k; j++) cost.push_back(c);
            cost.push_back(c + (k > 1 ? uc.rt * std::ceil((double)k * (double)rws[i] / (double)(1 << kRowBits)) : 0.0));
            continue;
        }
        const double c = (double)effs[i] / (double)k / kRate + kRow * (double)rws[i] + kFixed +
                         (k > 1 ? kSlab * (double)rws[i] * (double)k : 0.0);
        for (int64_t j = 0; j < k; j++) cost.push_back(c);
    }
    for (int64_t e : lsegs) cost.push_back((double)e / kRate + kFixed);
    std::sort(cost.begin(), cost.end(), std::greater<double>());
    std::priority_queue<double, std::vector<double>, std::greater<double>> slots;
    for (int i = 0; i < std::max(1, cus); i++) slots.push(0.0);
    double span = 0.0;
    for (double c : cost) {
        const double f = slots.top() + c;
        slots.pop();
        slots.push(f);
        span = std::max(span, f);
    }
    return span;
}

}  // namespace

// Plan: rows longer than long_nnz -> LONG segment blocks (longest first); runs of the other
// rows with entries -> blocks of <= block_nnz entries and <= sorted_rows rows, entries sorted
// by column and cut into units; the trailing rows without entries -> row-range workgroups.
int pr_plan_sorted(PrPart *p, HostView<int64_t> h_rp, HostView<int32_t> h_outdeg) {
    const int64_t rows = (int64_t)h_rp.size() - 1;
    const uint64_t nnz = (uint64_t)h_rp[rows];
    const int64_t cus = std::max(1, p->ctx->num_cus);
    // Sorted blocks of up to block_nnz entries and sorted_rows rows, each cut into units of at
    // most T entries (interleaved rounds), one workgroup each, one workgroup per CU; rows longer
    // than block_nnz / 4 take the LONG path.  block_nnz = 1 Mi with 4 Ki rows, 4 Mi once nnz / CUs
    // passes 384 Ki, 32 Mi with 16 Ki rows once it passes 2 Mi, at most 4x (16x past 2 Mi) the
    // power of two nearest nnz / CUs; T is a quarter block, or past 2 Mi entries per CU chosen by simulating
    // the launch (pr_unit_makespan).  GX_PR_BLOCK_NNZ, GX_PR_SORTED_ROWS, GX_PR_LONG_NNZ,
    // GX_PR_UNIT_NNZ override.  Measured (tools/pr_units_sweep.sh, us per launch): SYN-7_5 100;
    // graph500-22 267; SYN-8_5 1064-1070 (round 2, before X4).  Larger blocks cut the x line
    // requests (tools/pr_line_model.py) but give the last arriver more slabs per row.
    const double per_cu = std::max(1.0, (double)nnz / (double)cus);
    // GX_PR_HUGE=1: the huge-graph plan whatever the size (a rank of a block partition,
    // pr_partition.block_relabel, cuts its rows as the whole graph's plan does)
    const bool huge = per_cu > (double)(2 << 20) || env_int("GX_PR_HUGE", 0, 0, 1) == 1 || p->force_huge;
    // a rank of a block partition (pr_partition.block_relabel: the whole graph's 32 Mi-entry
    // blocks dealt whole; bench.py sets GX_PR_HUGE=1 for it): the whole graph's block cut, and
    // the unit cost model fitted to its pieces (below)
    const bool piece = huge && p->nranks > 1;
    const int rmax = kMaxBlockRows;   // rows per block (LDS accumulators: 16 Ki rows = 128 KiB, the top 64 junk)
    p->sorted_rows = env_int("GX_PR_SORTED_ROWS", huge ? rmax : 4096, 64, rmax);
    // ... and at most 4x the power of two nearest nnz / CUs, so that a small partition (one rank
    // of eight) keeps about 4 units per block: a 1/8 piece of SYN-7_5 with 1 Mi blocks cut into
    // 32 units each ran 50 us per launch against 34 with 128 Ki blocks
    int64_t pow2 = 1 << 14;
    while (pow2 < (1 << 24) && (double)(2 * pow2) <= per_cu * 1.41421356) pow2 *= 2;
    // huge graphs: 32 Mi-entry blocks since the work queue (SYN-8_5, us per launch: 8 Mi 714,
    // 16 Mi 690, 32 Mi 685, 64 Mi 700, 128 Mi 702; profiles/r04_pr_block_sweep_queue.txt):
    // fewer blocks re-read x, and the queue keeps the larger units balanced
    const int64_t bdef = piece ? kPlanBlockNnz
                       : huge ? std::min<int64_t>(32 << 20, 16 * pow2)
                              : std::min<int64_t>(per_cu > 384.0 * 1024 ? 4 << 20 : 1 << 20, 4 * pow2);
    const int64_t B = env_int("GX_PR_BLOCK_NNZ", (int)bdef, 1024, 1 << 30);
    p->long_nnz = env_int("GX_PR_LONG_NNZ", (int)std::max<int64_t>(B / 4, kRound), 1024, 1 << 30);
    p->sorted_nnz = (int)B;
    // Cache policy (round 3, tools/r03_cp_ab.sh, r03_ntx_ab.sh, r03_lanemajor.sh), when x is
    // larger than the 32 MiB of all eight L2s (the exchanged chunks: SYN-8_5's live rows are
    // 44.6 MB): the index stream, read once per launch, loaded non-temporally
    // (bit 0: SYN-8_5, 67 MB of x, 898 -> 871-877 us per launch), and so are the gathers of the
    // narrow supergroups from column nt_col = 64 Ki on (bit 2: 780 -> 757-760 us), so the XCD's
    // L2 keeps the hub lines.  Wide (sparse tail) gathers stay cached: non-temporal they ran
    // 965 us.  SYN-7_5 (8 MB of x) keeps plain loads everywhere: 83 -> 91 us with bit 0, 72.5 ->
    // 79.6 with bit 2.  GX_PR_CP = 0 / 1 / 5 and GX_PR_NT_COL override.
    const uint64_t xbytes = (uint64_t)p->chunk * (uint64_t)std::max(1, p->nranks) * sizeof(double);
    p->cache_policy = env_int("GX_PR_CP", xbytes >= (32ull << 20) ? 5 : 0, 0, 5);
    if (p->cache_policy != 0 && p->cache_policy != 1) p->cache_policy = 5;
    p->nt_col = (uint32_t)env_int("GX_PR_NT_COL", 65536, 0, 1 << 30);
    PlanClock clk("sorted", p->ctx->stream);
    const int64_t R = p->sorted_rows, LT = std::max<int64_t>(p->long_nnz, 1);
    std::vector<RowBlock> longb, sortb;
    std::vector<int32_t> lfirst, lnseg;
    std::vector<std::pair<int64_t, int32_t>> longrows;
    int32_t nsegs = 0;
    int64_t r = 0;
    if (p->rows_desc) {
        // lengths non-increasing: the LONG rows are a prefix, and each block's end is the row
        // limit or the last row pointer within B of its start, found by binary search (the
        // row-by-row loop below took 3.5 ms for SYN-8_5's 8.4 M rows; this cut is the same)
        while (r < rows && h_rp[r + 1] - h_rp[r] > LT) {
            longrows.push_back({h_rp[r + 1] - h_rp[r], (int32_t)r});
            r++;
        }
        while (r < rows) {
            const int64_t start = r, lim = std::min<int64_t>(rows, start + R);
            const int64_t limit = h_rp[start] + B;
            int64_t lo = start + 1, hi = lim + 1;   // first e in (start, lim] with h_rp[e] > limit
            while (lo < hi) {
                const int64_t mid = (lo + hi) / 2;
                if (h_rp[mid] > limit) hi = mid;
                else lo = mid + 1;
            }
            r = std::max<int64_t>(start + 1, lo - 1);
            sortb.push_back({h_rp[start], h_rp[r], (int32_t)start, (int32_t)r, -1, 0});
        }
    }
    while (r < rows) {
        const int64_t len = h_rp[r + 1] - h_rp[r];
        if (len > LT) {
            longrows.push_back({len, (int32_t)r});
            r++;
            continue;
        }
        const int64_t start = r;
        int64_t nz = 0;
        while (r < rows && r - start < R) {
            const int64_t l = h_rp[r + 1] - h_rp[r];
            if (l > LT || nz + l > B) break;
            nz += l;
            r++;
        }
        sortb.push_back({h_rp[start], h_rp[r], (int32_t)start, (int32_t)r, -1, 0});
    }
    int64_t maxrows = 1;   // LDS accumulators
    for (const RowBlock &b : sortb) maxrows = std::max<int64_t>(maxrows, b.row_end - b.row_begin);
    // seg of a sorted block = index of its first 256-entry supergroup in gbase
    int64_t ngroups = 0;
    for (RowBlock &b : sortb) {
        b.seg = (int32_t)ngroups;
        ngroups += (b.nz_end - b.nz_begin + 255) / 256;
    }
    std::stable_sort(longrows.begin(), longrows.end(), [](const auto &x, const auto &y) { return x.first > y.first; });
    for (const auto &lr : longrows) {
        const int32_t row = lr.second;
        const int32_t nseg = (int32_t)((lr.first + kSegNnz - 1) / kSegNnz);
        const int32_t sp = (int32_t)lfirst.size();
        lfirst.push_back(nsegs);
        lnseg.push_back(nseg);
        for (int32_t s = 0; s < nseg; s++) {
            const int64_t zb = h_rp[row] + (int64_t)s * kSegNnz;
            longb.push_back({zb, std::min(zb + kSegNnz, h_rp[row + 1]), row, row + 1, sp, s});
        }
        nsegs += nseg;
    }
    p->sorted_lds = (int)(maxrows * sizeof(double));
    std::vector<RowBlock> all(longb);
    all.insert(all.end(), sortb.begin(), sortb.end());
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
    clk.mark("blocks (host)");

    // block-sorted columns and packed entries, by one radix sort of (segment, column) keys
    GX_TRY(p->sci.alloc(std::max<uint64_t>(nnz, 1), 16));
    GX_TRY(p->spk.alloc(std::max<uint64_t>(nnz, 1), 16));
    GX_TRY(p->gbase.alloc(std::max<int64_t>(ngroups, 1), 16));
    hipStream_t s = p->ctx->stream;
    const RowBlock *d_sort = p->blocks.p + longb.size();
    std::vector<uint32_t> h_nsplit(sortb.size(), 0), h_ncode(sortb.size(), 0);   // narrow prefix per sorted block
    std::vector<int64_t> h_nbeg(sortb.size(), 0);
    p->ncodes = 0;
    p->nnarrow = 0;
    // device temporaries of the plan, released after the unit-size search (which runs on the
    // host while the narrow codes and the lane permutation are built)
    DBuf<int32_t> d_seg_row;
    DBuf<SegDesc> d_segd;
    DBuf<int64_t> srow;
    DBuf<int32_t> d_rowseg;
    DBuf<PackChunk> d_pch;
    DBuf<uint32_t> d_fill, d_noff, d_nsplit, d_ncode;
    DBuf<int64_t> d_nbeg;
    if (nnz > 0) {
        // segments in row order: the sorted blocks and the LONG rows
        std::vector<std::pair<int32_t, int32_t>> order_;   // (first row, index: block i >= 0, LONG row -1 - j)
        for (size_t i = 0; i < sortb.size(); i++) order_.push_back({sortb[i].row_begin, (int32_t)i});
        for (size_t j = 0; j < longrows.size(); j++) order_.push_back({longrows[j].second, -1 - (int32_t)j});
        std::sort(order_.begin(), order_.end());
        std::vector<int32_t> seg_row;
        std::vector<SegDesc> segd;
        for (const auto &o : order_) {
            const int32_t r0 = o.first;
            const bool blk = o.second >= 0;
            const int32_t r1 = blk ? sortb[o.second].row_end : r0 + 1;
            if (h_rp[r0] == h_rp[r1]) continue;   // no entries: no key names it (fewer segment bits)
            seg_row.push_back(r0);
            segd.push_back({h_rp[r0], h_rp[r1], blk ? sortb[o.second].seg : -1, 0});
        }
        seg_row.push_back((int32_t)rows);
        // column bits from the columns that occur: one rank's plan holds vertex ids < n (the
        // chunk's padding slots are never a column), a partition's the chunk layout
        int colbits = 1;
        const uint64_t ncols = p->nranks == 1 ? std::max<uint64_t>(p->n_global, 1) : p->chunk * (uint64_t)p->nranks;
        while ((1ull << colbits) < ncols) colbits++;
        int segbits = 1;
        while ((1ull << segbits) < segd.size()) segbits++;
        GX_TRY(d_seg_row.alloc(seg_row.size()));
        GX_TRY(d_segd.alloc(segd.size()));
        GX_HIP_TRY(hipMemcpyAsync(d_seg_row.p, seg_row.data(), seg_row.size() * 4, hipMemcpyHostToDevice, s));
        GX_HIP_TRY(hipMemcpyAsync(d_segd.p, segd.data(), segd.size() * sizeof(SegDesc), hipMemcpyHostToDevice, s));
        // 4-byte keys whenever the columns leave room: segments are contiguous entry ranges, so
        // groups of 2^(32 - colbits) of them sort independently with the segment's low bits in
        // the key (SYN-8_5: 556 segments x 2^23 columns = 33 bits, two groups of 32-bit keys
        // instead of one sort of 64-bit keys)
        const bool narrow = colbits <= 31 && !env_int("GX_PR_WIDE_KEYS", 0, 0, 1);
        // (column-only keys and one rocPRIM segmented sort of the ~556 segments ran the plan's sort
        // in 494 ms against 16 ms: it sorts a segment per workgroup; gpurun_out run m6, removed)
        const int gbits = narrow ? std::min({segbits, 32 - colbits, env_int("GX_PR_SORT_GROUP_BITS", 32, 1, 32)}) : segbits;
        const KeySrc ks{p->rp, rows, p->src_rp, p->src_ci, p->src_order, p->src_perm, d_seg_row.p,
                        (int32_t)segd.size(), colbits, (int32_t)((1ll << gbits) - 1)};
        const int64_t nslabs = (int64_t)((nnz + kWave - 1) / kWave);
        GX_TRY(srow.alloc(nslabs + 1));
        GX_TRY(slab_rows(p->rp, rows, nslabs, srow.p, s));
        GX_TRY(d_rowseg.alloc(std::max<int64_t>(rows, 1)));
        hipLaunchKernelGGL(k_row_seg, dim3((unsigned)std::min<size_t>(segd.size(), 65535)), dim3(256), 0, s, d_seg_row.p,
                           (int32_t)segd.size(), d_rowseg.p);
        GX_TRY(check_launch("k_row_seg"));
        // the pack's chunks: kPackChunk entries of one segment each, from the segment's start
        std::vector<PackChunk> pch;
        for (size_t g = 0; g < segd.size(); g++)
            for (int64_t z = segd[g].z0; z < segd[g].z1; z += kPackChunk) pch.push_back({z, (int32_t)g, 0});
        GX_TRY(d_pch.alloc(std::max<size_t>(pch.size(), 1)));
        if (!pch.empty())
            GX_HIP_TRY(hipMemcpyAsync(d_pch.p, pch.data(), pch.size() * sizeof(PackChunk), hipMemcpyHostToDevice, s));
        clk.mark("segments + slab rows");
        const unsigned kgrid = grid_for((uint64_t)((nslabs + kKeyU - 1) / kKeyU) * kWave, 256, 16384);
        const unsigned pgrid = (unsigned)std::min<size_t>(std::max<size_t>(pch.size(), 1), 1u << 20);
        const uint32_t colmask = (uint32_t)((1ull << colbits) - 1);
        // keys and values in the kept plan scratch: [k0 | k1 | v0 | v1]
        const size_t kb = narrow ? 4 : 8, align = 256;
        auto up = [&](size_t x) { return (x + align - 1) / align * align; };
        const size_t kbytes = up((size_t)nnz * kb), vbytes = up((size_t)nnz * 2);
        char *scr = nullptr;
        GX_TRY(plan_scratch(2 * kbytes + 2 * vbytes, reinterpret_cast<void **>(&scr)));
        uint16_t *v0 = reinterpret_cast<uint16_t *>(scr + 2 * kbytes), *v1 = reinterpret_cast<uint16_t *>(scr + 2 * kbytes + vbytes);
        clk.mark("key buffers");
        // the key pass: over the local rows (gather), or chunk by chunk from the source side while
        // the source columns are still being uploaded (PrPart::job, gx_pagerank_csr)
        auto key_pass = [&](auto *kk) -> int {
            using K = std::remove_pointer_t<decltype(kk)>;
            if (!p->job) {
                hipLaunchKernelGGL(k_sorted_keys<K>, dim3(kgrid), dim3(256), 0, s, ks, (int64_t)nnz, srow.p, nslabs,
                                   d_rowseg.p, kk, v0);
                return check_launch("k_sorted_keys");
            }
            const int64_t n_src = (int64_t)p->n_global;
            DBuf<int64_t> ssrow;
            GX_TRY(ssrow.alloc(nslabs + 1));
            GX_TRY(slab_rows(p->src_rp, n_src, nslabs, ssrow.p, s));
            UploadJob *job = p->job;
            for (size_t c = 0; c < job->ev.size(); c++) {
                GX_TRY(job->wait_chunk((int)c));
                GX_HIP_TRY(hipStreamWaitEvent(s, job->ev[c], 0));
                const int64_t e0 = c ? job->end[c - 1] : 0, e1 = job->end[c];
                const int64_t sl0 = e0 / kWave, sl1 = (e1 + kWave - 1) / kWave;   // chunks are 64-aligned
                hipLaunchKernelGGL(k_scatter_keys<K>, dim3(grid_for((uint64_t)(sl1 - sl0) * kWave, 256, 4096)), dim3(256),
                                   0, s, ks, n_src, ssrow.p, sl0, sl1, (int64_t)nnz, d_rowseg.p, kk, v0);
                GX_TRY(check_launch("k_scatter_keys"));
            }
            GX_TRY(job->join());
            GX_HIP_TRY(hipStreamSynchronize(s));   // ssrow is freed on return
            return GX_SUCCESS;
        };
        if (narrow) {
            uint32_t *k0 = reinterpret_cast<uint32_t *>(scr), *k1 = reinterpret_cast<uint32_t *>(scr + kbytes);
            GX_TRY(key_pass(k0));
            clk.mark("keys");
            const size_t G = (size_t)1 << gbits;
            for (size_t g0 = 0; g0 < segd.size(); g0 += G) {
                const size_t g1 = std::min(segd.size(), g0 + G) - 1;
                const int64_t z0 = segd[g0].z0, z1 = segd[g1].z1;
                GX_TRY(sort_pairs_u32_u16(k0 + z0, k1 + z0, v0 + z0, v1 + z0, (size_t)(z1 - z0), gbits + colbits, s));
            }
            clk.mark("sort");
            hipLaunchKernelGGL(k_sorted_pack<uint32_t>, dim3(pgrid), dim3(256), 0, s, d_segd.p, d_pch.p,
                               (int64_t)pch.size(), k1, v1, colmask, p->sci.p, p->spk.p, p->gbase.p);
        } else {
            uint64_t *k0 = reinterpret_cast<uint64_t *>(scr), *k1 = reinterpret_cast<uint64_t *>(scr + kbytes);
            GX_TRY(key_pass(k0));
            GX_TRY(sort_pairs_u64_u16(k0, k1, v0, v1, (size_t)nnz, segbits + colbits, s));
            hipLaunchKernelGGL(k_sorted_pack<uint64_t>, dim3(pgrid), dim3(256), 0, s, d_segd.p, d_pch.p,
                               (int64_t)pch.size(), k1, v1, colmask, p->sci.p, p->spk.p, p->gbase.p);
        }
        GX_TRY(check_launch("k_sorted_pack"));
        clk.mark("keys + sort + pack");
        // the narrow prefixes (GX_PR_NARROW=0: none) and their codes, before the lane permutation
        if (!sortb.empty()) {
            const unsigned nsb = (unsigned)sortb.size();
            GX_TRY(d_fill.alloc(std::max<int64_t>(ngroups, 1)));
            GX_TRY(d_noff.alloc(std::max<int64_t>(ngroups, 1)));
            GX_TRY(d_nsplit.alloc(nsb));
            GX_TRY(d_ncode.alloc(nsb));
            GX_TRY(d_nbeg.alloc(nsb));
            hipLaunchKernelGGL(k_narrow_cost, dim3(64, nsb), dim3(256), 0, s, d_sort, p->sci.p, d_fill.p);
            GX_TRY(check_launch("k_narrow_cost"));
            hipLaunchKernelGGL(k_narrow_split, dim3(nsb), dim3(1024), 0, s, d_sort, d_fill.p,
                               env_int("GX_PR_NARROW", 1, 0, 1), (int64_t)env_int("GX_PR_NARROW_MIN", 0, 0, 1 << 30),
                               d_nsplit.p, d_ncode.p, d_noff.p);
            GX_TRY(check_launch("k_narrow_split"));
            GX_HIP_TRY(hipMemcpyAsync(h_nsplit.data(), d_nsplit.p, nsb * 4, hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipMemcpyAsync(h_ncode.data(), d_ncode.p, nsb * 4, hipMemcpyDeviceToHost, s));
            GX_HIP_TRY(hipStreamSynchronize(s));
            uint64_t run = 0;
            for (size_t i = 0; i < sortb.size(); i++) {
                h_nbeg[i] = (int64_t)run;
                run += ((uint64_t)h_ncode[i] + kNSg - 1) / kNSg * kNSg;
                p->nnarrow += (uint64_t)std::min<int64_t>((int64_t)h_nsplit[i] * 256, sortb[i].nz_end - sortb[i].nz_begin);
            }
            p->null_sg = (uint32_t)(run / kNSg);
            p->ncodes = run + kNSg;
            GX_TRY(p->npk.alloc(p->ncodes, 16));
            GX_TRY(p->nbase.alloc(p->ncodes / kNSg));
            GX_HIP_TRY(hipMemcpyAsync(d_nbeg.p, h_nbeg.data(), nsb * 8, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_narrow_fill, dim3(grid_for(p->ncodes, 256, 16384)), dim3(256), 0, s, p->npk.p, p->ncodes,
                               p->nbase.p, p->null_sg, (uint32_t)(p->chunk - 2));
            GX_TRY(check_launch("k_narrow_fill"));
            hipLaunchKernelGGL(k_narrow_emit, dim3(64, nsb), dim3(256), 0, s, d_sort, p->sci.p, p->spk.p, d_nsplit.p,
                               d_ncode.p, d_noff.p, d_nbeg.p, p->npk.p, p->nbase.p);
            GX_TRY(check_launch("k_narrow_emit"));
            clk.mark("narrow codes");
        }
        // GX_PR_LANEPERM=0 keeps every group in column order
        if (env_int("GX_PR_LANEPERM", 1, 0, 1) && !sortb.empty()) {
            hipLaunchKernelGGL(k_sorted_laneperm, dim3(64, (unsigned)sortb.size()), dim3(256), 0, s, d_sort, d_nsplit.p,
                               p->spk.p, p->sci.p);
            GX_TRY(check_launch("k_sorted_laneperm"));
        }
    }
    p->ci = p->sci.p;   // the LONG rows read their (column-sorted) entries there
    clk.mark("laneperm");
    p->nsorted = (uint32_t)sortb.size();
    p->nlong_pad = (p->nlong_blocks + 7u) & ~7u;
    // units of the split blocks: ceil(entries / T) per sorted block (at most one per round)
    int64_t T = 0;
    p->nunits = 0;
    // the cost of a block's entries in the unit order and the launch simulation: narrow ones 1,
    // wide (sparse-tail) ones GX_PR_WIDE_COST / 4 each, since their x lines are shared by fewer
    // entries.  On huge graphs 6, with the units cut by this cost (unit_by_cost below): SYN-8_5
    // under the work queue 687 -> 630 us per launch (weight 4: 632, 8: 642; by entries with
    // weight 6: 664; profiles/r04_pr_wide_cost_ab.txt).  Round 3, before the queue: 3 (757-764
    // -> 755-756 us, tools/r03_wc_ab.sh).  1 otherwise (SYN-7_5: no change)
    const int64_t wide_cost4 = env_int("GX_PR_WIDE_COST", piece ? 11 : huge ? 24 : 4, 4, 64);
    // GX_PR_COST_CODES=1: the narrow part priced by its codes, fillers included, not by its
    // entries -- a mid-density block's column steps need up to one filler per entry, and its
    // units ran at ~2.3 K entries/us against ~4.7 K for the hub blocks (1/8 piece, unit stamps)
    // GX_PR_FILL_COST: a filler's cost in quarters of a narrow entry's.  Fitted to the unit
    // stamps of the 8 pieces of SYN-8_5 (2 330 units, rms 8.6 us on 74): 8.3 us + 177 ps per
    // narrow entry, 2.0x that per filler, 2.7x per wide entry (the piece defaults, GX_PR_SIM_*
    // below); the whole graph's units fit 1.3x per filler and 7.4x per wide entry.  Fillers
    // priced as entries ran faster than at the fitted 2x (139 against 150 us per piece launch)
    const bool cost_codes = env_int("GX_PR_COST_CODES", piece ? 1 : 0, 0, 1) == 1;
    const int64_t fill_cost4 = env_int("GX_PR_FILL_COST", 4, 0, 64);
    auto eff_entries = [&](int64_t i) -> int64_t {
        const int64_t E = sortb[i].nz_end - sortb[i].nz_begin;
        const int64_t En = std::min<int64_t>(E, 256 * (int64_t)h_nsplit[i]);
        const int64_t fill = cost_codes ? std::max<int64_t>(0, (int64_t)h_ncode[i] - En) : 0;
        return En + fill * fill_cost4 / 4 + (E - En) * wide_cost4 / 4;
    };
    // huge graphs: units per block by weighted entries (GX_PR_UNIT_BY_COST=0: by entries), so a
    // block of mostly wide entries, ~half the hub blocks' entry rate, is cut into more units
    const bool unit_by_cost = env_int("GX_PR_UNIT_BY_COST", huge ? 1 : 0, 0, 1) == 1;
    // GX_PR_COMBINE=1: the multi-unit blocks combined by k_pr_combine (stripes), not by their
    // last arriving unit
    p->comb_kernel = env_int("GX_PR_COMBINE", piece ? 1 : 0, 0, 1) == 1;
    std::vector<CombStripe> stripes;
    std::vector<char> multi(longb.size() + sortb.size(), 0);
    if (sortb.empty()) GX_HIP_TRY(hipStreamSynchronize(s));   // the temporaries above
    if (!sortb.empty()) {
        if (std::getenv("GX_PR_UNIT_NNZ")) {
            T = env_int("GX_PR_UNIT_NNZ", 65536, 1024, 1 << 30);
        } else if (!huge && !env_int("GX_PR_UNIT_SIM", 0, 0, 1)) {
            // a quarter block: measured best on SYN-7_5 (256 Ki of 1 Mi: 100 us per launch;
            // 232 Ki: 130) and on its 1/8 partition (32 Ki of 128 Ki: 33.5 us; 24 Ki: 38.8;
            // 64 Ki: 47.7; tools/pr_piece_sweep.sh)
            T = std::max<int64_t>(kRound, (B / 4 + kRound - 1) / kRound * kRound);
        } else {
            // the unit size whose simulated launch is shortest, over multiples of a round
            // (sampled coarsely past 256 rounds: the curve is flat there)
            std::vector<int64_t> ents, effs, rws, lsegs;
            for (const RowBlock &b : sortb) {
                ents.push_back(b.nz_end - b.nz_begin);
                effs.push_back(eff_entries(&b - sortb.data()));
                rws.push_back(b.row_end - b.row_begin);
            }
            for (const RowBlock &b : longb) lsegs.push_back(b.nz_end - b.nz_begin);
            double best = 0.0;
            const int64_t emax = *std::max_element(ents.begin(), ents.end());
            // candidates: every round up to 64 rounds, then 4 % apart (the makespan curve is
            // flat there; every round up to emax cost ~16 ms of host time on SYN-8_5), simulated
            // on up to 8 host threads (13 ms on one thread for SYN-8_5), then scanned in order
            std::vector<int64_t> cand;
            for (int64_t t = kRound; t <= std::max<int64_t>(kRound, emax);
                 t = t < 64 * kRound ? t + kRound : (t + t / 25 + kRound - 1) / kRound * kRound)
                cand.push_back(t);
            std::vector<double> span(cand.size());
            UnitCost uc;
            if (piece) {   // the fit above; the combine kernel leaves the units only their slab stores
                uc.rate = 5650.0;
                uc.row = 0.0;
                uc.fixed = 8.3;
                uc.slab = 0.0002;
                uc.model = 1;
                uc.rt = p->comb_kernel ? 0.0 : 2.0;
            }
            uc.rate = (double)env_int("GX_PR_SIM_RATE", (int)uc.rate, 100, 1 << 20);
            uc.row = 1e-6 * (double)env_int("GX_PR_SIM_ROW_PS", (int)(uc.row * 1e6), 0, 1 << 20);
            uc.slab = 1e-6 * (double)env_int("GX_PR_SIM_SLAB_PS", (int)(uc.slab * 1e6), 0, 1 << 20);
            uc.model = env_int("GX_PR_SIM_MODEL", uc.model, 0, 1);
            uc.rt = 1e-3 * (double)env_int("GX_PR_SIM_RT_NS", (int)(uc.rt * 1e3), 0, 1 << 20);
            uc.fixed = 1e-3 * (double)env_int("GX_PR_SIM_FIXED_NS", (int)(uc.fixed * 1e3), 0, 1 << 20);
            const int nth = (int)std::max<size_t>(1, std::min<size_t>({8, cand.size(),
                                                                       (size_t)std::max(1u, std::thread::hardware_concurrency())}));
            std::vector<std::thread> th;
            for (int w = 0; w < nth; w++)
                th.emplace_back([&, w]() {
                    for (size_t i = (size_t)w; i < cand.size(); i += (size_t)nth)
                        span[i] = pr_unit_makespan(ents, effs, rws, lsegs, cand[i], (int)cus, unit_by_cost, uc);
                });
            for (auto &x : th) x.join();
            for (size_t i = 0; i < cand.size(); i++)
                if (T == 0 || span[i] < best * 0.999) {
                    best = span[i];
                    T = cand[i];
                }
            if (env_int("GX_PR_VERBOSE", 0, 0, 3))
                std::fprintf(stderr, "[gx_pr] unit size %lld: simulated launch %.1f us\n", (long long)T, best);
            if (env_int("GX_PR_VERBOSE", 0, 0, 3) >= 2) {
                // the blocks whose units cost most at the chosen size
                std::vector<std::pair<double, size_t>> top;
                for (size_t i = 0; i < ents.size(); i++) {
                    const int64_t k = std::max<int64_t>(1, std::min((ents[i] + kRound - 1) / kRound, ((unit_by_cost ? effs[i] : ents[i]) + T - 1) / T));
                    top.push_back({pr_unit_makespan({ents[i]}, {effs[i]}, {rws[i]}, {}, T, 1 << 14, unit_by_cost, uc), i});
                    (void)k;
                }
                std::sort(top.begin(), top.end(), std::greater<>());
                for (size_t q = 0; q < std::min<size_t>(8, top.size()); q++) {
                    const size_t i = top[q].second;
                    std::fprintf(stderr, "[gx_pr]   block %zu: entries %lld eff %lld rows %lld -> longest unit %.1f us\n", i,
                                 (long long)ents[i], (long long)effs[i], (long long)rws[i], top[q].first);
                }
            }
        }
        GX_HIP_TRY(hipStreamSynchronize(s));   // narrow codes + lane permutation done: temporaries may go
        clk.mark("unit size");
        std::vector<SortedUnit> units;
        int64_t slab = 0;
        int32_t parts = 0;
        for (size_t i = 0; i < sortb.size(); i++) {
            const RowBlock &b = sortb[i];
            const int64_t E = b.nz_end - b.nz_begin;
            const int64_t rounds = (E + kRound - 1) / kRound;
            // units per block: by weighted entries (eff_entries; = E unless the plan weights wide
            // entries, GX_PR_WIDE_COST), as the simulation that picked T counts them
            const int64_t Ek = unit_by_cost ? eff_entries((int64_t)i) : E;
            const int32_t k = (int32_t)std::max<int64_t>(1, std::min<int64_t>(rounds, (Ek + T - 1) / T));
            const int64_t rows_b = b.row_end - b.row_begin;
            for (int32_t j = 0; j < k; j++) {
                SortedUnit u;
                u.lo = b.nz_begin + 256 * (int64_t)h_nsplit[i] + (int64_t)kRound * j;   // the wide part
                u.hi = b.nz_end;
                u.step = (int64_t)kRound * k;
                u.slab = k > 1 ? slab : 0;
                u.nbeg = h_nbeg[i];
                u.nsg = (int32_t)(((int64_t)h_ncode[i] + kNSg - 1) / kNSg);
                u.seg = b.seg;
                u.z0 = b.nz_begin;
                u.z1 = b.nz_end;
                u.r0 = b.row_begin;
                u.r1 = b.row_end;
                u.blk = (int32_t)(longb.size() + i);
                u.part = k > 1 ? parts : -1;
                u.unit = j;
                u.nunits = k;
                units.push_back(u);
            }
            if (env_int("GX_PR_VERBOSE", 0, 0, 3) == 3)
                std::fprintf(stderr, "[gx_pr blk] %zu E %lld En %lld codes %u eff %lld k %d rows %lld\n", i, (long long)E,
                             (long long)std::min<int64_t>(E, 256 * (int64_t)h_nsplit[i]), h_ncode[i],
                             (long long)eff_entries((int64_t)i), k, (long long)rows_b);
            if (k > 1) {
                if (p->comb_kernel)
                    for (int64_t s0 = 0; s0 < rows_b; s0 += kCombBS)
                        stripes.push_back({slab, b.row_begin, (int32_t)rows_b, (int32_t)s0,
                                           (int32_t)std::min<int64_t>(rows_b, s0 + kCombBS), k, -1});
                multi[longb.size() + i] = 1;
                slab += (int64_t)k * rows_b;
                parts++;
            }
        }
        // Largest units first: the launch lasts as long as the unit that finishes last, so the
        // big units start in the first wave and the small ones fill the gaps at the end.  Cost ~
        // entries + 4 per row (zeroing, epilogue).  Ties keep block order, so a block's units
        // stay adjacent.
        const int64_t rowc = env_int("GX_PR_ROW_COST", 4, 0, 1024);
        auto cost = [&](const SortedUnit &u) {
            const RowBlock &b = sortb[u.blk - longb.size()];
            const int64_t E = b.nz_end - b.nz_begin, R = b.row_end - b.row_begin;
            (void)E;
            return (eff_entries(u.blk - (int32_t)longb.size()) + u.nunits - 1) / u.nunits + rowc * R;
        };
        std::stable_sort(units.begin(), units.end(),
                         [&](const SortedUnit &x, const SortedUnit &y) { return cost(x) > cost(y); });
        // (Smallest first, or largest and smallest alternating, ran 88 and 120 us against 72 on
        // SYN-7_5 and 1133 against 753 on SYN-8_5: a block's interleaved units must run
        // together, tools/r03_order_ab.sh.)
        // (Co-scheduling similar units on one XCD -- slices of 32 dealt to 8 queues, grid slot
        // 8 i + q -- cut the fabric reads of SYN-8_5 by 9 % and still ran slower: 955 against
        // 925 us per launch, SYN-7_5 100 against 84; round 3)
        p->nunits = (uint32_t)units.size();
        if (env_int("GX_PR_VERBOSE", 0, 0, 3))
            std::fprintf(stderr, "[gx_pr] plan: rows %lld nnz %llu unit_nnz %lld block_nnz %d "
                         "long_nnz %d: %zu sorted blocks, %u LONG blocks (%u rows), %u units, %d multi-unit blocks, "
                         "slab %lld doubles; narrow %llu entries in %llu codes\n",
                         (long long)rows, (unsigned long long)nnz, (long long)T,
                         p->sorted_nnz, p->long_nnz, sortb.size(), p->nlong_blocks, p->nlong, p->nunits, parts,
                         (long long)slab, (unsigned long long)p->nnarrow, (unsigned long long)p->ncodes);
        GX_TRY(p->units.alloc(units.size()));
        GX_HIP_TRY(hipMemcpy(p->units.p, units.data(), units.size() * sizeof(SortedUnit), hipMemcpyHostToDevice));
        GX_TRY(p->uslab.alloc(std::max<int64_t>(slab, 1)));
        GX_TRY(p->uticket.alloc(std::max<int32_t>(parts, 1)));
        GX_HIP_TRY(hipMemset(p->uticket.p, 0, p->uticket.n * 4));
    }
    p->unit_nnz = T;
    // work queue: on (1), off (0), or (default) when the launch has at least two items per CU
    // (SYN-8_5, 887 items: 755 -> 716 us per launch; SYN-7_5 ran 3 % slower from a queue)
    p->queue_on = env_int("GX_PR_QUEUE", -1, -1, 1);
    GX_TRY(p->queue.alloc(2));
    GX_HIP_TRY(hipMemset(p->queue.p, 0, 2 * sizeof(uint32_t)));
    // paced sweep (GX_PR_PACE=1; GX_PR_PACE_H first boundary column, GX_PR_PACE_W log2 window
    // columns, GX_PR_PACE_D windows of lead, GX_PR_PACE_POLLS the bound on a wait)
    p->pace = env_int("GX_PR_PACE", 0, 0, 1);
    if (p->pace && p->nunits) {
        const uint64_t ncols = p->nranks == 1 ? std::max<uint64_t>(p->n_global, 1) : p->chunk * (uint64_t)p->nranks;
        p->pace_h = (uint32_t)env_int("GX_PR_PACE_H", 524288, 0, 1 << 30);
        p->pace_wshift = (uint32_t)env_int("GX_PR_PACE_W", 18, 10, 30);
        p->pace_d = (uint32_t)env_int("GX_PR_PACE_D", 1, 0, 1 << 14);
        p->pace_polls = (uint32_t)env_int("GX_PR_PACE_POLLS", 64, 0, 1 << 20);
        const uint64_t wcols = 1ull << p->pace_wshift;
        p->pace_nw = 1 + (uint32_t)(ncols > p->pace_h ? (ncols - p->pace_h + wcols - 1) / wcols : 0);
        if (p->pace_nw > 65000) p->pace_nw = 65000;
        GX_TRY(p->pace_rounds.alloc((size_t)p->nunits * 2 * (p->pace_nw + 1)));
        GX_TRY(p->pace_prog.alloc(8 * 256));
        GX_HIP_TRY(hipMemsetAsync(p->pace_prog.p, 0, 8 * 256 * sizeof(uint32_t), p->ctx->stream));
        hipLaunchKernelGGL(k_pace_rounds, dim3(p->nunits), dim3(64), 0, p->ctx->stream, p->units.p, p->nunits,
                           p->nbase.p ? p->nbase.p : nullptr, p->sci.p, p->pace_nw, p->pace_h, p->pace_wshift,
                           p->pace_rounds.p);
        GX_TRY(check_launch("k_pace_rounds"));
        GX_HIP_TRY(hipStreamSynchronize(p->ctx->stream));
    }
    clk.mark("units");
    // fused dangling sum: every dangling row in a sorted block (none in a LONG block), one slot
    // per block holding dangling rows
    {
        std::vector<int32_t> slot(all.size(), -1);
        bool long_dangling = false;
        for (const RowBlock &b : longb) long_dangling |= h_outdeg[b.row_begin] == 0;
        uint32_t nd = 0;
        auto dangling_in = [&](int64_t r0, int64_t r1) {
            if (p->d_range)   // the dangling rows are [d0, d0 + nd)
                return p->nd > 0 && r0 < p->d0 + (int64_t)p->nd && r1 > p->d0;
            for (int64_t r2 = r0; r2 < r1; r2++)
                if (h_outdeg[r2] == 0) return true;
            return false;
        };
        for (size_t i = longb.size(); i < all.size(); i++) {
            if (p->comb_kernel && multi[i]) continue;   // its stripes publish instead
            if (dangling_in(all[i].row_begin, all[i].row_end)) slot[i] = (int32_t)nd++;
        }
        for (CombStripe &c : stripes)
            if (dangling_in((int64_t)c.r0 + c.s0, (int64_t)c.r0 + c.s1)) c.dslot = (int32_t)nd++;
        p->fused_dangling = p->nd > 0 && nd > 0 && !long_dangling;
        p->ndblocks = nd;
        if (p->fused_dangling) {
            GX_TRY(p->dslot.alloc(std::max<size_t>(all.size(), 1)));
            GX_TRY(p->fdpart.alloc(nd));
            GX_TRY(p->fdticket.alloc(1));
            if (!all.empty()) GX_HIP_TRY(hipMemcpy(p->dslot.p, slot.data(), all.size() * 4, hipMemcpyHostToDevice));
            GX_HIP_TRY(hipMemset(p->fdticket.p, 0, 4));
        }
    }
    p->ncstripes = (uint32_t)stripes.size();
    if (!stripes.empty()) {
        GX_TRY(p->cstripes.alloc(stripes.size()));
        GX_HIP_TRY(hipMemcpy(p->cstripes.p, stripes.data(), stripes.size() * sizeof(CombStripe), hipMemcpyHostToDevice));
    }
    clk.mark("dangling slots");
    return GX_SUCCESS;
}

int pr_step_sorted(PrPart *p, const double *x_full, double *x_local, double *rank_out, hipStream_t s) {
    const double dn = (double)p->n_global;
    SortedArgs a;
    a.blocks = p->blocks.p;
    a.ci = p->ci;
    a.sci = p->sci.p;
    a.spk = p->spk.p;
    a.gbase = p->gbase.p;
    a.outdeg = p->outdeg;
    a.x_in = x_full;
    a.x_out = x_local;
    a.rank_out = rank_out;
    a.chunk = (int64_t)p->chunk;
    a.nranks = p->nranks;
    a.zero_slot = p->nd == 0 ? 1 : 0;
    a.zero_col = (int32_t)p->chunk - 2;
    a.teleport0 = (1.0 - p->damping) / dn;
    a.damping_over_n = p->damping / dn;
    a.damping = p->damping;
    a.long_first = p->long_first.p;
    a.long_nseg = p->long_nseg.p;
    a.long_part = p->long_part.p;
    a.long_ticket = p->long_ticket.p;
    a.nlong = p->nlong_blocks;
    a.nlong_pad = p->nlong_pad;
    a.dslot = p->fused_dangling ? p->dslot.p : nullptr;
    a.dpart = p->fdpart.p;
    a.dticket = p->fdticket.p;
    a.ndblocks = p->ndblocks;
    a.units = p->units.p;
    a.nunits = p->nunits;
    a.uslab = p->uslab.p;
    a.uticket = p->uticket.p;
    a.comb = p->ncstripes > 0 ? 1 : 0;
    a.cstripes = p->cstripes.p;
    a.xd = p->xd.p;
    a.live = (int64_t)p->live;
    a.utimes = nullptr;
    a.npk = p->npk.p;
    a.nbase = p->nbase.p;
    a.null_sg = p->null_sg;
    a.nt_col = p->nt_col;
    a.pace_rounds = p->pace_rounds.p;
    a.pace_prog = p->pace_prog.p;
    a.pace_nw = p->pace_nw;
    a.pace_d = p->pace_d;
    a.pace_polls = p->pace_polls;
    a.pace_ncus = (uint32_t)std::max(1, p->ctx->num_cus);
    a.queue = p->queue.p;
    const char *times_path = std::getenv("GX_PR_UNIT_TIMES");   // debug: not under graph capture
    const uint32_t nw = p->nlong_pad + p->nunits;
    if (times_path && nw) {
        if (!p->utimes.p) GX_TRY(p->utimes.alloc(4 * (size_t)nw));
        a.utimes = p->utimes.p;
    }
    if (nw) {
        KTimer kt(p->ctx, "pr_pull", s);   // one iteration's SpMV (+ fused dangling sum)
        // One 1024-thread workgroup per CU, 16 Ki accumulators (128 KiB of LDS) whatever the block's
        // rows: an entry outside its unit's range adds 0.0 to any row below 16 Ki (gather_units).
        // One workgroup per CU also keeps fewer concurrent sweeps of x: SYN-7_5 ran 100-104 us per
        // launch against 109-125 with two (round 2, tools/pr_units_sweep.sh).
        const size_t lds = (size_t)(1 << kRowBits) * sizeof(double);
        const bool use_queue = p->queue_on == 1 || (p->queue_on == -1 && nw >= 2u * (unsigned)std::max(1, p->ctx->num_cus));
        const unsigned nq = std::min<unsigned>(nw, (unsigned)std::max(1, p->ctx->num_cus));
        if (a.utimes) {
            // (per-item stamps; the queued debug kernel runs without the cache policy)
            if (use_queue) hipLaunchKernelGGL((k_pr_pull_units<true, 0, 0, false, true>), dim3(nq), dim3(kBS), lds, s, a);
            else hipLaunchKernelGGL((k_pr_pull_units<true>), dim3(nw), dim3(kBS), lds, s, a);
        } else {
#ifdef GX_PR_PROBES
            if (const char *pe = std::getenv("GX_PR_PROBE")) {
                switch (std::atoi(pe)) {
// the probes run under the plan's cache policy (0, or 5 for a large x)
#define GX_PROBE_CASE(k) case k: if (p->cache_policy == 5) hipLaunchKernelGGL((k_pr_pull_units<false, k, 5>), dim3(nw), dim3(kBS), lds, s, a); \
                                 else hipLaunchKernelGGL((k_pr_pull_units<false, k>), dim3(nw), dim3(kBS), lds, s, a); break;
                GX_PROBE_CASE(1) GX_PROBE_CASE(2) GX_PROBE_CASE(3) GX_PROBE_CASE(4) GX_PROBE_CASE(5) GX_PROBE_CASE(6) GX_PROBE_CASE(7)
                GX_PROBE_CASE(8) GX_PROBE_CASE(9) GX_PROBE_CASE(10) GX_PROBE_CASE(11) GX_PROBE_CASE(12)
                GX_PROBE_CASE(13) GX_PROBE_CASE(14) GX_PROBE_CASE(15) GX_PROBE_CASE(16) GX_PROBE_CASE(17) GX_PROBE_CASE(18)
#undef GX_PROBE_CASE
                default: hipLaunchKernelGGL((k_pr_pull_units<false>), dim3(nw), dim3(kBS), lds, s, a);
                }
            } else
#endif
            // (narrow gathers three rounds deep ran the same: SYN-8_5 752-753 against 753-754
            // us, SYN-7_5 72.1-73.2 against 71.5-72.4; tools/r03_depth_ab.sh)
            if (p->pace && p->nunits) {
                if (p->cache_policy == 5) hipLaunchKernelGGL((k_pr_pull_units<false, 0, 5, true>), dim3(nw), dim3(kBS), lds, s, a);
                else if (p->cache_policy == 1) hipLaunchKernelGGL((k_pr_pull_units<false, 0, 1, true>), dim3(nw), dim3(kBS), lds, s, a);
                else hipLaunchKernelGGL((k_pr_pull_units<false, 0, 0, true>), dim3(nw), dim3(kBS), lds, s, a);
            } else if (use_queue) {
                // one resident workgroup per CU (the LDS allows no second), never more than the items
                if (p->cache_policy == 5) hipLaunchKernelGGL((k_pr_pull_units<false, 0, 5, false, true>), dim3(nq), dim3(kBS), lds, s, a);
                else if (p->cache_policy == 1) hipLaunchKernelGGL((k_pr_pull_units<false, 0, 1, false, true>), dim3(nq), dim3(kBS), lds, s, a);
                else hipLaunchKernelGGL((k_pr_pull_units<false, 0, 0, false, true>), dim3(nq), dim3(kBS), lds, s, a);
            } else if (p->cache_policy == 5) hipLaunchKernelGGL((k_pr_pull_units<false, 0, 5>), dim3(nw), dim3(kBS), lds, s, a);
            else if (p->cache_policy == 1) hipLaunchKernelGGL((k_pr_pull_units<false, 0, 1>), dim3(nw), dim3(kBS), lds, s, a);
            else hipLaunchKernelGGL((k_pr_pull_units<false>), dim3(nw), dim3(kBS), lds, s, a);
        }
        // (inside the iteration's timer: the SpMV is both launches)
        if (p->ncstripes) hipLaunchKernelGGL(k_pr_combine, dim3(p->ncstripes), dim3(kCombBS), 0, s, a);
        if (a.utimes && ++p->utimes_launch == env_int("GX_PR_UNIT_TIMES_LAUNCH", 5, 1, 1 << 30)) {
            std::vector<uint64_t> t(4 * (size_t)nw);
            std::vector<SortedUnit> us(p->nunits);
            std::vector<RowBlock> bs(p->nblocks);
            GX_HIP_TRY(hipStreamSynchronize(s));
            GX_HIP_TRY(hipMemcpy(t.data(), p->utimes.p, t.size() * 8, hipMemcpyDeviceToHost));
            if (p->nunits) GX_HIP_TRY(hipMemcpy(us.data(), p->units.p, us.size() * sizeof(SortedUnit), hipMemcpyDeviceToHost));
            if (p->nblocks) GX_HIP_TRY(hipMemcpy(bs.data(), p->blocks.p, bs.size() * sizeof(RowBlock), hipMemcpyDeviceToHost));
            // a "%d" in the path numbers the plans that reach the launch (every piece its file)
            static std::atomic<int> ndump{0};
            char path[512];
            std::snprintf(path, sizeof path, times_path, ndump.fetch_add(1));
            if (FILE *f = std::fopen(path, "w")) {
                std::fprintf(f, "wg kind blk unit nunits entries rows t0 tgather t1 xcc\n");
                for (size_t w = 0; w < nw; w++) {
                    if (w >= p->nlong_blocks && w < p->nlong_pad) continue;
                    const bool lng = w < p->nlong_blocks;
                    long long ents = 0, nrows = 0;
                    int blk = -1, unit = 0, nunits = 1;
                    if (lng) {
                        ents = bs[w].nz_end - bs[w].nz_begin;
                        nrows = 1;
                        blk = (int)w;
                    } else {
                        const SortedUnit &u = us[w - p->nlong_pad];
                        for (int64_t k0 = u.lo; k0 < u.hi; k0 += u.step) ents += std::min<int64_t>(u.step / u.nunits, u.hi - k0);
                        for (int64_t r = u.unit; r * 16 < u.nsg; r += u.nunits)   // narrow codes (fillers included)
                            ents += std::min<int64_t>(16, u.nsg - r * 16) * kNSg;
                        blk = u.blk;
                        unit = u.unit;
                        nunits = u.nunits;
                        nrows = bs[u.blk].row_end - bs[u.blk].row_begin;
                    }
                    std::fprintf(f, "%zu %s %d %d %d %lld %lld %llu %llu %llu %llu\n", w,
                                 lng ? "long" : "unit", blk, unit, nunits, ents, nrows,
                                 (unsigned long long)t[4 * w], (unsigned long long)t[4 * w + 1],
                                 (unsigned long long)t[4 * w + 2], (unsigned long long)t[4 * w + 3]);
                }
                std::fclose(f);
            }
        }
    } else if (a.zero_slot) {
        GX_HIP_TRY(hipMemsetAsync(x_local + p->chunk - 1, 0, sizeof(double), s));
    }
    GX_TRY(check_launch("k_pr_pull_units"));
    return p->fused_dangling ? GX_SUCCESS : pr_dangling(p, x_local, s);
}

}  // namespace gx

GX_MODULE_WARMER(pr_sorted)
