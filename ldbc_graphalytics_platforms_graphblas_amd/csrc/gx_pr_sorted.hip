// gx_pr_sorted.hip -- PageRank pull SpMV over column-sorted row blocks (k_pr_pull_sorted).
//
// Same iteration as k_pr_pull (gx_pr.hip; Graphalytics PR, LAGr_PageRankGX pr.cpp:61):
//     r(v) = teleport + sum_{u in in(v)} x(u);   x'(v) = r(v) / (outdeg(v)/d)
// but the x gathers are issued in column order.
//
// Why: the x gathers are random 8-byte reads, and what bounds them is the number of 128-B
// line requests they generate (each distinct line a wave-instruction touches is one L1
// miss), not the HBM bytes of the matrix.  Gathering row by row, a 64-lane
// instruction covered 1.33 gathers per line on SYN-7_5 (44.7 M L2 requests per launch).
// Sorting the entries of a block of rows by column id puts equal and neighbouring columns
// into the same instruction, and each block sweeps x in increasing address order
// (17.1 M requests with 64 Ki-entry blocks).
//
// Layout (built once per plan on the device by a radix sort of (block << 32 | column)):
//   spk[e]   uint32 : (column - group base) << 14 | row of the entry within its block
//   gbase[g] uint32 : base column of 64-entry group g (one wave-instruction); bit 31 set =
//                     escape: the group spans >= 2^18 columns and reads them from sci
//   sci[e]   int32  : the block-sorted columns (escape groups, pass split, plan)
// A block keeps the CSR range [rp[row_begin], rp[row_end]) of its <= 4096 rows, so the
// per-row epilogue is unchanged, and streams 4 B per entry like the CSR column index.
// Gathered values are added into LDS row accumulators (ds_add_f64) in wave-arrival order:
// scores agree with the row-order sum to ~1e-15 relative but are not bit-reproducible run
// to run (the parity bar is 1e-12 relative, tests/test_gpu_parity.py).
//
// Two passes (one rank, columns reaching past `hot_cols`): the hub pass gathers only
// columns below hot_cols (2 MiB of x by default, 96 % of SYN-7_5's entries; that slice
// stays resident in every XCD's 4 MiB L2) and stores the row sums; the tail pass adds the
// other columns and runs the epilogue.  A block's hub entries are a prefix of its sorted
// order, so each pass streams one contiguous range per block (`split`).
//
// Rows longer than `long_nnz` keep the LONG path of k_pr_pull (a workgroup per 8192-entry
// segment of the row, segments combined by the last arriver) in the hub pass; their blocks
// come first.
#include <algorithm>
#include <functional>
#include <queue>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gx_pr.h"

namespace gx {
namespace {

constexpr int kRowBits = 14;   // packed entry: (column - group base) << kRowBits | row in block

struct SortedArgs {
    const RowBlock *blocks;
    const int64_t *split;    // per block: first sorted entry whose column is >= hot_cols
    const int32_t *ci;       // row-order columns (LONG rows)
    const int32_t *sci;      // block-sorted columns (escape groups)
    const uint32_t *spk;     // packed entries
    const uint32_t *gbase;   // per 64-entry group: base column, bit 31 = escape
    const int32_t *outdeg;
    const double *x_in;
    double *x_out;
    double *rank_out;
    double *ypart;           // hub-pass row sums (two passes)
    int64_t chunk;
    int nranks;
    int zero_slot;
    double teleport0, damping_over_n, damping;
    const int32_t *long_first;
    const int32_t *long_nseg;
    double *long_part;
    uint32_t *long_ticket;
    // XCD slices (k_pr_pull_sliced)
    const int64_t *sbound;   // per sorted block: slices + 1 entry boundaries
    int64_t rows;            // local rows (ypart holds `slices` arrays of them)
    uint32_t nlong, nlong_pad, nsorted;
    // fused dangling sum (one pass): per block slot or -1, partials, ticket
    const int32_t *dslot;
    double *dpart;
    uint32_t *dticket;
    uint32_t ndblocks;
    // split blocks (k_pr_pull_units)
    const SortedUnit *units;
    double *uslab;
    uint32_t *uticket;
    uint64_t *utimes;        // debug (GX_PR_UNIT_TIMES): per workgroup start, gather end, end, XCC
    double *xd;              // x of the rows past `live` (store_x, gx_pr.h)
    int64_t live;
};

// Returns the row's score if the row is dangling (out-degree 0), else 0.
__device__ __forceinline__ double sorted_epilogue(const SortedArgs &a, int32_t row, double s, double teleport) {
    const double r = teleport + s;
    if (a.rank_out) a.rank_out[row] = r;
    const int32_t deg = a.outdeg[row];
    store_x(a.x_out, a.xd, a.live, row, deg > 0 ? r / ((double)deg / a.damping) : r);
    return deg > 0 ? 0.0 : r;
}

// Fused dangling sum: the block's dangling scores d (one value per thread) are reduced, the
// block publishes its partial in its slot (agent scope) and takes a ticket; the last of the
// ndblocks participants adds the partials up with the whole workgroup (thread t takes slots
// t, t + BS, ...; fixed tree, so the order is fixed) into the chunk's last x slot.  One thread
// looping over agent-scope loads took ~8 us at the end of the launch.
template <int BS>
__device__ __forceinline__ void dangling_publish(const SortedArgs &a, int32_t slot, double d, double *wred,
                                                 int *last) {
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

// A long row's sum: the epilogue, or (sliced mode) slot 0 of the row's slice partials, the
// other slices zero.
__device__ __forceinline__ void long_finish(const SortedArgs &a, int32_t row, double s, double teleport, double *yout,
                                            int slices, int64_t rows) {
    if (!yout) {
        sorted_epilogue(a, row, s, teleport);
        return;
    }
    yout[row] = s;
    for (int j = 1; j < slices; j++) yout[(int64_t)j * rows + row] = 0.0;
}

// LONG: one segment of one long row (row order), a whole workgroup; segments of one row are
// combined by the last arriver (agent-scope release/acquire ticket).
template <int BS, int U>
__device__ __forceinline__ void long_segment(const SortedArgs &a, const RowBlock &b, double *wred, double teleport,
                                             double *yout, int slices, int64_t rows) {
    const int tid = threadIdx.x;
    const int64_t zb = b.nz_begin, ze = b.nz_end;
    double s0 = 0.0, s1 = 0.0;
    for (int64_t k0 = zb + tid; k0 < ze; k0 += (int64_t)U * BS) {
        int32_t c[U];
#pragma unroll
        for (int u = 0; u < U; u++) c[u] = __builtin_nontemporal_load(a.ci + min(k0 + (int64_t)u * BS, ze - 1));
        double g[U];
#pragma unroll
        for (int u = 0; u < U; u++) g[u] = a.x_in[c[u]];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (k0 + (int64_t)u * BS < ze) ((u & 1) ? s1 : s0) += g[u];
    }
    const double s = wave_sum(s0 + s1);
    if ((tid & (kWave - 1)) == 0) wred[tid / kWave] = s;
    __syncthreads();
    if (tid != 0) return;
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < BS / kWave; w++) tot += wred[w];
    const int32_t sp = b.split;
    const int32_t nseg = a.long_nseg[sp];
    if (nseg == 1) {
        long_finish(a, b.row_begin, tot, teleport, yout, slices, rows);
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
    long_finish(a, b.row_begin, all, teleport, yout, slices, rows);
}

// Adds x(column) of the sorted entries [lo, hi) of block b into the LDS row accumulators
// (the loop starts at the 64-entry group holding lo, so wave-instructions stay group-aligned).
// `step` (a multiple of U * BS) > U * BS: only every (step / (U * BS))-th round of U * BS
// entries, from the one at lo (interleaved units of a split block).
//
// X4 (the units kernel's default): four consecutive entries per lane from one 16-B load, so a
// round costs U / 4 index-load instructions per lane instead of U.  What bounds the launch is
// the CU's rate of vector memory instructions, not bytes or cache lines (timing probes,
// DESIGN.md 4): with every gather folded into 32 KiB of x, or into 1/16 of its lines, a launch
// still took 93-94 us against 101-103; without the LDS adds 98.5; with 3 of 8 gathers 79.5;
// with no gathers 70.  Wave w takes the U / 4 256-entry supergroups [R + 256 (w U/4 + v), +256)
// of round R; lane l holds entries 4l .. 4l+3 of each, all in 64-entry group l / 16 of the
// supergroup.  The four group bases are scalar loads issued with the index loads and selected
// per lane when the round is computed (a select right after the loads waited for them).
// PROBE (diagnostic builds only, -DGX_PR_PROBES; wrong results by design): 1 no LDS adds
// (register sum), 2 no gathers, 3 neither, 4 gathers folded into x[c & 4095] (L1 hits),
// 5 no gathers + conflict-free LDS adds (acc[tid]), 6 gathers + conflict-free LDS adds,
// 7 no index loads (entries synthesised from the position).
template <int BS, int U, bool PIPE, bool X4 = false, bool P2 = false, int PROBE = 0>
__device__ __forceinline__ void gather_range(const SortedArgs &a, const RowBlock &b, int64_t lo, int64_t hi,
                                             double *acc, int64_t step = (int64_t)U * BS) {
    const int tid = threadIdx.x;
    const int64_t z0 = b.nz_begin, z1 = b.nz_end;
    if (lo >= hi) return;
    const int64_t glast = (z1 - 1 - z0) >> 6;
    const int64_t start = z0 + ((lo - z0) & ~(int64_t)(kWave - 1));   // 64-entry group aligned
    const int lane = tid & (kWave - 1);
    if constexpr (X4 && P2) {
        // X4 pipelined across rounds (GX_PR_PIPE2): round k+1's gathers are issued before
        // round k's LDS adds, with the index loads two rounds ahead; buffers A/B alternate
        // (no copies of pending loads, which would wait for them)
        constexpr int V = U / 4;
        const int wave = tid >> 6;
        const int sub = lane >> 4;
        struct Rd {
            uint4 q[V];
            uint32_t gbs[V][4];
        };
        struct Gt {
            double g[U];
            uint32_t r[U];
            bool ok[U];
        };
        auto load = [&](Rd &d, int64_t R) {
#pragma unroll
            for (int v = 0; v < V; v++) {
                const int64_t sg = R + (int64_t)(wave * V + v) * 256;
                if constexpr (PROBE == 7) {
                    const uint32_t e0 = (uint32_t)(sg + 4 * lane - z0);
                    d.q[v] = make_uint4(((e0 >> 4) << kRowBits) | (e0 & 4095u), (((e0 + 1) >> 4) << kRowBits) | ((e0 + 1) & 4095u),
                                        (((e0 + 2) >> 4) << kRowBits) | ((e0 + 2) & 4095u), (((e0 + 3) >> 4) << kRowBits) | ((e0 + 3) & 4095u));
                } else {
                    const gx_u32x4 q4 = *reinterpret_cast<const gx_u32x4 *>(a.spk + min(sg + 4 * lane, z1 - 1));
                    d.q[v] = make_uint4(q4.x, q4.y, q4.z, q4.w);
                }
                const int g = __builtin_amdgcn_readfirstlane((int)(b.seg + min((sg - z0) >> 6, glast)));
#pragma unroll
                for (int k = 0; k < 4; k++) d.gbs[v][k] = __builtin_amdgcn_readfirstlane(a.gbase[g + k]);
            }
        };
        auto issue = [&](const Rd &d, int64_t R, Gt &t) {
            int32_t c[U];
            uint32_t esc = 0, gb[V];
#pragma unroll
            for (int v = 0; v < V; v++) {
                gb[v] = sub == 0 ? d.gbs[v][0] : sub == 1 ? d.gbs[v][1] : sub == 2 ? d.gbs[v][2] : d.gbs[v][3];
                const uint32_t w4[4] = {d.q[v].x, d.q[v].y, d.q[v].z, d.q[v].w};
                const int64_t e4 = R + (int64_t)(wave * V + v) * 256 + 4 * lane;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int i = 4 * v + j;
                    t.ok[i] = e4 + j >= lo && e4 + j < hi;
                    t.r[i] = t.ok[i] ? (w4[j] & ((1u << kRowBits) - 1)) : 0u;
                    c[i] = t.ok[i] ? (int32_t)(gb[v] + (w4[j] >> kRowBits)) : 0;
                }
                esc |= gb[v];
            }
            if (PROBE != 7 && __builtin_amdgcn_readfirstlane(__ballot(esc & 0x80000000u) != 0)) {
#pragma unroll
                for (int v = 0; v < V; v++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int i = 4 * v + j;
                        const int64_t e = R + (int64_t)(wave * V + v) * 256 + 4 * lane + j;
                        if ((gb[v] & 0x80000000u) && t.ok[i]) c[i] = a.sci[e];
                    }
            }
#pragma unroll
            for (int i = 0; i < U; i++) {
                if constexpr (PROBE == 2 || PROBE == 3 || PROBE == 5) t.g[i] = (double)c[i];
                else if constexpr (PROBE == 4) t.g[i] = a.x_in[c[i] & 4095];
                else t.g[i] = a.x_in[c[i]];
            }
        };
        double rsum = 0.0;   // PROBE 1 / 3
        auto add = [&](const Gt &t) {
#pragma unroll
            for (int i = 0; i < U; i++) {
                if constexpr (PROBE == 1 || PROBE == 3) rsum += t.ok[i] ? t.g[i] : 0.0;
                else if constexpr (PROBE == 5 || PROBE == 6) atomicAdd(&acc[tid], t.ok[i] ? t.g[i] : 0.0);
                else atomicAdd(&acc[t.r[i]], t.ok[i] ? t.g[i] : 0.0);
            }
        };
        Rd dA, dB;
        Gt tA, tB;
        int64_t R = start;
        load(dA, R);
        load(dB, R + step);
        issue(dA, R, tA);
        load(dA, R + 2 * step);
        for (;;) {
            if (R + step >= hi) {
                add(tA);
                break;
            }
            issue(dB, R + step, tB);
            load(dB, R + 3 * step);
            add(tA);
            R += step;
            if (R + step >= hi) {
                add(tB);
                break;
            }
            issue(dA, R + step, tA);
            load(dA, R + 3 * step);
            add(tB);
            R += step;
        }
        if constexpr (PROBE == 1 || PROBE == 3) atomicAdd(&acc[tid], rsum);
        return;
    }
    if constexpr (X4) {
        static_assert(U % 4 == 0, "X4 takes four entries per load");
        constexpr int V = U / 4;
        const int wave = tid >> 6;
        const int sub = lane >> 4;
        uint4 q[V];
        uint32_t gbs[V][4];   // the 4 group bases of each supergroup (uniform)
        auto load_round = [&](int64_t R) {
#pragma unroll
            for (int v = 0; v < V; v++) {
                const int64_t sg = R + (int64_t)(wave * V + v) * 256;
                // clamped into the block; spk's allocation slack covers the 3 entries past z1 - 1
                // (dword-aligned 16-B loads)
                const gx_u32x4 q4 = *reinterpret_cast<const gx_u32x4 *>(a.spk + min(sg + 4 * lane, z1 - 1));
                q[v] = make_uint4(q4.x, q4.y, q4.z, q4.w);
                // readfirstlane is convergent, so the loads cannot sink into the select's
                // branches.  A supergroup past the block's end (the tail of the last round, or
                // the prefetch past it) reads the last group's bases; the up to 3 groups past
                // the last read the next block's bases or gbase's allocation slack, for entries
                // that ok[] masks.
                const int g = __builtin_amdgcn_readfirstlane((int)(b.seg + min((sg - z0) >> 6, glast)));
#pragma unroll
                for (int k = 0; k < 4; k++) gbs[v][k] = __builtin_amdgcn_readfirstlane(a.gbase[g + k]);
            }
        };
        int64_t R = start;
        load_round(R);
        for (; R < hi; R += step) {
            int32_t c[U];
            uint32_t r[U];
            bool ok[U];
            uint32_t esc = 0, gb[V];
#pragma unroll
            for (int v = 0; v < V; v++) {
                gb[v] = sub == 0 ? gbs[v][0] : sub == 1 ? gbs[v][1] : sub == 2 ? gbs[v][2] : gbs[v][3];
                const uint32_t w4[4] = {q[v].x, q[v].y, q[v].z, q[v].w};
                const int64_t e4 = R + (int64_t)(wave * V + v) * 256 + 4 * lane;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    // entries outside [lo, hi) (and whatever the clamped load brought) gather
                    // x(0) and add 0.0 to row 0
                    const int i = 4 * v + j;
                    ok[i] = e4 + j >= lo && e4 + j < hi;
                    r[i] = ok[i] ? (w4[j] & ((1u << kRowBits) - 1)) : 0u;
                    c[i] = ok[i] ? (int32_t)(gb[v] + (w4[j] >> kRowBits)) : 0;
                }
                esc |= gb[v];
            }
            if (__builtin_amdgcn_readfirstlane(__ballot(esc & 0x80000000u) != 0)) {   // an escape group
#pragma unroll
                for (int v = 0; v < V; v++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int i = 4 * v + j;
                        const int64_t e = R + (int64_t)(wave * V + v) * 256 + 4 * lane + j;
                        if ((gb[v] & 0x80000000u) && ok[i]) c[i] = a.sci[e];
                    }
            }
            double g[U];
#pragma unroll
            for (int i = 0; i < U; i++) g[i] = a.x_in[c[i]];
            load_round(R + step);
#pragma unroll
            for (int i = 0; i < U; i++) atomicAdd(&acc[r[i]], ok[i] ? g[i] : 0.0);
        }
        return;
    }
    uint32_t pk[U], gb[U];
    auto load_round = [&](int64_t k0) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t e = k0 + (int64_t)u * BS;
            pk[u] = __builtin_nontemporal_load(a.spk + min(e, z1 - 1));
            // the group of the wave's first lane: the same for all 64 lanes
            const int g = (int)min((e - lane - z0) >> 6, glast);
            gb[u] = a.gbase[b.seg + __builtin_amdgcn_readfirstlane(g)];
        }
    };
    int64_t k0 = start + tid;
    if (PIPE) load_round(k0);
    for (; k0 < hi; k0 += step) {
        if (!PIPE) load_round(k0);
        int32_t c[U];
        uint32_t r[U];
        uint32_t esc = 0;
#pragma unroll
        for (int u = 0; u < U; u++) {
            r[u] = pk[u] & ((1u << kRowBits) - 1);
            c[u] = (int32_t)(gb[u] + (pk[u] >> kRowBits));
            esc |= gb[u];
        }
        if (esc & 0x80000000u) {   // wave-uniform: an escape group in this round
#pragma unroll
            for (int u = 0; u < U; u++)
                if (gb[u] & 0x80000000u) c[u] = a.sci[min(k0 + (int64_t)u * BS, z1 - 1)];
        }
        double g[U];
#pragma unroll
        for (int u = 0; u < U; u++) g[u] = a.x_in[c[u]];
        if (PIPE) load_round(k0 + step);
        // entries outside [lo, hi) add 0.0 instead of branching round the add: behind a
        // branch the compiler sank the first gather below the next round's entry loads and
        // waited for all of them (vmcnt(0)) before the first add
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t e = k0 + (int64_t)u * BS;
            atomicAdd(&acc[r[u]], e >= lo && e < hi ? g[u] : 0.0);
        }
    }
}

// BS threads, U gathers in flight per lane.
//   PASS 0 : every entry, then the epilogue (one pass).
//   PASS 1 : hub pass -- entries with column < hot_cols, row sums stored to ypart; LONG rows
//            are complete here.
//   PASS 2 : tail pass over the sorted blocks only -- entries with column >= hot_cols added
//            to ypart, then the epilogue.
// PIPE: the next round's entries are loaded while this round's gathers are in flight.
template <int BS, int U, int PASS, bool PIPE>
__global__ __launch_bounds__(BS) void k_pr_pull_sorted(SortedArgs a) {
    extern __shared__ double acc[];   // one fp64 accumulator per row of the block
    __shared__ double wred[BS / kWave];
    __shared__ int last;

    const RowBlock b = a.blocks[blockIdx.x];
    const int tid = threadIdx.x;
    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    if (PASS != 2 && a.zero_slot && blockIdx.x == 0 && tid == 0) a.x_out[a.chunk - 1] = 0.0;

    if (b.split < 0) {
        // ---------------- block of rows, entries in column order ----------------
        const int nrows = b.row_end - b.row_begin;
        for (int i = tid; i < nrows; i += BS) acc[i] = PASS == 2 ? a.ypart[b.row_begin + i] : 0.0;
        __syncthreads();
        const int64_t z0 = b.nz_begin, z1 = b.nz_end;
        const int64_t lo = PASS == 2 ? a.split[blockIdx.x] : z0;
        const int64_t hi = PASS == 1 ? a.split[blockIdx.x] : z1;
        gather_range<BS, U, PIPE>(a, b, lo, hi, acc);
        __syncthreads();
        if (PASS == 1) {
            for (int i = tid; i < nrows; i += BS) a.ypart[b.row_begin + i] = acc[i];
        } else {
            double d = 0.0;
            for (int i = tid; i < nrows; i += BS) d += sorted_epilogue(a, b.row_begin + i, acc[i], teleport);
            if (PASS == 0 && a.dslot) {
                const int32_t slot = a.dslot[blockIdx.x];
                if (slot >= 0) dangling_publish<BS>(a, slot, d, wred, &last);
            }
        }
        return;
    }
    if (PASS == 2) return;   // LONG rows are complete after the hub pass

    long_segment<BS, U>(a, b, wred, teleport, nullptr, 0, 0);
}

// One-pass SpMV over split blocks.  Why split: a wave-instruction's gather costs one L2
// request per distinct x line among its 64 sorted columns, so the more entries a block sorts
// together, the more of them share a line (tools/pr_line_model.py on SYN-7_5: 12.8 M requests
// per launch with 64 Ki-entry blocks, 5.0 M with 512 Ki).  A block that large would leave too
// few workgroups for 256 CUs, so its sorted entries are cut into units of <= sorted_nnz
// entries (whole 64-entry groups), one workgroup each, all with LDS accumulators for every
// row of the block.  A multi-unit block's units store their row sums write-through (sc1) to
// their own slab, drain them (vmcnt(0)) and take a ticket; the last arriver adds the slabs in
// unit order with sc1 loads and runs the epilogue (MI355X_MICROARCH.md "Valid forms": sc1
// stores drained before the counter add, sc1 loads by the workgroup whose add came last).
// Workgroups [0, nlong) are the LONG row segments, as in k_pr_pull_sorted, padded to nlong_pad
// (a multiple of 8, so that grid slot nlong_pad + 8 i + x lands on XCD list x).
// TIMES: debug build with per-workgroup timestamps (GX_PR_UNIT_TIMES).
template <int BS, int U, bool TIMES, bool X4 = false, bool P2 = false, int PROBE = 0>
__global__ __launch_bounds__(BS, TIMES ? 1 : (BS >= 1024 ? (U >= 16 || P2 ? 4 : 8) : 1)) void k_pr_pull_units(SortedArgs a) {   // 1024: two per CU
    extern __shared__ double acc[];
    __shared__ double wred[BS / kWave];
    __shared__ int last;

    const uint32_t w = blockIdx.x;
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
    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    if (a.zero_slot && w == 0 && tid == 0) a.x_out[a.chunk - 1] = 0.0;
    if (w < a.nlong_pad) {
        if (w < a.nlong) long_segment<BS, U>(a, a.blocks[w], wred, teleport, nullptr, 0, 0);
        stamp();
        return;
    }
    const SortedUnit u = a.units[w - a.nlong_pad];
    if (u.blk < 0) return;   // padding of an XCD list
    const RowBlock b = a.blocks[u.blk];
    const int nrows = b.row_end - b.row_begin;
    for (int i = tid; i < nrows; i += BS) acc[i] = 0.0;
    __syncthreads();
    gather_range<BS, U, true, X4, P2, PROBE>(a, b, u.lo, u.hi, acc, u.step);
    __syncthreads();
    if (TIMES && tid == 0) ts[1] = __builtin_amdgcn_s_memrealtime();
    if (u.nunits > 1) {
        double *mine = a.uslab + u.slab + (int64_t)u.unit * nrows;
        for (int i = tid; i < nrows; i += BS)
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
        // other units' slabs; four rows per thread at a time keep 4 x nunits loads in flight
        // (a dependent chain of nunits loads per row left the last arriver reading for tens of
        // microseconds on 16 Ki-row blocks)
        const double *slabs = a.uslab + u.slab;
        for (int i0 = tid; i0 < nrows; i0 += 4 * BS) {
            double s[4] = {0.0, 0.0, 0.0, 0.0};
            for (int j = 0; j < u.nunits; j++) {
                const double *sl = slabs + (int64_t)j * nrows;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (i0 + q * BS < nrows) s[q] += sl[i0 + q * BS];
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (i0 + q * BS < nrows) acc[i0 + q * BS] = s[q];
        }
        // each thread reads back only the acc entries it wrote: no barrier needed
    }
    double d = 0.0;
    for (int i = tid; i < nrows; i += BS) d += sorted_epilogue(a, b.row_begin + i, acc[i], teleport);
    if (a.dslot) {
        const int32_t slot = a.dslot[u.blk];
        if (slot >= 0) dangling_publish<BS>(a, slot, d, wred, &last);
    }
    stamp();
}

// XCD slices: the columns are cut into S ranges holding equal shares of the entries, and the
// workgroups of slice j run on the XCDs with (workgroup index % 8) % S == j (blocks are dealt
// round-robin over the 8 XCDs), so an XCD's L2 only ever holds its slices' part of x instead
// of all of it.  Workgroup (block, slice) adds the block's entries of that column range into
// LDS row sums and stores them to ypart[slice][row]; k_pr_sliced_epilogue adds the S partial
// sums of every row in slice order and runs the epilogue.  LONG rows (the first nlong
// workgroups, padded to a multiple of 8) write their sum to slice 0 and zeros elsewhere.
template <int BS, int U, int S, bool PIPE>
__global__ __launch_bounds__(BS) void k_pr_pull_sliced(SortedArgs a) {
    extern __shared__ double acc[];
    __shared__ double wred[BS / kWave];
    const uint32_t w = blockIdx.x;
    const int tid = threadIdx.x;
    if (a.zero_slot && w == 0 && tid == 0) a.x_out[a.chunk - 1] = 0.0;
    if (w < a.nlong_pad) {
        if (w >= a.nlong) return;
        long_segment<BS, U>(a, a.blocks[w], wred, 0.0, a.ypart, S, a.rows);
        return;
    }
    const uint32_t t = w - a.nlong_pad;
    const int xcd = (int)(t & 7u), j = xcd % S;
    const int64_t bi = (int64_t)(t >> 3) * (8 / S) + xcd / S;
    if (bi >= a.nsorted) return;
    const RowBlock b = a.blocks[a.nlong + bi];
    const int nrows = b.row_end - b.row_begin;
    for (int i = tid; i < nrows; i += BS) acc[i] = 0.0;
    __syncthreads();
    gather_range<BS, U, PIPE>(a, b, a.sbound[bi * (S + 1) + j], a.sbound[bi * (S + 1) + j + 1], acc);
    __syncthreads();
    double *y = a.ypart + (int64_t)j * a.rows + b.row_begin;
    for (int i = tid; i < nrows; i += BS) y[i] = acc[i];
}

template <int S>
__global__ __launch_bounds__(256) void k_pr_sliced_epilogue(SortedArgs a) {
    double dsum = 0.0;
    for (int k = 0; k < a.nranks; k++) dsum += a.x_in[(int64_t)k * a.chunk + a.chunk - 1];
    const double teleport = a.teleport0 + a.damping_over_n * dsum;
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.rows; r += (int64_t)gridDim.x * 256) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < S; j++) s += a.ypart[(int64_t)j * a.rows + r];
        sorted_epilogue(a, (int32_t)r, s, teleport);
    }
}

// sbound[i * (S + 1) + j] = first entry of sorted block i whose column is >= cuts[j]
// (cuts[0] = 0, cuts[S] = every column): the block's entries of column slice j.
__global__ void k_sorted_bounds(const RowBlock *__restrict__ blocks, uint32_t nsorted, const int32_t *__restrict__ sci,
                                const int64_t *__restrict__ cuts, int S, int64_t *__restrict__ sbound) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsorted; i += gridDim.x * blockDim.x) {
        const RowBlock b = blocks[i];
        for (int j = 0; j <= S; j++) {
            int64_t lo = b.nz_begin, hi = b.nz_end;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if ((int64_t)sci[mid] < cuts[j]) lo = mid + 1;
                else hi = mid;
            }
            sbound[(int64_t)i * (S + 1) + j] = lo;
        }
    }
}

__global__ void k_col_hist(const int32_t *__restrict__ ci, int64_t nnz, uint32_t *__restrict__ cnt) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[ci[e]], 1u);
}

// keys[coff + t] = (block << 32) | column, vals = block-relative row, for the t-th entry of
// sorted block `blockIdx.x` (one workgroup per block, a wave per row).
__global__ __launch_bounds__(256) void k_sorted_keys(const RowBlock *__restrict__ blocks, const int64_t *__restrict__ coff,
                                                     const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                     uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const RowBlock b = blocks[blockIdx.x];
    const int64_t base = coff[blockIdx.x] - b.nz_begin;
    const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    for (int32_t i = wave; i < b.row_end - b.row_begin; i += 256 / kWave) {
        const int32_t row = b.row_begin + i;
        for (int64_t e = rp[row] + lane; e < rp[row + 1]; e += kWave) {
            keys[base + e] = ((uint64_t)blockIdx.x << 32) | (uint32_t)ci[e];
            vals[base + e] = (uint32_t)i;
        }
    }
}

__global__ __launch_bounds__(256) void k_sorted_unpack(const RowBlock *__restrict__ blocks, const int64_t *__restrict__ coff,
                                                       const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                       int32_t *__restrict__ sci, uint16_t *__restrict__ srl) {
    const RowBlock b = blocks[blockIdx.x];
    const int64_t c0 = coff[blockIdx.x];
    for (int64_t t = threadIdx.x; t < b.nz_end - b.nz_begin; t += 256) {
        sci[b.nz_begin + t] = (int32_t)(uint32_t)keys[c0 + t];
        srl[b.nz_begin + t] = (uint16_t)vals[c0 + t];
    }
}

// spk / gbase from the sorted sci / srl: one workgroup per sorted block, 64-entry groups
// aligned to the block's first entry (the kernel's wave-instructions).
__global__ __launch_bounds__(256) void k_sorted_pack(const RowBlock *__restrict__ blocks, const int32_t *__restrict__ sci,
                                                     const uint16_t *__restrict__ srl, uint32_t *__restrict__ spk,
                                                     uint32_t *__restrict__ gbase) {
    const RowBlock b = blocks[blockIdx.x];
    const int64_t z0 = b.nz_begin, z1 = b.nz_end;
    for (int64_t e = z0 + threadIdx.x; e < z1; e += 256) {
        const int64_t g = (e - z0) >> 6;
        const int64_t first = z0 + (g << 6), last = min(first + 63, z1 - 1);
        const uint32_t base = (uint32_t)sci[first];
        const bool esc = (uint32_t)sci[last] - base >= (1u << (32 - kRowBits));
        spk[e] = esc ? (uint32_t)srl[e] : (((uint32_t)sci[e] - base) << kRowBits) | (uint32_t)srl[e];
        if (e == first) gbase[b.seg + g] = esc ? (base | 0x80000000u) : base;
    }
}

// split[i] = first entry of sorted block i whose column is >= hot (LONG blocks: nz_begin).
__global__ void k_sorted_split(const RowBlock *__restrict__ blocks, uint32_t nblocks, const int32_t *__restrict__ sci,
                               int64_t hot, int64_t *__restrict__ split) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nblocks; i += gridDim.x * blockDim.x) {
        const RowBlock b = blocks[i];
        int64_t lo = b.nz_begin, hi = b.nz_end;
        if (b.split < 0) {
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if ((int64_t)sci[mid] < hot) lo = mid + 1;
                else hi = mid;
            }
        }
        split[i] = lo;
    }
}

int env_int(const char *name, int dflt, int lo, int hi) {
    if (const char *e = std::getenv(name)) {
        const int v = std::atoi(e);
        if (v >= lo && v <= hi) return v;
    }
    return dflt;
}

template <int BS, int U, bool PIPE>
void launch_sorted(const PrPart *p, const SortedArgs &a, hipStream_t s) {
    const size_t lds = (size_t)p->sorted_lds;
    if (!p->two_pass) {
        hipLaunchKernelGGL((k_pr_pull_sorted<BS, U, 0, PIPE>), dim3(p->nblocks), dim3(BS), lds, s, a);
        return;
    }
    hipLaunchKernelGGL((k_pr_pull_sorted<BS, U, 1, PIPE>), dim3(p->nblocks), dim3(BS), lds, s, a);
    const uint32_t ns = p->nblocks - p->nlong_blocks;
    if (ns) {
        SortedArgs t = a;
        t.blocks += p->nlong_blocks;
        t.split += p->nlong_blocks;
        hipLaunchKernelGGL((k_pr_pull_sorted<BS, U, 2, PIPE>), dim3(ns), dim3(BS), lds, s, t);
    }
}

template <int BS, int U, int S>
void launch_sliced(const PrPart *p, const SortedArgs &a, hipStream_t s) {
    const uint32_t per = 8 / S;   // sorted blocks per group of 8 workgroups and slice
    const uint32_t grid = p->nlong_pad + (p->nsorted + per - 1) / per * 8;
    hipLaunchKernelGGL((k_pr_pull_sliced<BS, U, S, true>), dim3(grid), dim3(BS), (size_t)p->sorted_lds, s, a);
    hipLaunchKernelGGL((k_pr_sliced_epilogue<S>), dim3(grid_for(p->rows, 256, 4096)), dim3(256), 0, s, a);
}

// Simulated duration (us) of one k_pr_pull_units launch: the units of every sorted block
// (entries ents[i], rows rws[i]) cut at unit size t, and the LONG segments (lsegs), dealt
// largest first to one workgroup slot per CU, each slot taking the next unit when it frees
// (list scheduling; the grid is issued in that order).  Per-unit cost from the per-workgroup
// timestamps (tools/unit_times.py on SYN-7_5): ~2,900 entries/us of gathers, ~2 ns per row
// (zeroing, epilogue, slab store), ~1.5 us fixed, and the last arriver's slab reads.  It
// picks the unit size, so that the units of the large blocks land in as few waves as the
// CUs allow: e.g. SYN-7_5 at 232 Ki-entry units (5 per 1 Mi block, 325 large units for 256
// CUs) took 130 us per launch against 100 at 256 Ki (4 per block, 260).
double pr_unit_makespan(const std::vector<int64_t> &ents, const std::vector<int64_t> &rws,
                        const std::vector<int64_t> &lsegs, int64_t t, int64_t round, int cus) {
    constexpr double kRate = 2900.0, kRow = 0.002, kFixed = 1.5, kSlab = 0.0005;
    std::vector<double> cost;
    for (size_t i = 0; i < ents.size(); i++) {
        const int64_t E = ents[i];
        const int64_t k = std::max<int64_t>(1, std::min((E + round - 1) / round, (E + t - 1) / t));
        const double c = (double)E / (double)k / kRate + kRow * (double)rws[i] + kFixed +
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
// rows -> blocks of <= sorted_nnz entries and <= sorted_rows rows, entries sorted by column.
int pr_plan_sorted(PrPart *p, const std::vector<int64_t> &h_rp, const std::vector<int32_t> &h_outdeg) {
    const int64_t rows = (int64_t)h_rp.size() - 1;
    const uint64_t nnz = (uint64_t)h_rp[rows];
    // GX_PR_SORTED_VARIANT = 0 (1024 threads, 8 gathers in flight per lane, entry loads
    // pipelined) | 1 (1024, 8, not pipelined) | 2 (512, 16, pipelined) | 3 (512, 8, pipelined)
    p->sorted_variant = env_int("GX_PR_SORTED_VARIANT", 0, 0, 4);
    p->index_x4 = env_int("GX_PR_INDEX_X4", 1, 0, 1);
    p->pipe2 = env_int("GX_PR_PIPE2", 1, 0, 1);
    // hub slice of x for the two-pass mode (GX_PR_HOT_COLS = 0: one pass).  One rank only:
    // in a multi-rank exchange layout the hub columns are spread over every rank's chunk.
    p->hot_cols = env_int("GX_PR_HOT_COLS", (int)p->hot_cols, 0, 1 << 30);
    p->two_pass = p->hot_cols > 0 && p->nranks == 1 && (int64_t)p->chunk > p->hot_cols;
    // XCD column slices (GX_PR_SLICES = 1, 2, 4 or 8; 1 = off); not combined with two passes
    p->slices = env_int("GX_PR_SLICES", p->slices, 1, 8);
    if (8 % p->slices) p->slices = 1;
    if (p->two_pass) p->slices = 1;
    const int64_t cus = std::max(1, p->ctx->num_cus);
    // Split blocks (k_pr_pull_units; one pass, pipelined variants): sorted blocks of up to
    // block_nnz entries and sorted_rows rows, each cut into units of at most T entries
    // (interleaved rounds), one workgroup each, one workgroup per CU; rows longer than
    // block_nnz / 4 take the LONG path.  block_nnz = 1 Mi with 4 Ki rows, 4 Mi once nnz / CUs
    // passes 384 Ki, 8 Mi with 16 Ki rows once it passes 2 Mi, at most 4x the power of two
    // nearest nnz / CUs; T is a quarter block, or past 2 Mi entries per CU chosen below by
    // simulating the launch
    // (pr_unit_makespan).  GX_PR_BLOCK_NNZ, GX_PR_SORTED_ROWS, GX_PR_LONG_NNZ, GX_PR_UNIT_NNZ
    // override.  Measured (tools/pr_units_sweep.sh, us per launch; round 1's 64 Ki
    // single-workgroup blocks in brackets): SYN-7_5 100 [140]; graph500-22 267 [384]; SYN-8_5
    // 1064-1070 [1489].  Larger blocks cut the x line requests (tools/pr_line_model.py) but
    // give the last arriver more slabs per row.
    p->units_mode = !p->two_pass && p->slices == 1 && p->sorted_variant != 1 && !std::getenv("GX_PR_SORTED_NNZ");
    const int64_t round = p->sorted_variant == 3 ? 512 * 8 : p->sorted_variant == 4 ? 1024 * 16 : 1024 * 8;   // U * BS of the launch
    const double per_cu = std::max(1.0, (double)nnz / (double)cus);
    const bool huge = per_cu > (double)(2 << 20);
    // rows per block (LDS accumulators, kRowBits-bit row field; 16 Ki rows = 128 KiB of LDS,
    // which the split-block mode's one workgroup per CU can take)
    const int rmax = p->units_mode && (p->sorted_variant == 0 || p->sorted_variant == 4) ? 1 << kRowBits : 4096;
    p->sorted_rows = env_int("GX_PR_SORTED_ROWS", p->units_mode && huge ? rmax : 4096, 64, rmax);
    int64_t B, T = 0;
    if (p->units_mode) {
        // ... and at most 4x the power of two nearest nnz / CUs, so that a small partition
        // (one rank of eight) keeps about 4 units per block: a 1/8 piece of SYN-7_5 with 1 Mi
        // blocks cut into 32 units each ran 50 us per launch against 34 with 128 Ki blocks
        int64_t pow2 = 1 << 14;
        while (pow2 < (1 << 24) && (double)(2 * pow2) <= per_cu * 1.41421356) pow2 *= 2;
        const int64_t bdef = std::min<int64_t>(huge ? 8 << 20 : per_cu > 384.0 * 1024 ? 4 << 20 : 1 << 20, 4 * pow2);
        B = env_int("GX_PR_BLOCK_NNZ", (int)bdef, 1024, 1 << 30);
        p->long_nnz = env_int("GX_PR_LONG_NNZ", (int)std::max<int64_t>(B / 4, round), 1024, 1 << 30);
    } else {
        // entries per block: GX_PR_SORTED_NNZ, else 65536 -- 32768 when the partition gives
        // fewer than one block per CU (the 1/4 and 1/8 partitions of SYN-7_5 ran best at 32 Ki:
        // 35 us vs 37 at 16 Ki and 67 at 64 Ki for 1/8), or doubled up to 1 Mi while it gives
        // more than four per CU (round 1, one workgroup per block: tools/pr_sorted_sweep.sh)
        B = p->sorted_nnz;
        if (std::getenv("GX_PR_SORTED_NNZ")) {
            B = env_int("GX_PR_SORTED_NNZ", p->sorted_nnz, 1024, 1 << 22);
        } else {
            while (B > 32768 && (int64_t)nnz < B * cus) B >>= 1;
            while (B < (1 << 20) && (int64_t)nnz > 4 * B * cus) B <<= 1;
        }
        p->long_nnz = env_int("GX_PR_LONG_NNZ", (int)B, 1024, 1 << 24);
    }
    p->sorted_nnz = (int)B;
    p->unit_nnz = T;
    const int64_t BB = B;
    const int64_t R = p->sorted_rows, LT = std::max<int64_t>(p->long_nnz, 1);
    std::vector<RowBlock> longb, sortb;
    std::vector<int32_t> lfirst, lnseg;
    std::vector<std::pair<int64_t, int32_t>> longrows;
    int32_t nsegs = 0;
    int64_t r = 0;
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
            if (l > LT || nz + l > BB) break;
            nz += l;
            r++;
        }
        sortb.push_back({h_rp[start], h_rp[r], (int32_t)start, (int32_t)r, -1, 0});
    }
    // seg of a sorted block = index of its first 64-entry group in gbase
    int64_t ngroups = 0;
    for (RowBlock &b : sortb) {
        b.seg = (int32_t)ngroups;
        ngroups += (b.nz_end - b.nz_begin + 63) / 64;
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
    int64_t maxrows = 1;
    for (const RowBlock &b : sortb) maxrows = std::max<int64_t>(maxrows, b.row_end - b.row_begin);
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
    GX_TRY(p->ssplit.alloc(std::max<size_t>(all.size(), 1)));
    if (p->two_pass) GX_TRY(p->ypart.alloc(std::max<int64_t>(rows, 1)));

    // block-sorted columns and packed entries (entries of LONG rows stay unused there)
    GX_TRY(p->sci.alloc(std::max<uint64_t>(nnz, 1), 16));
    GX_TRY(p->spk.alloc(std::max<uint64_t>(nnz, 1), 16));
    GX_TRY(p->gbase.alloc(std::max<int64_t>(ngroups, 1), 16));
    hipStream_t s = p->ctx->stream;
    std::vector<int64_t> coff(sortb.size());
    int64_t m = 0;
    for (size_t j = 0; j < sortb.size(); j++) {
        coff[j] = m;
        m += sortb[j].nz_end - sortb[j].nz_begin;
    }
    const RowBlock *d_sort = p->blocks.p + longb.size();
    if (m > 0) {
        DBuf<int64_t> d_coff;
        DBuf<uint64_t> k0, k1;
        DBuf<uint32_t> v0, v1;
        DBuf<uint16_t> srl;
        GX_TRY(d_coff.alloc(coff.size()));
        GX_TRY(k0.alloc(m));
        GX_TRY(k1.alloc(m));
        GX_TRY(v0.alloc(m));
        GX_TRY(v1.alloc(m));
        GX_TRY(srl.alloc(std::max<uint64_t>(nnz, 1), 16));
        GX_HIP_TRY(hipMemcpy(d_coff.p, coff.data(), coff.size() * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_sorted_keys, dim3((unsigned)sortb.size()), dim3(256), 0, s, d_sort, d_coff.p, p->rp, p->ci,
                           k0.p, v0.p);
        GX_TRY(check_launch("k_sorted_keys"));
        int bits = 1;
        while ((1ull << bits) < sortb.size()) bits++;
        GX_TRY(sort_pairs_u64_u32(k0.p, k1.p, v0.p, v1.p, (size_t)m, 32 + bits, s));
        hipLaunchKernelGGL(k_sorted_unpack, dim3((unsigned)sortb.size()), dim3(256), 0, s, d_sort, d_coff.p, k1.p, v1.p,
                           p->sci.p, srl.p);
        GX_TRY(check_launch("k_sorted_unpack"));
        hipLaunchKernelGGL(k_sorted_pack, dim3((unsigned)sortb.size()), dim3(256), 0, s, d_sort, p->sci.p, srl.p,
                           p->spk.p, p->gbase.p);
        GX_TRY(check_launch("k_sorted_pack"));
        GX_HIP_TRY(hipStreamSynchronize(s));   // the key buffers are freed at return
    }
    p->nsorted = (uint32_t)sortb.size();
    p->nlong_pad = (p->nlong_blocks + 7u) & ~7u;
    if (p->slices > 1 && !sortb.empty()) {
        // column cuts with equal shares of the sorted blocks' entries
        const int S = p->slices;
        const uint64_t ncols = p->chunk * (uint64_t)p->nranks;
        DBuf<uint32_t> cnt;
        GX_TRY(cnt.alloc(ncols));
        GX_HIP_TRY(hipMemsetAsync(cnt.p, 0, ncols * 4, s));
        if (nnz) {
            hipLaunchKernelGGL(k_col_hist, dim3(grid_for(nnz, 256, 16384)), dim3(256), 0, s, p->ci, (int64_t)nnz, cnt.p);
            GX_TRY(check_launch("k_col_hist"));
        }
        std::vector<uint32_t> h(ncols);
        GX_HIP_TRY(hipMemcpyAsync(h.data(), cnt.p, ncols * 4, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        std::vector<int64_t> cuts(S + 1, 0);
        cuts[S] = (int64_t)ncols;
        uint64_t acc = 0;
        int j = 1;
        for (uint64_t c = 0; c < ncols && j < S; c++) {
            acc += h[c];
            while (j < S && acc * (uint64_t)S >= (uint64_t)j * nnz) cuts[j++] = (int64_t)c + 1;
        }
        for (; j < S; j++) cuts[j] = (int64_t)ncols;
        DBuf<int64_t> d_cuts;
        GX_TRY(d_cuts.alloc(S + 1));
        GX_TRY(p->sbound.alloc((size_t)sortb.size() * (S + 1)));
        GX_TRY(p->ypart.alloc((size_t)S * std::max<int64_t>(rows, 1)));
        GX_HIP_TRY(hipMemcpy(d_cuts.p, cuts.data(), (S + 1) * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_sorted_bounds, dim3(grid_for(sortb.size(), 256, 1024)), dim3(256), 0, s, d_sort,
                           (uint32_t)sortb.size(), p->sci.p, d_cuts.p, S, p->sbound.p);
        GX_TRY(check_launch("k_sorted_bounds"));
        GX_HIP_TRY(hipStreamSynchronize(s));
    }
    // units of the split blocks (one pass): ceil(entries / T) per sorted block (at most one
    // per round of entries)
    p->nunits = 0;
    if (p->units_mode && !sortb.empty()) {
        if (std::getenv("GX_PR_UNIT_NNZ")) {
            T = env_int("GX_PR_UNIT_NNZ", 65536, 1024, 1 << 30);
        } else if (!huge) {
            // a quarter block: measured best on SYN-7_5 (256 Ki of 1 Mi: 100 us per launch;
            // 232 Ki: 130) and on its 1/8 partition (32 Ki of 128 Ki: 33.5 us; the simulation's
            // choice, 24 Ki: 38.8; 64 Ki: 47.7; tools/pr_piece_sweep.sh)
            T = std::max<int64_t>(round, (B / 4 + round - 1) / round * round);
        } else {
            // the unit size whose simulated launch is shortest, over multiples of a round
            std::vector<int64_t> ents, rws, lsegs;
            for (const RowBlock &b : sortb) {
                ents.push_back(b.nz_end - b.nz_begin);
                rws.push_back(b.row_end - b.row_begin);
            }
            for (const RowBlock &b : longb) lsegs.push_back(b.nz_end - b.nz_begin);
            double best = 0.0;
            const int64_t emax = *std::max_element(ents.begin(), ents.end());
            for (int64_t t = round; t <= std::max<int64_t>(round, emax); t += round) {
                const double m = pr_unit_makespan(ents, rws, lsegs, t, round, (int)cus);
                if (T == 0 || m < best * 0.999) {
                    best = m;
                    T = t;
                }
            }
            if (env_int("GX_PR_VERBOSE", 0, 0, 1))
                std::fprintf(stderr, "[gx_pr] unit size %lld: simulated launch %.1f us\n", (long long)T, best);
        }
        p->unit_nnz = T;
        // GX_PR_UNIT_LAYOUT = 1 (default): interleaved rounds of kUnitRound entries; 0:
        // contiguous ranges (each unit its own column range: the units of a block then need
        // different parts of x at the same time)
        const bool interleave = env_int("GX_PR_UNIT_LAYOUT", 1, 0, 1) == 1;
        const int64_t kUnitRound = round;
        std::vector<SortedUnit> units;
        int64_t slab = 0;
        int32_t parts = 0;
        for (size_t i = 0; i < sortb.size(); i++) {
            const RowBlock &b = sortb[i];
            const int64_t E = b.nz_end - b.nz_begin, G = (E + 63) / 64;
            const int64_t rounds = (E + kUnitRound - 1) / kUnitRound;
            const int32_t k = (int32_t)std::max<int64_t>(
                1, std::min<int64_t>(interleave ? rounds : G, (E + T - 1) / T));
            const int64_t rows_b = b.row_end - b.row_begin;
            for (int32_t j = 0; j < k; j++) {
                SortedUnit u;
                if (interleave) {
                    u.lo = b.nz_begin + kUnitRound * j;
                    u.hi = b.nz_end;
                    u.step = kUnitRound * k;
                } else {
                    u.lo = b.nz_begin + 64 * (G * j / k);
                    u.hi = std::min(b.nz_begin + 64 * (G * (j + 1) / k), b.nz_end);
                    u.step = kUnitRound;
                }
                u.slab = k > 1 ? slab : 0;
                u.blk = (int32_t)(longb.size() + i);
                u.part = k > 1 ? parts : -1;
                u.unit = j;
                u.nunits = k;
                units.push_back(u);
            }
            if (k > 1) {
                slab += (int64_t)k * rows_b;
                parts++;
            }
        }
        // Largest units first (GX_PR_UNIT_ORDER=1, the default): the launch lasts as long as
        // the unit that finishes last, so the big units start in the first wave and the small
        // ones fill the gaps at the end.  Cost ~ entries + 4 per row (zeroing, epilogue).
        // Ties keep block order, so a block's units stay adjacent.
        if (env_int("GX_PR_UNIT_ORDER", 1, 0, 1)) {
            auto cost = [&](const SortedUnit &u) {
                const RowBlock &b = sortb[u.blk - longb.size()];
                const int64_t E = b.nz_end - b.nz_begin;
                return (E + u.nunits - 1) / u.nunits + 4 * (int64_t)(b.row_end - b.row_begin);
            };
            std::stable_sort(units.begin(), units.end(),
                             [&](const SortedUnit &x, const SortedUnit &y) { return cost(x) > cost(y); });
        }
        // XCD grouping (GX_PR_UNIT_XCD=1; off by default: SYN-7_5 took 117.7 us per launch with
        // it against 102.9 without, tools/pr_units_sweep.sh): the units of one block sweep the same
        // column range at the same time, so they share x lines -- if they run on one XCD, its
        // L2 fetches each line once for all of them.  Workgroups are dealt round-robin over
        // the 8 XCDs (MI355X_MICROARCH.md, dispatch: w and w + 8 share one; speed only, never
        // correctness), so each block goes whole to the least-loaded of 8 lists and grid slot
        // 8 i + x runs list x's i-th unit; short lists are padded with empty units (blk -1).
        if (env_int("GX_PR_UNIT_XCD", 0, 0, 1) && units.size() > 8) {
            std::vector<std::vector<SortedUnit>> lists(8);
            std::vector<int64_t> load(8, 0);
            for (size_t i = 0; i < units.size();) {
                size_t j = i;
                while (j < units.size() && units[j].blk == units[i].blk) j++;
                const RowBlock &b = sortb[units[i].blk - longb.size()];
                const int x = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                for (size_t k = i; k < j; k++) lists[x].push_back(units[k]);
                load[x] += b.nz_end - b.nz_begin;
                i = j;
            }
            size_t L = 0;
            for (const auto &l : lists) L = std::max(L, l.size());
            SortedUnit empty{};
            empty.blk = -1;
            std::vector<SortedUnit> grid(8 * L, empty);
            for (int x = 0; x < 8; x++)
                for (size_t i = 0; i < lists[x].size(); i++) grid[8 * i + x] = lists[x][i];
            units.swap(grid);
        }
        p->nunits = (uint32_t)units.size();
        if (env_int("GX_PR_VERBOSE", 0, 0, 1))
            std::fprintf(stderr, "[gx_pr] plan: rows %lld nnz %llu unit_nnz %lld block_nnz %d long_nnz %d: "
                         "%zu sorted blocks, %u LONG blocks (%u rows), %u units, %d multi-unit blocks, slab %lld doubles\n",
                         (long long)rows, (unsigned long long)nnz, (long long)T, p->sorted_nnz, p->long_nnz,
                         sortb.size(), p->nlong_blocks, p->nlong, p->nunits, parts, (long long)slab);
        GX_TRY(p->units.alloc(units.size()));
        GX_HIP_TRY(hipMemcpy(p->units.p, units.data(), units.size() * sizeof(SortedUnit), hipMemcpyHostToDevice));
        GX_TRY(p->uslab.alloc(std::max<int64_t>(slab, 1)));
        GX_TRY(p->uticket.alloc(std::max<int32_t>(parts, 1)));
        GX_HIP_TRY(hipMemset(p->uticket.p, 0, p->uticket.n * 4));
    }
    // fused dangling sum: one pass, and every dangling row in a sorted block
    {
        std::vector<int32_t> slot(all.size(), -1);
        bool long_dangling = false;
        for (const RowBlock &b : longb) long_dangling |= h_outdeg[b.row_begin] == 0;
        uint32_t nd = 0;
        for (size_t i = longb.size(); i < all.size(); i++) {
            bool any = false;
            for (int32_t r2 = all[i].row_begin; r2 < all[i].row_end && !any; r2++) any = h_outdeg[r2] == 0;
            if (any) slot[i] = (int32_t)nd++;
        }
        p->fused_dangling = p->nd > 0 && nd > 0 && !long_dangling && !p->two_pass && p->slices == 1;
        p->ndblocks = nd;
        if (p->fused_dangling) {
            GX_TRY(p->dslot.alloc(all.size()));
            GX_TRY(p->fdpart.alloc(nd));
            GX_TRY(p->fdticket.alloc(1));
            GX_HIP_TRY(hipMemcpy(p->dslot.p, slot.data(), all.size() * 4, hipMemcpyHostToDevice));
            GX_HIP_TRY(hipMemset(p->fdticket.p, 0, 4));
        }
    }
    if (!all.empty()) {
        hipLaunchKernelGGL(k_sorted_split, dim3(grid_for(all.size(), 256, 1024)), dim3(256), 0, s, p->blocks.p,
                           (uint32_t)all.size(), p->sci.p, (int64_t)p->hot_cols, p->ssplit.p);
        GX_TRY(check_launch("k_sorted_split"));
        GX_HIP_TRY(hipStreamSynchronize(s));
    }
    return GX_SUCCESS;
}

int pr_step_sorted(PrPart *p, const double *x_full, double *x_local, double *rank_out, hipStream_t s) {
    const double dn = (double)p->n_global;
    SortedArgs a;
    a.blocks = p->blocks.p;
    a.split = p->ssplit.p;
    a.ci = p->ci;
    a.sci = p->sci.p;
    a.spk = p->spk.p;
    a.gbase = p->gbase.p;
    a.outdeg = p->outdeg;
    a.x_in = x_full;
    a.x_out = x_local;
    a.rank_out = rank_out;
    a.ypart = p->ypart.p;
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
    a.sbound = p->sbound.p;
    a.rows = (int64_t)p->rows;
    a.nlong = p->nlong_blocks;
    a.nlong_pad = p->nlong_pad;
    a.nsorted = p->nsorted;
    a.dslot = p->fused_dangling ? p->dslot.p : nullptr;
    a.dpart = p->fdpart.p;
    a.dticket = p->fdticket.p;
    a.ndblocks = p->ndblocks;
    a.units = p->units.p;
    a.uslab = p->uslab.p;
    a.uticket = p->uticket.p;
    a.xd = p->xd.p;
    a.live = (int64_t)p->live;
    a.utimes = nullptr;
    const char *times_path = std::getenv("GX_PR_UNIT_TIMES");   // debug: not under graph capture
    if (times_path && p->nunits) {
        if (!p->utimes.p) GX_TRY(p->utimes.alloc(4 * (size_t)(p->nlong_blocks + p->nunits)));
        a.utimes = p->utimes.p;
    }
    if (p->nunits) {
        KTimer kt(p->ctx, "pr_pull", s);   // one iteration's SpMV (+ fused dangling sum)
        const dim3 grid(p->nlong_pad + p->nunits);
        // One 1024-thread workgroup per CU (GX_PR_UNIT_LDS, bytes: the LDS reserved per
        // workgroup; 0 = only the accumulators, two per CU).  Fewer concurrent sweeps keep
        // the XCD's L2 window of x smaller: SYN-7_5 one per CU 100-104 us per launch against
        // 109-125 with two (tools/pr_units_sweep.sh).
        const int pad = p->sorted_variant == 0 || p->sorted_variant == 4 ? 96 * 1024 : 0;
        const size_t lds = std::max<size_t>((size_t)p->sorted_lds, (size_t)env_int("GX_PR_UNIT_LDS", pad, 0, 160 * 1024 - 4096));
        if (a.utimes) {
            if (p->index_x4) hipLaunchKernelGGL((k_pr_pull_units<1024, 8, true, true>), grid, dim3(1024), lds, s, a);
            else hipLaunchKernelGGL((k_pr_pull_units<1024, 8, true, false>), grid, dim3(1024), lds, s, a);
        } else {
            switch (p->sorted_variant) {
            case 2: hipLaunchKernelGGL((k_pr_pull_units<512, 16, false>), grid, dim3(512), lds, s, a); break;
            case 3: hipLaunchKernelGGL((k_pr_pull_units<512, 8, false>), grid, dim3(512), lds, s, a); break;
            case 4: hipLaunchKernelGGL((k_pr_pull_units<1024, 16, false, true>), grid, dim3(1024), lds, s, a); break;
            default:
                // GX_PR_INDEX_X4=0: one 4-B index load per entry (round 2's kernel)
#ifdef GX_PR_PROBES
                if (const char *pe = std::getenv("GX_PR_PROBE")) {
                    switch (std::atoi(pe)) {
#define GX_PROBE_CASE(k) case k: hipLaunchKernelGGL((k_pr_pull_units<1024, 8, false, true, true, k>), grid, dim3(1024), lds, s, a); break;
                    GX_PROBE_CASE(1) GX_PROBE_CASE(2) GX_PROBE_CASE(3) GX_PROBE_CASE(4) GX_PROBE_CASE(5) GX_PROBE_CASE(6) GX_PROBE_CASE(7)
#undef GX_PROBE_CASE
                    default: hipLaunchKernelGGL((k_pr_pull_units<1024, 8, false, true, true>), grid, dim3(1024), lds, s, a);
                    }
                    break;
                }
#endif
                if (p->index_x4 && p->pipe2) hipLaunchKernelGGL((k_pr_pull_units<1024, 8, false, true, true>), grid, dim3(1024), lds, s, a);
                else if (p->index_x4) hipLaunchKernelGGL((k_pr_pull_units<1024, 8, false, true>), grid, dim3(1024), lds, s, a);
                else hipLaunchKernelGGL((k_pr_pull_units<1024, 8, false, false>), grid, dim3(1024), lds, s, a);
                break;
            }
        }
        if (a.utimes && ++p->utimes_launch == env_int("GX_PR_UNIT_TIMES_LAUNCH", 5, 1, 1 << 30)) {
            const size_t nw = p->nlong_pad + p->nunits;
            std::vector<uint64_t> t(4 * nw);
            std::vector<SortedUnit> us(p->nunits);
            std::vector<RowBlock> bs(p->nblocks);
            GX_HIP_TRY(hipStreamSynchronize(s));
            GX_HIP_TRY(hipMemcpy(t.data(), p->utimes.p, t.size() * 8, hipMemcpyDeviceToHost));
            GX_HIP_TRY(hipMemcpy(us.data(), p->units.p, us.size() * sizeof(SortedUnit), hipMemcpyDeviceToHost));
            GX_HIP_TRY(hipMemcpy(bs.data(), p->blocks.p, bs.size() * sizeof(RowBlock), hipMemcpyDeviceToHost));
            if (FILE *f = std::fopen(times_path, "w")) {
                std::fprintf(f, "wg kind blk unit nunits entries rows t0 tgather t1 xcc\n");
                for (size_t w = 0; w < nw; w++) {
                    if (w >= p->nlong_blocks && w < p->nlong_pad) continue;
                    if (w >= p->nlong_pad && us[w - p->nlong_pad].blk < 0) continue;
                    const bool lng = w < p->nlong_blocks;
                    const RowBlock &b = lng ? bs[w] : bs[us[w - p->nlong_pad].blk];
                    long long ents = lng ? b.nz_end - b.nz_begin : 0;
                    if (!lng) {
                        const SortedUnit &u = us[w - p->nlong_pad];
                        for (int64_t k0 = u.lo; k0 < u.hi; k0 += u.step) ents += std::min<int64_t>(u.step / u.nunits, u.hi - k0);
                    }
                    std::fprintf(f, "%zu %s %d %d %d %lld %d %llu %llu %llu %llu\n", w, lng ? "long" : "unit",
                                 lng ? (int)w : us[w - p->nlong_pad].blk, lng ? 0 : us[w - p->nlong_pad].unit,
                                 lng ? 1 : us[w - p->nlong_pad].nunits, ents, b.row_end - b.row_begin,
                                 (unsigned long long)t[4 * w], (unsigned long long)t[4 * w + 1],
                                 (unsigned long long)t[4 * w + 2], (unsigned long long)t[4 * w + 3]);
                }
                std::fclose(f);
            }
        }
    } else if (p->nblocks && p->slices > 1) {
        KTimer kt(p->ctx, "pr_pull", s);   // sliced SpMV + epilogue: one iteration
        switch (p->slices) {
        case 2: launch_sliced<1024, 8, 2>(p, a, s); break;
        case 4: launch_sliced<1024, 8, 4>(p, a, s); break;
        default: launch_sliced<1024, 8, 8>(p, a, s); break;
        }
    } else if (p->nblocks) {
        KTimer kt(p->ctx, "pr_pull", s);   // both passes: one iteration's SpMV
        switch (p->sorted_variant) {
        case 1: launch_sorted<1024, 8, false>(p, a, s); break;
        case 2: launch_sorted<512, 16, true>(p, a, s); break;
        case 3: launch_sorted<512, 8, true>(p, a, s); break;
        default: launch_sorted<1024, 8, true>(p, a, s); break;
        }
    } else if (a.zero_slot) {
        GX_HIP_TRY(hipMemsetAsync(x_local + p->chunk - 1, 0, sizeof(double), s));
    }
    GX_TRY(check_launch("k_pr_pull_sorted"));
    return p->fused_dangling ? GX_SUCCESS : pr_dangling(p, x_local, s);
}

}  // namespace gx

GX_MODULE_WARMER(pr_sorted)
