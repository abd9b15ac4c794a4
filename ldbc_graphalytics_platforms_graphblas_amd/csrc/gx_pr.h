// gx_pr.h -- PageRank pull plan (row blocks of the pull matrix of one rank).
#pragma once

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <algorithm>

#include "gx_device.h"

namespace gx {

// GX_PLAN_TIMES=1: the host-side phase times of a plan build on stderr (the stream is
// synchronised at every mark, so device phases are attributed too).  Diagnostics only.
// GX_PLAN_TIMES=2: host time only, no stream synchronisation (the phases' host-side cost,
// without perturbing a call whose upload overlaps its plan).
struct PlanClock {
    bool on = false, sync = true;
    hipStream_t s = nullptr;
    const char *what = "";
    std::chrono::steady_clock::time_point t;
    PlanClock(const char *w, hipStream_t st) : s(st), what(w) {
        const char *e = std::getenv("GX_PLAN_TIMES");
        on = e && std::atoi(e) != 0;
        sync = !(e && std::atoi(e) == 2);
        if (on) {
            if (sync) (void)hipStreamSynchronize(s);
            t = std::chrono::steady_clock::now();
        }
    }
    void mark(const char *phase) {
        if (!on) return;
        if (sync) (void)hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[plan %s] %-28s %8.2f ms\n", what, phase,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// One workgroup's share of the pull SpMV (the CSR-Adaptive split):
//   split <  0 : STREAM  -- rows [row_begin, row_end), all of them short, <= kStreamNnz
//                 entries in total; staged through LDS, reduced per row.
//   split >= 0 : LONG    -- entries [nz_begin, nz_end) of the single row row_begin;
//                 rows longer than kSegNnz are cut into several segments whose partial
//                 sums are combined by the last-arriving workgroup (ticket per row).
struct RowBlock {
    int64_t nz_begin;
    int64_t nz_end;
    int32_t row_begin;
    int32_t row_end;
    int32_t split;      // -1 stream; else index into the per-long-row ticket/partials
    int32_t seg;        // segment number within the long row
};

// One workgroup's share of a column-sorted block (k_pr_pull_units, gx_pr_sorted.hip): the
// sorted entries [lo, hi) of block `blk` in rounds of the kernel's U * BS entries, taking
// every (step / (U * BS))-th round (interleaved units: every unit sweeps the block's whole
// column range, so the units of a block move through x together).  A block cut into
// nunits > 1 units sums its rows through per-unit partial slabs (slab + unit * rows doubles);
// the last unit to arrive (ticket[part]) adds them in unit order and runs the epilogue.
// The block's column-sorted prefix of dense columns is stored as narrow 2-byte codes (nbeg,
// nsg: the block's first code in PrPart::npk and its 512-code supergroups); [lo, hi) is the
// wide 4-byte remainder.  Unit j of k takes narrow rounds j, j + k, ... as well.
struct SortedUnit {
    int64_t lo;
    int64_t hi;
    int64_t step;
    int64_t slab;       // first double of the block's slabs in PrPart::uslab
    int64_t nbeg;       // first narrow code of the block (a multiple of 512)
    int32_t nsg;        // narrow supergroups (512 codes each) of the block
    int32_t blk;        // index into PrPart::blocks
    int32_t part;       // ticket index of a multi-unit block, -1 when nunits == 1
    int32_t unit;       // this unit's number within the block
    int32_t nunits;
    int32_t seg;        // the block's fields (RowBlock), so a workgroup's first loads are
    int64_t z0, z1;     //   independent: its block's entries [z0, z1), rows [r0, r1), first
    int32_t r0, r1;     //   supergroup seg
};

// A row stripe of a multi-unit block, combined by k_pr_combine after the units' launch
// (PrPart::comb_kernel): rows [s0, s1) of the block whose rows start at local row r0 and whose
// k slabs of nrows doubles begin at uslab[slab]; dslot its dangling partial's slot or -1.
struct CombStripe {
    int64_t slab;
    int32_t r0, nrows, s0, s1, k, dslot;
};

// x of local row `row`: rows [0, live) sit in the exchanged chunk, the rest (out-degree 0, so
// no rank ever gathers them) in the rank-private xd, so that only the gathered prefix of each
// rank's rows travels in the all-gather (gx_pr_part_create_live).
__device__ __forceinline__ void store_x(double *x_out, double *xd, int64_t live, int64_t row, double v) {
    if (row < live) x_out[row] = v;
    else xd[row - live] = v;
}

constexpr int kPullBlock = 256;      // 4 waves
constexpr int kStreamNnz = 2048;     // LDS stage: 16 KiB of fp64 per workgroup
constexpr int kStreamRows = 256;     // at most one row per lane in stream mode
constexpr int kSegNnz = 8192;        // entries per LONG segment

struct PrPart {
    gx_ctx *ctx = nullptr;
    uint64_t n_global = 0;
    int nranks = 1, rank = 0;
    uint64_t rows = 0;       // local rows
    uint64_t chunk = 0;      // doubles per rank chunk (last one = dangling slot)
    uint64_t live = ~0ull;   // local rows kept in the chunk; rows [live, rows) have x in xd (~0: all)
    DBuf<double> xd;         // x of the rows past `live` (out-degree 0, never gathered)
    double damping = 0.85;
    // pull matrix of the local rows (column ids already in the padded chunk layout)
    DBuf<int64_t> rp_own;    // when the plan owns its matrix
    DBuf<int32_t> ci_own;
    const int64_t *rp = nullptr;
    const int32_t *ci = nullptr;
    DBuf<int32_t> outdeg_own;
    const int32_t *outdeg = nullptr;   // out-degree of each local row's vertex
    // row blocks
    DBuf<RowBlock> blocks;
    uint32_t nblocks = 0;
    uint32_t nlong_blocks = 0;   // LONG blocks come first in `blocks`
    DBuf<int32_t> long_first;  // per long row: index of its first partial
    DBuf<int32_t> long_nseg;   // per long row: number of segments
    DBuf<double> long_part;    // per segment partial sum
    DBuf<uint32_t> long_ticket;
    uint32_t nlong = 0, nsegs = 0;
    // dangling rows (out-degree 0) of this rank
    DBuf<int32_t> dlist;      // only when the dangling rows are not one contiguous range
    uint64_t nd = 0;
    bool d_range = false;
    int64_t d0 = 0;
    uint32_t dgrid = 0;
    DBuf<double> dpart;
    DBuf<uint32_t> dticket;
    // column-sorted blocks (k_pr_pull_units, gx_pr_sorted.hip; the default)
    DBuf<int32_t> sci;           // columns sorted within each block
    DBuf<uint32_t> spk;          // packed (column - group base) << 14 | row
    DBuf<uint32_t> gbase;        // base column per 256-entry supergroup (bit 31: escape to sci)
    // narrow codes (gx_pr_sorted.hip): (column delta 0..3) << 14 | row, per block a 512-aligned
    // run; the column of a code is its 512-code supergroup's base plus the deltas up to it
    DBuf<uint16_t> npk;
    DBuf<uint32_t> nbase;        // per narrow supergroup: the column before its first code
    uint64_t nnarrow = 0;        // narrow entries (without the delta-only fillers)
    uint64_t ncodes = 0;         // narrow codes, fillers and padding included
    uint32_t null_sg = 0;        // an all-padding supergroup gathering x's zero slot
    int sorted_nnz = 65536;      // entries per block
    int sorted_rows = 4096;      // rows per block (LDS accumulators)
    int64_t unit_nnz = 0;        // target entries per unit
    DBuf<SortedUnit> units;      // one workgroup per unit, after the LONG blocks
    uint32_t nunits = 0;
    DBuf<double> uslab;          // partial row sums of the multi-unit blocks
    DBuf<uint32_t> uticket;      // per multi-unit block: arrivals of the current iteration
    // GX_PR_COMBINE=1: the multi-unit blocks' slabs are added up and their epilogue run by a
    // second kernel over row stripes (k_pr_combine), not by each block's last arriving unit
    bool comb_kernel = false;
    bool force_huge = false;     // the huge-graph plan whatever the size (a block partition's rank)
    DBuf<CombStripe> cstripes;
    uint32_t ncstripes = 0;
    DBuf<uint64_t> utimes;       // debug (GX_PR_UNIT_TIMES): per-workgroup timestamps
    int utimes_launch = 0;
    int long_nnz = 65536;        // longer rows take the LONG segment path
    int sorted_lds = 0;          // dynamic LDS bytes of the launch
    int cache_policy = 0;        // k_pr_pull_units CP: 1 index stream non-temporal, 5 also the narrow
                                 // gathers from column nt_col on (x larger than the L2s)
    uint32_t nt_col = 65536;
    uint32_t nsorted = 0, nlong_pad = 0;
    // paced sweep (GX_PR_PACE, gx_pr_sorted.hip): x's columns cut into windows (window 0 below
    // pace_h, then 2^pace_wshift columns each); per unit the round at which each window starts
    // (narrow rounds, then wide rounds: units x 2 (nw + 1)); per XCD one progress word per CU
    // slot.  The units of one XCD and generation keep within pace_d windows of each other, so
    // the x lines one fetches into the XCD's L2 are still there for the others.
    bool rows_desc = false;      // row lengths non-increasing (an undirected hub-first plan): the
                                 // block cut jumps by binary search
    int pace = 0;
    int queue_on = -1;           // GX_PR_QUEUE: one resident workgroup per CU pulling work items (-1 auto)
    DBuf<uint32_t> queue;        // its counters (k_pr_pull_units QUEUE)
    uint32_t pace_nw = 0, pace_h = 0, pace_wshift = 18, pace_d = 1, pace_polls = 64;
    DBuf<int32_t> pace_rounds;
    DBuf<uint32_t> pace_prog;
    // dangling-score sum fused into the kernel: blocks holding out-degree-0 rows publish a
    // partial, the last of them adds them up in slot order
    bool fused_dangling = false;
    DBuf<int32_t> dslot;         // per block: its partial's slot, -1 = no dangling rows
    DBuf<double> fdpart;
    DBuf<uint32_t> fdticket;
    uint32_t ndblocks = 0;
    int kernel = 2;              // 1 = k_pr_pull (CSR-Adaptive, GX_PR_KERNEL=adaptive), 2 = k_pr_pull_units
    // where the sorted plan reads its entries: local row i is row order[i] of (src_rp, src_ci)
    // with every column c renamed perm[c] (gx_pagerank's hub-first plan), or row i itself with
    // its columns as stored (order / perm null: a partition already in its final order)
    const int64_t *src_rp = nullptr;
    const int32_t *src_ci = nullptr;
    const int32_t *src_order = nullptr;
    const int32_t *src_perm = nullptr;
    UploadJob *job = nullptr;  // the source columns still arriving (gx_pagerank_csr): the plan's key
                               // pass scatters each chunk from the source order once it has landed
    DBuf<int32_t> order;       // hub-first position -> old vertex id (gx_pagerank)
    // single-GPU driver buffers (gx_pagerank): vertices relabelled hub-first
    DBuf<double> xa, xb, rank_out, result;
    DBuf<int32_t> perm;        // old vertex id -> position in the hub-first order
};

// A non-increasing sequence of n row lengths as its runs of equal values: run k covers
// positions [pos[k], pos[k+1]) with length val[k], and base[k] entries come before it.  The row
// pointers and lengths of an undirected graph's hub-first rows, known from the device's sorted
// degrees without moving 12 n bytes to the host (pr_single_plan).
struct LengthRuns {
    std::vector<int64_t> pos, val, base;
    uint64_t n = 0;
    int64_t total = 0;
    size_t run(uint64_t i) const {
        return (size_t)(std::upper_bound(pos.begin(), pos.end(), (int64_t)i) - pos.begin()) - 1;
    }
    int64_t prefix(uint64_t i) const {
        if (i >= n) return total;
        const size_t k = run(i);
        return base[k] + ((int64_t)i - pos[k]) * val[k];
    }
    int64_t length(uint64_t i) const { return val[run(i)]; }
};

// Read-only host array (a std::vector, or a buffer the plan filled without zeroing it), or the
// row pointers (prefix) / lengths of a LengthRuns.  Elements are values, not references.
template <typename T>
struct HostView {
    const T *p = nullptr;
    size_t n = 0;
    const LengthRuns *runs = nullptr;
    bool prefix = false;
    template <typename Alloc>
    HostView(const std::vector<T, Alloc> &v) : p(v.data()), n(v.size()) {}
    HostView(const T *ptr, size_t count) : p(ptr), n(count) {}
    HostView(const LengthRuns *r, bool pre) : n(pre ? r->n + 1 : r->n), runs(r), prefix(pre) {}
    size_t size() const { return n; }
    T operator[](size_t i) const { return p ? p[i] : (T)(prefix ? runs->prefix(i) : runs->length(i)); }
};

// Build the row-block plan and dangling list from a local pull CSR (host row pointers
// h_rp, device rp/ci) and device out-degrees.  Borrowed device pointers must outlive it.
int pr_plan(PrPart *p, HostView<int64_t> h_rp, const int64_t *d_rp,
            const int32_t *d_ci, const int32_t *d_outdeg, HostView<int32_t> h_outdeg);

// Column-sorted block plan (k_pr_pull_units) and its iteration (gx_pr_sorted.hip).
int pr_plan_sorted(PrPart *p, HostView<int64_t> h_rp, HostView<int32_t> h_outdeg);
int pr_step_sorted(PrPart *p, const double *x_full, double *x_local, double *rank_out, hipStream_t s);
// Dangling-score sum of this rank into x_local's last chunk slot.
int pr_dangling(PrPart *p, double *x_local, hipStream_t s);

int pr_init(PrPart *p, double *x_local, hipStream_t s);
// gx_pagerank's single-rank plan of a graph: its pull matrix (A' when directed, which must be
// built) relabelled hub-first, column-sorted blocks, x buffers and the hub-first perm.
int pr_single_plan(gx_graph *g, PrPart **out);
// Rows of a huge graph's sorted block (gx_pr_sorted.hip kMaxBlockRows) and its entries.
constexpr int kPlanBlockRows = 16320;
constexpr int64_t kPlanBlockNnz = 32 << 20;

// gx_pagerank_multi's block partition (pr_partition.block_relabel restated): the hub-first
// order cut into the single-GPU plan's blocks, dealt whole to the devices largest first (LPT);
// per device its hub-first positions in order, per hub-first position its exchange slot
// (owner * chunk + local row).
struct MultiBlocks {
    std::vector<std::vector<int32_t>> pos;
    std::vector<int32_t> slot;
    uint64_t chunk = 0;
    std::vector<int32_t> order, perm;   // the host hub-first order: position -> vertex, vertex -> position
};
int pr_multi_blocks(const gx_csr *A, int directed, int ndev, MultiBlocks *out);
// The interleaved partition in the same form: hub-first position h to rank h % ndev as its
// local row h / ndev (pr_partition.interleaved_relabel).
int pr_multi_interleave(const gx_csr *A, int ndev, MultiBlocks *out);

// gx_pagerank_multi's plan of device d of ndev from its copy of the graph (A' built when
// directed): hub-first positions d, d + ndev, ... as rows (or mb's blocks), columns in the
// exchange layout.
int pr_multi_plan(gx_graph *g, int ndev, int d, uint64_t chunk, double damping, const MultiBlocks *mb,
                  PrPart **out);
// A rank's plan from its local pull rows (h_rp from 0) with columns already in the exchange
// layout (ci), the out-degree of each row's vertex, and its live prefix (gx_pr_part_create_live).
// force_huge: plan with the whole graph's block cut (a rank of a block partition).
int pr_part_build(gx_ctx *ctx, uint64_t n_global, int nranks, int rank, uint64_t chunk, uint64_t live,
                  const std::vector<int64_t> &h_rp, const std::vector<int32_t> &ci, const std::vector<int32_t> &h_outdeg,
                  double damping, PrPart **out, bool force_huge = false);
// gx_pagerank_multi's partitioned upload: a rank's rows `rows` (vertex ids of A, an undirected
// graph's pull rows) picked from the host CSR A straight into the staging buffers (original
// column ids, narrowed and checked), renamed to the exchange layout by the plan's key pass
// through colmap (device, n entries: vertex -> owner * chunk + local row).
int pr_part_build_rows(gx_ctx *ctx, const gx_csr *A, int nranks, int rank, uint64_t chunk,
                       const std::vector<int32_t> &rows, const int32_t *colmap, double damping, bool force_huge,
                       PrPart **out);
int pr_step(PrPart *p, const double *x_full, double *x_local, double *rank_out, hipStream_t s);

}  // namespace gx
