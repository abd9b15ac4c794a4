// gx_device.h -- device-side internals of libgx (gfx950 / CDNA4, wave64).
//
// HBM layout of a graph (gx_graph):
//   A   : out-edge CSR as stored in the .grb (rows = sources), int64 row pointers,
//         int32 column indices (n < 2^31), optional fp64 weights.
//   AT  : in-edge CSR (A transposed), built on the device by a radix sort when a
//         directed algorithm needs in-edges (PR pull, CDLP in-labels, BFS bottom-up).
//   S   : undirected closure A U A' without self-loops, sorted rows, one flag byte per
//         entry (bit0: v->u stored in A, bit1: u->v stored in A); built for LCC.
// Column-index arrays are allocated with 16 bytes of slack so int4 loads that start at
// an aligned-down address and run past the last entry stay inside the allocation.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <thread>
#include <memory>
#include <string>
#include <vector>

#include "gx_internal.h"

#define GX_HIP_TRY(expr)                                                              \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess)                                                         \
            return ::gx::fail(GX_DEVICE_ERROR, std::string(#expr " failed: ") +       \
                                                   hipGetErrorString(_e));            \
    } while (0)

#define GX_TRY(expr)                  \
    do {                              \
        int _rc = (expr);             \
        if (_rc != GX_SUCCESS) return _rc; \
    } while (0)

namespace gx {

constexpr int kWave = 64;

struct PrPart;

// While set (this thread), device frees are deferred into the list: a hipFree waits for the
// whole device, so a plan's temporaries freed while the columns upload on another stream
// (gx_pagerank_csr) waited for the queued copies -- SYN-8_5's fused plan spent 21 ms there.
inline thread_local std::vector<void *> *g_deferred_frees = nullptr;

// Drops the cached gx_*_multi cliques that include ctx (gx_comm.hip); gx_free calls it first.
void forget_cliques(gx_ctx *ctx);

// RAII device allocation (hipMalloc / hipFree); size in elements of T.
template <typename T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) {
            if (g_deferred_frees) g_deferred_frees->push_back(p);
            else (void)hipFree(p);
        }
        p = nullptr;
        n = 0;
    }
    // `slack_bytes` extra zeroed bytes past the end (for over-reading vector loads)
    int alloc(size_t count, size_t slack_bytes = 0) {
        release();
        size_t bytes = count * sizeof(T) + slack_bytes;
        if (bytes == 0) bytes = 16;
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&p), bytes);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(GX_OUT_OF_MEMORY, std::string("hipMalloc(") + std::to_string(bytes) +
                                              ") failed: " + hipGetErrorString(e));
        }
        n = count;
        if (slack_bytes) {
            e = hipMemset(reinterpret_cast<char *>(p) + count * sizeof(T), 0, slack_bytes);
            if (e != hipSuccess) return fail(GX_DEVICE_ERROR, "hipMemset slack failed");
        }
        return GX_SUCCESS;
    }
};

// std::allocator whose value-less construct leaves the element uninitialised: a host array
// that is written in full next (row pointers filled by parallel copies or device downloads)
// is not zero-filled, page by page, on one thread first (13 ms for SYN-8_5's 67 MB).
template <typename T>
struct NoInitAlloc : std::allocator<T> {
    template <typename U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <typename U>
    NoInitAlloc(const NoInitAlloc<U> &) {}
    template <typename U>
    void construct(U *p) noexcept {
        ::new (static_cast<void *>(p)) U;
    }
    template <typename U, typename... Args>
    void construct(U *p, Args &&...args) {
        ::new (static_cast<void *>(p)) U(std::forward<Args>(args)...);
    }
};
using HostRowPtr = std::vector<int64_t, NoInitAlloc<int64_t>>;

struct DevCSR {
    uint64_t n = 0, nnz = 0;
    DBuf<int64_t> rp;         // n + 1
    DBuf<int32_t> ci;         // nnz (+16 B slack)
    DBuf<double> w;           // nnz or empty
    DBuf<uint8_t> flag;       // nnz or empty (closure only)
    HostRowPtr h_rp;            // host copy of the row pointers (row-block planning)
    bool built = false;
};

}  // namespace gx

struct gx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool timing = false;
    struct Pending {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;   // recycled by collect_timings
    std::map<std::string, std::pair<uint64_t, double>> stats;
    double last_device_ms = 0.0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string device_name;
    int num_cus = 0;
    // pinned staging for uploads and result hand-back (allocated by gx_init, outside the
    // Graphalytics processing time); several buffers so host work overlaps the DMA
    static constexpr size_t kStageBytes = 32u << 20;
    static constexpr int kStageBufs = 4;
    void *staging[kStageBufs] = {};
    hipEvent_t stage_ev[kStageBufs] = {};
    // the column upload's stream of gx_pagerank_csr (made by gx_init: creating a stream took
    // 10-30 ms inside the processing time)
    hipStream_t upload_stream = nullptr;
    // auxiliary streams for independent kernels of one step (fork/join by events), lazy
    hipStream_t aux[2] = {nullptr, nullptr};
    hipEvent_t fork_ev = nullptr, join_ev[2] = {nullptr, nullptr};
};

namespace gx {
int ensure_aux_streams(gx_ctx *ctx);
// The host copy of c's row pointers (c.h_rp), downloaded on first use: gx_graph_create keeps
// none, so a path that never plans from them (PageRank on an undirected graph) never pays
// for them.
int ensure_host_rp(gx_ctx *ctx, DevCSR &c);
// Device -> host copy of `count` elements through the context's pinned staging buffers, the
// conversion of each chunk (parallel, on the host) overlapping the next chunk's DMA.
enum class Xfer { Raw64, Raw32, Levels, Widen32 };   // 8 / 4 B as is; int32 level -> int64 (INF); int32 -> uint64
int download(gx_ctx *ctx, void *dst, const void *src_dev, uint64_t count, Xfer kind);
// Host -> device of `count` elements of `elem` bytes through the pinned staging buffers:
// fill(off, cnt, buf) writes elements [off, off + cnt) into buf (false: bad input, *bad set).
int upload_staged(gx_ctx *ctx, void *dst, uint64_t count, size_t elem,
                  const std::function<bool(uint64_t, uint64_t, void *)> &fill, bool *bad);
// SSSP edge layout: every row of A split into its light (w < delta) edges, then its heavy
// ones; built once per graph and delta by gx_sssp.
struct SsspLayout {
    double delta = 0.0;
    DBuf<int32_t> ci;
    DBuf<double> w;
    DBuf<int64_t> lend;   // end of the light part of row v (absolute entry index)
    int64_t n_active = 0; // vertices with at least one edge
    std::shared_ptr<void> work;   // gx_sssp's work buffers and captured step graph (gx_sssp.hip)
};
}  // namespace gx

namespace gx {
// An asynchronous column upload (gx_pagerank_csr, the executable's PageRank): a host thread
// narrows and copies A's columns chunk by chunk on a stream of its own; chunk c's copy is done
// once ev[c] fires, and `ready` counts the chunks whose copies (and events) are enqueued.  A
// consumer waits for `ready` on the host, then for ev[c] on its own stream, so its kernels on
// chunk c run while the later chunks are still crossing the host link.
struct UploadJob {
    hipStream_t us = nullptr;          // the context's upload stream (borrowed)
    std::vector<hipEvent_t> ev;
    std::vector<int64_t> end;          // entry index just past chunk c
    std::atomic<int> ready{0};
    std::atomic<int> failed{0};
    int rc = 0;
    std::string msg;
    std::thread th;
    int device = 0;
    DBuf<uint32_t> packed;             // 24-bit columns before k_unpack24 (freed with the job)
    ~UploadJob();
    int wait_chunk(int c);             // host: chunk c's copy is enqueued (GX_SUCCESS), or the job failed
    int join();                        // thread and stream finished; the job's error, if any
};
}  // namespace gx

struct gx_graph {
    gx_ctx *ctx = nullptr;
    uint64_t n = 0, nnz = 0;
    bool directed = false, weighted = false;
    gx::DevCSR A, AT, S;
    gx::DBuf<int32_t> outdeg;   // out-degree of every vertex (PR)
    gx::PrPart *pr = nullptr;   // cached single-rank PageRank plan
    double mean_w = -1.0;       // cached mean edge weight (SSSP bucket width), < 0 = not yet computed
    int bfs_calls = 0;          // BFS runs on this graph (a directed graph builds A^T from the second)
    int bfs_steps_hint = 0;     // device-driven level steps the last BFS took (gx_bfs first batch)
    gx::DBuf<int32_t> wcc_ids;  // Afforest's sampled vertices (+ one word: the giant root)
    int64_t wcc_ids_n = 0;
    int cdlp_calls = 0;         // CDLP runs (the relabelled copy is built from the second)
    gx::SsspLayout *sssp = nullptr;   // cached light/heavy edge layout
    std::shared_ptr<void> cdlp;       // gx_cdlp's tier lists and buffers (gx_cdlp.hip CdlpCache)
    std::shared_ptr<void> lcc;        // gx_lcc's orientation and work items (gx_lcc.hip LccCache)
    // Hub-first relabelled copy of an undirected graph (gx_runtime.hip hub_for): BFS, WCC and
    // SSSP run on it from their second call on the graph.  perm[v] = v's id in the copy, order
    // its inverse; on the copy, out_perm / out_order point at the parent's perm / order.
    std::shared_ptr<gx_graph> hub;
    gx::DBuf<int32_t> hub_perm, hub_order;
    std::vector<int32_t> h_hub_perm;
    const int32_t *out_perm = nullptr;
    const int32_t *out_order = nullptr;
    gx::DBuf<uint64_t> remap_tmp;         // on a copy: n words of scratch for the remap
    int64_t live = 0;                     // on a copy: vertices of degree > 0 (a prefix of its ids)
    bool rows_sorted = false;             // on a copy: every row sorted by (hub-first) column
    std::shared_ptr<gx::UploadJob> job;   // columns still arriving (gx_pagerank_csr), else null
    int sssp_calls = 0, wcc_calls = 0, hub_bfs_calls = 0;
};

namespace gx {

// Kernel timer: brackets one launch with hipEvents when ctx->timing is on.
struct KTimer {
    gx_ctx *ctx;
    const char *name;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    KTimer(gx_ctx *c, const char *nm, hipStream_t st) : ctx(c), name(nm), s(st) {
        if (ctx && ctx->timing) {
            a = take();
            b = take();
            (void)hipEventRecord(a, s);
        }
    }
    hipEvent_t take() {
        hipEvent_t e = nullptr;
        if (!ctx->event_pool.empty()) {
            e = ctx->event_pool.back();
            ctx->event_pool.pop_back();
        } else {
            (void)hipEventCreate(&e);
        }
        return e;
    }
    ~KTimer() {
        if (a) {
            (void)hipEventRecord(b, s);
            ctx->pending.push_back({name, a, b});
        }
    }
};

// The graph a call runs on: g itself, or its hub-first copy (built on demand and cached) when
// g is undirected and this is the algorithm's `calls`-th call with calls >= 2 (GX_HUB = 0 never,
// 1 from the second call (default), 2 from the first).  *src is renamed into the copy's ids.
int hub_for(gx_graph *g, int calls, gx_graph **out, uint64_t *src);
// The results to download: on a copy (g->out_perm set) buf scattered through out_order into
// the parent's vertex order (g->remap_tmp; elem = 4 or 8 bytes, n entries), else buf itself.
int remap_out(gx_graph *g, const void *buf, int elem, hipStream_t s, const void **res);

// Collect elapsed times of finished timed launches into ctx->stats.
int collect_timings(gx_ctx *ctx);

// Device work bracket for gx_last_device_ms.
int device_begin(gx_ctx *ctx);
int device_end(gx_ctx *ctx);

// Sort packed (row << 32 | col) keys (rows < n) in place (k1 = scratch of the same size)
// and build row pointers / column indices from them.  rp must hold n + 1 entries and ci
// m entries; keys end up sorted in *keys.
// Radix sort of (u64 key, u32 value) pairs on bits [0, end_bit) of the key, into k_out / v_out.
int sort_pairs_u64_u32(uint64_t *k_in, uint64_t *k_out, uint32_t *v_in, uint32_t *v_out, size_t m, int end_bit,
                       hipStream_t s);
// Radix sorts / scan (rocPRIM) enqueued on stream s, not synchronised; their temporary storage
// is one per device, ordered across streams by an event (gx_runtime.hip rocprim_tmp).
int sort_keys_u64(uint64_t *k_in, uint64_t *k_out, size_t m, int end_bit, hipStream_t s);
int sort_pairs_u32_u16(uint32_t *k_in, uint32_t *k_out, uint16_t *v_in, uint16_t *v_out, size_t m, int end_bit,
                       hipStream_t s);
int sort_pairs_u64_u16(uint64_t *k_in, uint64_t *k_out, uint16_t *v_in, uint16_t *v_out, size_t m, int end_bit,
                       hipStream_t s);
// stable descending sort of (key, value) pairs, all 32 key bits
int sort_pairs_desc_u32_i32(uint32_t *k_in, uint32_t *k_out, int32_t *v_in, int32_t *v_out, size_t m, hipStream_t s);
int scan_exclusive_i64(const int64_t *in, int64_t *out, size_t m, hipStream_t s);
// every row of (rp, ci_in) sorted by column into ci_out, weights (optional) alongside
// (rocPRIM segmented radix sort on bits [0, end_bit)); n, nnz < 2^32
int sort_rows_i32(const int64_t *rp, int64_t n, int64_t nnz, int32_t *ci_in, int32_t *ci_out, double *w_in,
                  double *w_out, int end_bit, hipStream_t s);
// grow-only device scratch of the current device, kept between calls (gx_runtime.hip)
int plan_scratch(size_t bytes, void **p);
int sort_keys_to_csr(DBuf<uint64_t> &keys, DBuf<uint64_t> &scratch, size_t m, int64_t n, int64_t *rp,
                     int32_t *ci, hipStream_t s);

// GX_OUT_OF_MEMORY when a split SSSP run stopped on a full settled list (gx_sssp_split.hip);
// synchronises s.
int sssp_split_check(gx_sssp_split *p, hipStream_t s);

// gx_pagerank_csr's graph: row pointers uploaded, the columns arriving through g->job (no
// weights); every other use of g must g->job->join() first.
int graph_create_async(gx_ctx *ctx, const gx_csr *A, int directed, gx_graph **out);

// Lazily build the transposed / closure CSR of a graph on the device.
int ensure_transpose(gx_graph *g);
int ensure_closure(gx_graph *g);
int ensure_outdeg(gx_graph *g);

// Launch-error check after hipLaunchKernelGGL.
inline int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(GX_DEVICE_ERROR, std::string("launch of ") + what + " failed: " +
                                         hipGetErrorString(e));
    return GX_SUCCESS;
}

inline unsigned grid_for(uint64_t work, int block, unsigned cap = 65535u * 4u) {
    uint64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---- device helpers -----------------------------------------------------------------

// Last row r with rp[r] <= e (rows with rp[r] == rp[r+1] are skipped): upper_bound - 1.
__device__ __forceinline__ int64_t row_of_edge(const int64_t *rp, int64_t nrows, int64_t e) {
    int64_t lo = 0, hi = nrows;   // invariant: rp[lo] <= e < rp[hi]
    while (hi - lo > 1) {
        int64_t mid = (lo + hi) >> 1;
        if (rp[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Raise a shared "something changed" flag.  Thousands of waves writing one word serialise
// on one L2 channel (~11 ns per access, MI355X_MICROARCH.md "dequeue"); only a wave that
// still reads it clear writes it (idempotent, so the race is harmless).
__device__ __forceinline__ void raise_flag(int *flag) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The same flag spread over `shards` words kFlagStride apart (one per 128-byte line): the
// raise of workgroup b goes to word b % shards, so ~16 K raising waves of a thread-per-vertex
// kernel hit kFlagShards lines instead of one (one word: ~150 us of serialised checks for
// CDLP's first iteration on SYN-7_5).  Readers OR the words.
constexpr int kFlagShards = 64;
constexpr int kFlagStride = 32;

__device__ __forceinline__ void raise_flag_sharded(int *flags, int shards) {
    raise_flag(flags + (int)(blockIdx.x % (unsigned)shards) * kFlagStride);
}

// ---- 64-entry slabs of a CSR (one wave per slab, lane = entry) ----
// srow[sl] = the row holding entry sl*64, srow[nslabs] = n - 1 (gx_runtime.hip).
int slab_rows(const int64_t *rp, int64_t n, int64_t nslabs, int64_t *srow, hipStream_t s);

// Row of entry ee (inside slab sl): the slab's rows lie in [srow[sl], srow[sl+1]]; when that
// range is at most 64 rows each lane finds its row by a 6-step shuffle search, else by its
// own binary search.  Every lane of the wave must call it (shuffles).
__device__ __forceinline__ int64_t slab_row_of(const int64_t *__restrict__ rp, const int64_t *__restrict__ srow,
                                               int64_t n, int64_t sl, int64_t ee, int lane) {
    const int64_t r0 = srow[sl], r1 = srow[sl + 1];
    if (r1 - r0 < kWave) {
        const int64_t rpk = rp[min(r0 + 1 + lane, n)];
        int o = 0;
#pragma unroll
        for (int step = kWave / 2; step > 0; step >>= 1)
            if (__shfl(rpk, o + step - 1, kWave) <= ee) o += step;
        return r0 + o;
    }
    int64_t lo = r0, hi = r1 + 1;   // rp[lo] <= ee < rp[hi]
    if (hi > n) hi = n;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (rp[mid] <= ee) lo = mid;
        else hi = mid;
    }
    return lo;
}

typedef int gx_v4i __attribute__((ext_vector_type(4)));
// four dwords loaded by one 16-B load from an address that is only 4-B aligned (a CSR offset):
// the type says so, and gfx950 still emits one global_load_dwordx4
typedef uint32_t gx_u32x4 __attribute__((ext_vector_type(4), aligned(4)));

// 16-byte non-temporal load (read-once streams: keep L2 for the gathered vectors).
__device__ __forceinline__ int4 load_nt(const int4 *p) {
    const gx_v4i v = __builtin_nontemporal_load(reinterpret_cast<const gx_v4i *>(p));
    return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace gx

// Module warm-up.  HIP loads a translation unit's code object on the first launch of one of
// its kernels (about 20 ms for gx_runtime.hip with its rocprim sorts): gx_init launches one
// empty kernel per .hip file, so that cost stays out of an algorithm's processing time, like
// the fill/copy warm-up there.
#define GX_MODULE_WARMER(name)                                                           \
    namespace gx {                                                                       \
    __global__ void warm_kernel_##name() {}                                              \
    hipError_t warm_##name(hipStream_t s) {                                              \
        hipLaunchKernelGGL(warm_kernel_##name, dim3(1), dim3(1), 0, s);                 \
        return hipGetLastError();                                                        \
    }                                                                                    \
    }
namespace gx {
hipError_t warm_bfs(hipStream_t s);
hipError_t warm_cdlp(hipStream_t s);
hipError_t warm_lcc(hipStream_t s);
hipError_t warm_ops(hipStream_t s);
hipError_t warm_part(hipStream_t s);
hipError_t warm_sssp_split(hipStream_t s);
hipError_t warm_pr(hipStream_t s);
hipError_t warm_pr_sorted(hipStream_t s);
hipError_t warm_runtime(hipStream_t s);
hipError_t warm_sssp(hipStream_t s);
hipError_t warm_wcc(hipStream_t s);
}  // namespace gx
