// gx_runtime.hip -- context, device graph upload and on-device graph transforms.
//
// Replaces LAGraph_Init / LAGraph_New / LAGraph_Cached_AT / the A LOR A' symmetrisation
// the reference runs inside SuiteSparse (pr.cpp:58-60, wcc.cpp:53-55, lcc.cpp:68).
// The transforms run on the device with rocPRIM radix sorts over packed 64-bit
// (row << 32 | col) keys, so their rows come out sorted by column.
#include <cstring>
#include <memory>
#include <cstdlib>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstring>

#include "gx_device.h"
#include "gx_pr.h"

using namespace gx;

// ----------------------------------------------------------------------------- ctx

extern "C" int gx_device_count(int *count) {
    if (!count) return fail(GX_NULL_POINTER, "gx_device_count: null");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *count = c;
    return GX_SUCCESS;
}

extern "C" int gx_init(int device, gx_ctx **out) {
    if (!out) return fail(GX_NULL_POINTER, "gx_init: null ctx");
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0)
        return fail(GX_DEVICE_ERROR, "gx_init: no HIP device visible (libgx has no CPU fallback)");
    if (device < 0 || device >= count) return fail(GX_INVALID_VALUE, "gx_init: bad device index");
    GX_HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    GX_HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(GX_DEVICE_ERROR, std::string("gx_init: libgx is built for gfx950, device is ") +
                                         prop.gcnArchName);
    gx_ctx *ctx = new gx_ctx();
    ctx->device = device;
    // the marketing name comes from libdrm's amdgpu.ids, absent on some images: keep the arch
    ctx->device_name = prop.name[0] ? std::string(prop.name) + " (" + prop.gcnArchName + ")"
                                    : std::string(prop.gcnArchName);
    ctx->num_cus = prop.multiProcessorCount;
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->upload_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev0);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev1);
    // two staging buffers now; GX_UPLOAD_BUFS > 2 adds the others on first use (ADVICE r04:
    // 64 MB of idle pinned memory per context otherwise)
    for (int i = 0; i < gx_ctx::kStageBufs && e == hipSuccess; i++) {
        if (i < 2) e = hipHostMalloc(&ctx->staging[i], gx_ctx::kStageBytes);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->stage_ev[i], hipEventDisableTiming);
    }
    // warm the runtime's fill and copy paths (first use initialises them): outside the
    // processing time, like the reference's LAGraph_Init
    if (e == hipSuccess) {
        void *d = nullptr;
        e = hipMalloc(&d, 1 << 20);
        if (e == hipSuccess) e = hipMemsetAsync(d, 0, 1 << 20, ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(d, ctx->staging[0], 1 << 20, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(ctx->staging[1], d, 1 << 20, hipMemcpyDeviceToHost, ctx->stream);
        // load every kernel module now (see GX_MODULE_WARMER)
        for (auto warm : {warm_bfs, warm_cdlp, warm_lcc, warm_ops, warm_part, warm_pr, warm_pr_sorted,
                          warm_runtime, warm_sssp, warm_sssp_split, warm_wcc})
            if (e == hipSuccess) e = warm(ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (d) (void)hipFree(d);
    }
    if (e != hipSuccess) {
        gx_free(ctx);
        return fail(GX_DEVICE_ERROR, std::string("gx_init: ") + hipGetErrorString(e));
    }
    *out = ctx;
    return GX_SUCCESS;
}

extern "C" int gx_free(gx_ctx *ctx) {
    if (!ctx) return GX_SUCCESS;
    forget_cliques(ctx);
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto &p : ctx->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->upload_stream) {
        (void)hipStreamSynchronize(ctx->upload_stream);
        (void)hipStreamDestroy(ctx->upload_stream);
    }
    for (int i = 0; i < 2; i++) {
        if (ctx->aux[i]) (void)hipStreamDestroy(ctx->aux[i]);
        if (ctx->join_ev[i]) (void)hipEventDestroy(ctx->join_ev[i]);
    }
    if (ctx->fork_ev) (void)hipEventDestroy(ctx->fork_ev);
    for (int i = 0; i < gx_ctx::kStageBufs; i++) {
        if (ctx->stage_ev[i]) (void)hipEventDestroy(ctx->stage_ev[i]);
        if (ctx->staging[i]) (void)hipHostFree(ctx->staging[i]);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return GX_SUCCESS;
}

extern "C" int gx_device_info(gx_ctx *ctx, char *name, size_t name_len, int *num_cus) {
    if (!ctx) return fail(GX_NULL_POINTER, "gx_device_info: null ctx");
    if (name && name_len) {
        std::strncpy(name, ctx->device_name.c_str(), name_len - 1);
        name[name_len - 1] = '\0';
    }
    if (num_cus) *num_cus = ctx->num_cus;
    return GX_SUCCESS;
}

// -------------------------------------------------------------------------- timing

namespace gx {

int collect_timings(gx_ctx *ctx) {
    if (ctx->pending.empty()) return GX_SUCCESS;
    GX_HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (auto &p : ctx->pending) {
        (void)hipEventSynchronize(p.b);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto &s = ctx->stats[p.name];
            s.first += 1;
            s.second += ms;
        }
        ctx->event_pool.push_back(p.a);
        ctx->event_pool.push_back(p.b);
    }
    ctx->pending.clear();
    return GX_SUCCESS;
}

// each row scatters its own slab starts: no per-slab binary search
__global__ void k_slab_rows(const int64_t *__restrict__ rp, int64_t n, int64_t nslabs, int64_t *srow) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = rp[v], e = rp[v + 1];
        for (int64_t sl = (b + kWave - 1) / kWave; sl * kWave < e; sl++) srow[sl] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) srow[nslabs] = n > 0 ? n - 1 : 0;
}

int slab_rows(const int64_t *rp, int64_t n, int64_t nslabs, int64_t *srow, hipStream_t s) {
    hipLaunchKernelGGL(k_slab_rows, dim3(grid_for((uint64_t)std::max<int64_t>(n, 1), 256, 8192)), dim3(256), 0, s, rp,
                       n, nslabs, srow);
    return check_launch("k_slab_rows");
}

int download(gx_ctx *ctx, void *dst, const void *src_dev, uint64_t count, Xfer kind) {
    const size_t elem = kind == Xfer::Raw64 ? 8 : 4;   // Raw32: 4 as well
    const uint64_t chunk = gx_ctx::kStageBytes / elem;
    hipStream_t s = ctx->stream;
    auto convert = [&](uint64_t off, uint64_t cnt, const void *buf) {
        switch (kind) {
            case Xfer::Raw64:
                host_copy(static_cast<char *>(dst) + off * 8, buf, cnt * 8);
                break;
            case Xfer::Raw32:
                host_copy(static_cast<char *>(dst) + off * 4, buf, cnt * 4);
                break;
            case Xfer::Levels:
                host_levels(static_cast<const int32_t *>(buf), cnt, static_cast<int64_t *>(dst) + off);
                break;
            case Xfer::Widen32:
                host_widen(static_cast<const int32_t *>(buf), cnt, static_cast<uint64_t *>(dst) + off);
                break;
        }
    };
    uint64_t prev_off = 0, prev_cnt = 0;
    int c = 0;
    for (uint64_t off = 0; off < count; off += chunk, c++) {
        const int b = c & 1;
        const uint64_t cnt = std::min<uint64_t>(chunk, count - off);
        GX_HIP_TRY(hipMemcpyAsync(ctx->staging[b], static_cast<const char *>(src_dev) + off * elem, cnt * elem,
                                  hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipEventRecord(ctx->stage_ev[b], s));
        if (c >= 1) {   // convert the previous chunk while this one copies
            GX_HIP_TRY(hipEventSynchronize(ctx->stage_ev[b ^ 1]));
            convert(prev_off, prev_cnt, ctx->staging[b ^ 1]);
        }
        prev_off = off;
        prev_cnt = cnt;
    }
    if (c >= 1) {
        GX_HIP_TRY(hipEventSynchronize(ctx->stage_ev[(c - 1) & 1]));
        convert(prev_off, prev_cnt, ctx->staging[(c - 1) & 1]);
    }
    return GX_SUCCESS;
}

int ensure_host_rp(gx_ctx *ctx, DevCSR &c) {
    if (c.h_rp.size() == c.n + 1) return GX_SUCCESS;
    HostRowPtr h(c.n + 1);
    GX_TRY(download(ctx, h.data(), c.rp.p, c.n + 1, Xfer::Raw64));
    c.h_rp.swap(h);
    return GX_SUCCESS;
}

int ensure_aux_streams(gx_ctx *ctx) {
    if (ctx->aux[0]) return GX_SUCCESS;
    for (int i = 0; i < 2; i++) {
        GX_HIP_TRY(hipStreamCreateWithFlags(&ctx->aux[i], hipStreamNonBlocking));
        GX_HIP_TRY(hipEventCreateWithFlags(&ctx->join_ev[i], hipEventDisableTiming));
    }
    GX_HIP_TRY(hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
    return GX_SUCCESS;
}

int device_begin(gx_ctx *ctx) {
    GX_HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    return GX_SUCCESS;
}

int device_end(gx_ctx *ctx) {
    GX_HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    GX_HIP_TRY(hipEventSynchronize(ctx->ev1));
    float ms = 0.f;
    GX_HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_device_ms = ms;
    return GX_SUCCESS;
}

}  // namespace gx

extern "C" int gx_set_kernel_timing(gx_ctx *ctx, int enable) {
    if (!ctx) return fail(GX_NULL_POINTER, "null ctx");
    ctx->timing = enable != 0;
    return GX_SUCCESS;
}

extern "C" int gx_kernel_stats(gx_ctx *ctx, const char *kernel, uint64_t *launches,
                               double *total_ms) {
    if (!ctx || !kernel) return fail(GX_NULL_POINTER, "null argument");
    GX_TRY(collect_timings(ctx));
    auto it = ctx->stats.find(kernel);
    if (launches) *launches = it == ctx->stats.end() ? 0 : it->second.first;
    if (total_ms) *total_ms = it == ctx->stats.end() ? 0.0 : it->second.second;
    return GX_SUCCESS;
}

extern "C" int gx_reset_kernel_stats(gx_ctx *ctx) {
    if (!ctx) return fail(GX_NULL_POINTER, "null ctx");
    GX_TRY(collect_timings(ctx));
    ctx->stats.clear();
    return GX_SUCCESS;
}

extern "C" int gx_last_device_ms(gx_ctx *ctx, double *ms) {
    if (!ctx || !ms) return fail(GX_NULL_POINTER, "null argument");
    *ms = ctx->last_device_ms;
    return GX_SUCCESS;
}

// --------------------------------------------------------------------------- graph

namespace gx {
namespace {

// Host -> device in chunks through the context's two pinned staging buffers: host threads
// fill one (conversion / validation) while the DMA engine drains the other.  Replaces one
// single-threaded conversion pass plus a pageable copy, which dominated the Graphalytics
// processing time of the small-iteration algorithms.
// fill(first, count, staging) writes `count` elements of `elem` bytes; false = bad input.
// On stream `us` (null: the context's); after(c) runs once chunk c's copy is enqueued; `sync`
// waits for the last copy.
struct NoAfter {
    int operator()(int) const { return GX_SUCCESS; }
};
// Entries per staging chunk: a multiple of `align`.  The packed 24-bit columns use kPackAlign =
// 64: a chunk must start on a 48-byte boundary (16 entries) for k_unpack24, and on a whole
// 64-entry slab for the source-side key pass of gx_pagerank_csr (k_scatter_keys covers slabs
// [e0/64, ceil(e1/64)), so a boundary inside a slab would read the next chunk before it lands).
constexpr uint64_t kPackAlign = 64;
uint64_t stage_chunk(size_t elem, uint64_t align = 1) { return gx_ctx::kStageBytes / elem / align * align; }

template <class Fill, class After = NoAfter>
int upload(gx_ctx *ctx, char *dst, uint64_t count, size_t elem, Fill fill, bool *bad, hipStream_t us = nullptr,
           After after = After(), bool sync = true, uint64_t align = 1) {
    const uint64_t chunk = stage_chunk(elem, align);
    hipStream_t s = us ? us : ctx->stream;
    *bad = false;
    int c = 0;
    static const bool times = [] {
        const char *e = std::getenv("GX_PLAN_TIMES");
        return e && std::atoi(e) != 0;
    }();
    auto env_int = [](const char *name, int def) {
        const char *e = std::getenv(name);
        return e ? std::atoi(e) : def;
    };
    const int nbuf = std::min(std::max(env_int("GX_UPLOAD_BUFS", 2), 2), gx_ctx::kStageBufs);
    for (int b = 2; b < nbuf; b++)
        if (!ctx->staging[b]) GX_HIP_TRY(hipHostMalloc(&ctx->staging[b], gx_ctx::kStageBytes));
    const int thr = env_int("GX_UPLOAD_THREADS", 0), saved_thr = host_threads();
    if (thr > 0) host_set_threads(thr);
    struct Restore {
        int t;
        bool on;
        ~Restore() {
            if (on) host_set_threads(t);
        }
    } restore{saved_thr, thr > 0};
    using clk = std::chrono::steady_clock;
    double t_wait = 0, t_fill = 0;
    const auto t0 = clk::now();
    for (uint64_t off = 0; off < count; off += chunk, c++) {
        const int b = c % nbuf;
        const uint64_t cnt = std::min<uint64_t>(chunk, count - off);
        auto ta = clk::now();
        if (c >= nbuf) GX_HIP_TRY(hipEventSynchronize(ctx->stage_ev[b]));   // its previous copy is done
        auto tb = clk::now();
        if (!fill(off, cnt, ctx->staging[b])) {
            *bad = true;
            break;
        }
        auto tc = clk::now();
        t_wait += std::chrono::duration<double, std::milli>(tb - ta).count();
        t_fill += std::chrono::duration<double, std::milli>(tc - tb).count();
        // (whole 4-byte words: a packed chunk's last entries may end inside one)
        GX_HIP_TRY(hipMemcpyAsync(dst + off * elem, ctx->staging[b], (cnt * elem + 3) / 4 * 4, hipMemcpyHostToDevice, s));
        GX_HIP_TRY(hipEventRecord(ctx->stage_ev[b], s));
        GX_TRY(after(c));
    }
    if (sync) GX_HIP_TRY(hipStreamSynchronize(s));
    if (times)
        std::fprintf(stderr, "[upload] %llu x %zu B, %d buffers, %d threads: %8.2f ms (host fill %.2f ms, copy wait %.2f ms)\n",
                     (unsigned long long)count, elem, nbuf, host_threads(),
                     std::chrono::duration<double, std::milli>(clk::now() - t0).count(), t_fill, t_wait);
    return GX_SUCCESS;
}

}  // namespace
}  // namespace gx

namespace gx {
namespace {

// Packed 24-bit columns (host_pack24) -> int32, entries [e0, e1): a thread per 4 entries, three
// aligned words in (e0 is a multiple of 16), four out.
__global__ __launch_bounds__(256) void k_unpack24(const uint32_t *__restrict__ words, int64_t e0, int64_t e1,
                                                  int32_t *__restrict__ out) {
    const int64_t ng = (e1 - e0 + 3) / 4;
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ng; g += (int64_t)gridDim.x * 256) {
        const int64_t e = e0 + 4 * g;
        const uint32_t *w = words + 3 * (e / 4);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
        const int32_t c0 = (int32_t)(w0 & 0xffffffu), c1 = (int32_t)((w0 >> 24) | ((w1 & 0xffffu) << 8)),
                      c2 = (int32_t)((w1 >> 16) | ((w2 & 0xffu) << 16)), c3 = (int32_t)(w2 >> 8);
        if (e + 3 < e1) {
            *reinterpret_cast<int4 *>(out + e) = make_int4(c0, c1, c2, c3);
        } else {
            out[e] = c0;
            if (e + 1 < e1) out[e + 1] = c1;
            if (e + 2 < e1) out[e + 2] = c2;
        }
    }
}

// GX_UPLOAD_PACK=0 keeps 4-byte columns; else columns of a graph with fewer than 2^24 vertices
// travel as 3 bytes (a quarter fewer bytes over the host link, which bounds the upload: SYN-8_5
// 2.51 GB at ~52 GB/s)
bool pack_columns(uint64_t n) {
    const char *e = std::getenv("GX_UPLOAD_PACK");
    return n <= (1ull << 24) && !(e && std::atoi(e) == 0);
}

// The columns into dst (int32 on the device) on stream s: packed (pack_columns) through
// `packed` (>= ceil(3 nnz / 4) + 4 words) and widened chunk by chunk, or narrowed on the host.
// after(c) runs once chunk c is on the device as int32 (in stream order).
template <class After>
int upload_columns(gx_ctx *ctx, const uint64_t *cols, uint64_t nnz, uint64_t n, int32_t *dst, uint32_t *packed,
                   bool nt, bool *bad, hipStream_t s, After after, bool sync) {
    if (!packed)
        return upload(ctx, reinterpret_cast<char *>(dst), nnz, 4,
                      [&](uint64_t off, uint64_t cnt, void *buf) {
                          return host_narrow(cols + off, cnt, n, static_cast<int32_t *>(buf), nt);
                      }, bad, s, after, sync);
    const uint64_t chunk = stage_chunk(3, kPackAlign);
    return upload(ctx, reinterpret_cast<char *>(packed), nnz, 3,
                  [&](uint64_t off, uint64_t cnt, void *buf) {
                      return host_pack24(cols + off, cnt, n, static_cast<uint32_t *>(buf));
                  }, bad, s,
                  [&](int c) -> int {
                      const uint64_t e0 = (uint64_t)c * chunk, e1 = std::min(nnz, e0 + chunk);
                      hipLaunchKernelGGL(k_unpack24, dim3(grid_for((e1 - e0 + 3) / 4, 256, 8192)), dim3(256), 0, s,
                                         packed, (int64_t)e0, (int64_t)e1, dst);
                      GX_TRY(check_launch("k_unpack24"));
                      return after(c);
                  }, sync, kPackAlign);
}

}  // namespace

int upload_staged(gx_ctx *ctx, void *dst, uint64_t count, size_t elem,
                  const std::function<bool(uint64_t, uint64_t, void *)> &fill, bool *bad) {
    return upload(ctx, static_cast<char *>(dst), count, elem, fill, bad);
}

UploadJob::~UploadJob() {
    if (th.joinable()) th.join();
    (void)hipSetDevice(device);
    if (us) (void)hipStreamSynchronize(us);
    for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
}

int UploadJob::wait_chunk(int c) {
    while (ready.load(std::memory_order_acquire) <= c) {
        if (failed.load(std::memory_order_acquire)) return join();
        std::this_thread::yield();
    }
    return GX_SUCCESS;
}

int UploadJob::join() {
    if (th.joinable()) th.join();
    if (us) GX_HIP_TRY(hipStreamSynchronize(us));
    if (rc != GX_SUCCESS) return fail(rc, msg);
    return GX_SUCCESS;
}

// The graph of gx_pagerank_csr: row pointers uploaded (and the context's stream drained), the
// columns on their way (g->job); no weights (PageRank does not read them).
int graph_create_async(gx_ctx *ctx, const gx_csr *A, int directed, gx_graph **out) {
    *out = nullptr;
    if (!A->rowptr || (A->nnz && !A->colidx)) return fail(GX_NULL_POINTER, "gx_pagerank_csr: null CSR arrays");
    if (A->n >= (1ull << 31) - 64) return fail(GX_NOT_IMPLEMENTED, "gx_pagerank_csr: n >= 2^31 needs 64-bit column indices");
    if (A->rowptr[0] != 0 || A->rowptr[A->n] != A->nnz)
        return fail(GX_INVALID_VALUE, "gx_pagerank_csr: inconsistent row pointers");
    if (!host_monotone(A->rowptr, A->n)) return fail(GX_INVALID_VALUE, "gx_pagerank_csr: row pointers not monotone");
    GX_HIP_TRY(hipSetDevice(ctx->device));
    PlanClock clk("graph_create_async", ctx->stream);
    const uint64_t n = A->n, nnz = A->nnz;
    std::unique_ptr<gx_graph> g(new gx_graph());
    g->ctx = ctx;
    g->n = n;
    g->nnz = nnz;
    g->directed = directed != 0;
    g->weighted = false;
    g->A.n = n;
    g->A.nnz = nnz;
    GX_TRY(g->A.rp.alloc(n + 1));
    GX_TRY(g->A.ci.alloc(nnz, 16));
    bool bad = false;
    GX_TRY(upload(ctx, reinterpret_cast<char *>(g->A.rp.p), n + 1, 8,
                  [&](uint64_t off, uint64_t cnt, void *buf) {
                      host_copy(buf, reinterpret_cast<const int64_t *>(A->rowptr) + off, cnt * 8);
                      return true;
                  }, &bad));
    clk.mark("buffers + row pointers");
    auto job = std::make_shared<UploadJob>();
    job->device = ctx->device;
    job->us = ctx->upload_stream;
    // the packed buffer and the chunk events are made by the upload thread (creating ~75 events
    // and a 1.9 GB buffer here cost the calling thread ~12 ms before its plan could start)
    const bool pack = pack_columns(n);
    const uint64_t chunk = pack ? stage_chunk(3, kPackAlign) : stage_chunk(4, kPackAlign);
    for (uint64_t off = 0; off < nnz; off += chunk) {
        job->ev.push_back(nullptr);
        job->end.push_back((int64_t)std::min(nnz, off + chunk));
    }
    // the key pass reads whole 64-entry slabs up to each chunk end: every end but the last must
    // be slab-aligned
    for (size_t c = 0; c + 1 < job->end.size(); c++)
        if (job->end[c] % 64) return fail(GX_PANIC, "graph_create_async: upload chunk not 64-entry aligned");
    const char *nt_env = std::getenv("GX_UPLOAD_NT");
    const bool nt = !nt_env || std::atoi(nt_env) != 0;
    UploadJob *j = job.get();
    int32_t *dst = g->A.ci.p;
    const uint64_t *cols = A->colidx;
    // half the caller's host threads (GX_UPLOAD_THREADS overrides): the calling thread plans
    // meanwhile, and the host link, not the narrowing, bounds the upload (SYN-8_5: 28 ms of fill
    // with 15 threads in 48 ms of copies); with every thread narrowing, the plan's host steps and
    // small copies ran 10x slower
    const int nthreads = std::max(1, host_threads() / 2);
    j->th = std::thread([ctx, j, dst, cols, n, nnz, nt, nthreads, pack] {
        host_set_threads(nthreads);
        bool bad2 = false;
        int rc = hipSetDevice(ctx->device) == hipSuccess ? GX_SUCCESS : fail(GX_DEVICE_ERROR, "hipSetDevice");
        if (rc == GX_SUCCESS && pack) rc = j->packed.alloc((3 * nnz + 3) / 4 + 4);
        if (rc == GX_SUCCESS)
            rc = upload_columns(ctx, cols, nnz, n, dst, pack ? j->packed.p : nullptr, nt, &bad2, j->us,
                                [&](int c) -> int {
                                    GX_HIP_TRY(hipEventCreateWithFlags(&j->ev[c], hipEventDisableTiming));
                                    GX_HIP_TRY(hipEventRecord(j->ev[c], j->us));
                                    j->ready.store(c + 1, std::memory_order_release);
                                    return GX_SUCCESS;
                                },
                                false);
        if (rc == GX_SUCCESS && bad2) rc = fail(GX_INVALID_INDEX, "gx_pagerank_csr: column out of range");
        if (rc != GX_SUCCESS) {
            j->rc = rc;
            j->msg = gx_last_error();
            j->failed.store(1, std::memory_order_release);
        }
    });
    g->A.built = true;
    g->job = job;
    *out = g.release();
    return GX_SUCCESS;
}

}  // namespace gx

extern "C" int gx_graph_create(gx_ctx *ctx, const gx_csr *A, int directed, gx_graph **out) {
    if (!ctx || !A || !out) return fail(GX_NULL_POINTER, "gx_graph_create: null argument");
    *out = nullptr;
    if (!A->rowptr || (A->nnz && !A->colidx))
        return fail(GX_NULL_POINTER, "gx_graph_create: null CSR arrays");
    if (A->n >= (1ull << 31) - 64)
        return fail(GX_NOT_IMPLEMENTED, "gx_graph_create: n >= 2^31 needs 64-bit column indices");
    if (A->rowptr[0] != 0 || A->rowptr[A->n] != A->nnz)
        return fail(GX_INVALID_VALUE, "gx_graph_create: inconsistent row pointers");
    PlanClock clk("graph_create", ctx->stream);
    if (!host_monotone(A->rowptr, A->n)) return fail(GX_INVALID_VALUE, "gx_graph_create: row pointers not monotone");
    GX_HIP_TRY(hipSetDevice(ctx->device));
    clk.mark("checks");
    const uint64_t n = A->n, nnz = A->nnz;
    std::unique_ptr<gx_graph> g(new gx_graph());
    g->ctx = ctx;
    g->n = n;
    g->nnz = nnz;
    g->directed = directed != 0;
    g->weighted = A->vals != nullptr;
    g->A.n = n;
    g->A.nnz = nnz;
    GX_TRY(g->A.rp.alloc(n + 1));
    GX_TRY(g->A.ci.alloc(nnz, 16));
    if (g->weighted) GX_TRY(g->A.w.alloc(nnz));
    clk.mark("device buffers");
    bool bad = false;
    const char *nt_env = std::getenv("GX_UPLOAD_NT");
    const bool nt = !nt_env || std::atoi(nt_env) != 0;   // streaming stores unless GX_UPLOAD_NT=0
    GX_TRY(upload(ctx, reinterpret_cast<char *>(g->A.rp.p), n + 1, 8,
                  [&](uint64_t off, uint64_t cnt, void *buf) {
                      host_copy(buf, reinterpret_cast<const int64_t *>(A->rowptr) + off, cnt * 8);
                      return true;
                  }, &bad));
    {
        DBuf<uint32_t> packed;
        if (pack_columns(n)) GX_TRY(packed.alloc((3 * nnz + 3) / 4 + 4));
        GX_TRY(upload_columns(ctx, A->colidx, nnz, n, g->A.ci.p, packed.p, nt, &bad, ctx->stream, NoAfter(), true));
    }
    if (bad) return fail(GX_INVALID_INDEX, "gx_graph_create: column out of range");
    clk.mark("upload");
    if (g->weighted)
        GX_TRY(upload(ctx, reinterpret_cast<char *>(g->A.w.p), nnz, 8,
                      [&](uint64_t off, uint64_t cnt, void *buf) {
                          host_copy(buf, static_cast<const double *>(A->vals) + off, cnt * 8);
                          return true;
                      }, &bad));
    g->A.built = true;
    *out = g.release();
    return GX_SUCCESS;
}

extern "C" int gx_graph_free(gx_graph *g) {
    if (!g) return GX_SUCCESS;
    if (g->job) (void)g->job->join();
    (void)hipSetDevice(g->ctx->device);
    (void)hipStreamSynchronize(g->ctx->stream);
    delete g->pr;
    delete g->sssp;
    delete g;
    return GX_SUCCESS;
}

namespace gx {
namespace {

// Row i of the copy = row order[i] of the parent, columns renamed through perm (one wave per
// row; row contents keep the parent's order until build_hub sorts them).
__global__ __launch_bounds__(256) void k_hub_copy(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                  const double *__restrict__ w, const int32_t *__restrict__ order,
                                                  const int32_t *__restrict__ perm, const int64_t *__restrict__ nrp,
                                                  int64_t n, int32_t *__restrict__ nci, double *__restrict__ nw) {
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kWave; i < n; i += (int64_t)gridDim.x * 256 / kWave) {
        const int64_t src = rp[order[i]], len = nrp[i + 1] - nrp[i], dst = nrp[i];
        for (int64_t k = lane; k < len; k += kWave) {
            nci[dst + k] = perm[ci[src + k]];
            if (w) nw[dst + k] = w[src + k];
        }
    }
}

// out[order[x]] = in[x]: the copy's results in the caller's order as a scatter (GX_REMAP=scatter).
// Measured slower than the gather below (BFS on SYN-g500-22 0.346-0.354 against 0.313-0.331 ms
// per run, SSSP on SYN-8_5 6.04-6.06 against 5.98-5.99; profiles/r05_remap_ab.txt): its random
// 4- or 8-byte stores write partial lines.
template <typename T>
__global__ void k_scatter_by(const T *__restrict__ in, const int32_t *__restrict__ order, int64_t n, T *__restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x)
        out[order[x]] = in[x];
}

// out[x] = in[perm[x]]: the remap as a gather (the default): coalesced stores of whole lines,
// random reads served by the Infinity Cache.
template <typename T>
__global__ void k_gather_by(const T *__restrict__ in, const int32_t *__restrict__ perm, int64_t n, T *__restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x)
        out[x] = in[perm[x]];
}

void free_copy(gx_graph *h) { (void)gx_graph_free(h); }

// Hub-first order by degree (descending, ties by id; a counting sort on the host row
// pointers), the copy's row pointers, then the rows renamed on the device.
int build_hub(gx_graph *g) {
    const int64_t n = (int64_t)g->n;
    hipStream_t s = g->ctx->stream;
    GX_TRY(ensure_host_rp(g->ctx, g->A));
    const HostRowPtr &h = g->A.h_rp;
    int64_t maxd = 0;
    for (int64_t v = 0; v < n; v++) maxd = std::max(maxd, h[v + 1] - h[v]);
    std::vector<int64_t> start((size_t)maxd + 2, 0);
    for (int64_t v = 0; v < n; v++) start[(size_t)(maxd - (h[v + 1] - h[v])) + 1]++;
    for (size_t k = 1; k < start.size(); k++) start[k] += start[k - 1];
    std::vector<int32_t> order(n);
    g->h_hub_perm.assign(n, 0);
    for (int64_t v = 0; v < n; v++) {
        const int64_t pos = start[(size_t)(maxd - (h[v + 1] - h[v]))]++;
        order[pos] = (int32_t)v;
        g->h_hub_perm[v] = (int32_t)pos;
    }
    std::shared_ptr<gx_graph> c(new gx_graph(), free_copy);
    c->ctx = g->ctx;
    c->n = g->n;
    c->nnz = g->nnz;
    c->directed = false;
    c->weighted = g->weighted;
    c->mean_w = g->mean_w;
    c->A.n = g->n;
    c->A.nnz = g->nnz;
    c->A.h_rp.assign(n + 1, 0);
    for (int64_t i = 0; i < n; i++) c->A.h_rp[i + 1] = c->A.h_rp[i] + (h[order[i] + 1] - h[order[i]]);
    GX_TRY(g->hub_perm.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(g->hub_order.alloc(std::max<int64_t>(n, 1)));
    GX_TRY(c->A.rp.alloc(n + 1));
    GX_TRY(c->A.ci.alloc(g->nnz, 16));
    if (g->weighted) GX_TRY(c->A.w.alloc(g->nnz));
    GX_HIP_TRY(hipMemcpyAsync(g->hub_perm.p, g->h_hub_perm.data(), n * 4, hipMemcpyHostToDevice, s));
    GX_HIP_TRY(hipMemcpyAsync(g->hub_order.p, order.data(), n * 4, hipMemcpyHostToDevice, s));
    GX_HIP_TRY(hipMemcpyAsync(c->A.rp.p, c->A.h_rp.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (n) {
        hipLaunchKernelGGL(k_hub_copy, dim3(grid_for((uint64_t)n * kWave, 256, 1u << 20)), dim3(256), 0, s, g->A.rp.p,
                           g->A.ci.p, g->weighted ? g->A.w.p : nullptr, g->hub_order.p, g->hub_perm.p, c->A.rp.p, n,
                           c->A.ci.p, g->weighted ? c->A.w.p : nullptr);
        GX_TRY(check_launch("k_hub_copy"));
        // rows sorted by their hub-first ids (GX_HUB_SORT=0 keeps the parent's entry order): a
        // row's first entries are then its largest hubs.  Afforest's first sampling round alone
        // (each vertex hooked to its first neighbour) then joins the giant component: on
        // SYN-g500-22 2.40 M vertices under one root and 1 507 outside it, where the parent's
        // order left 17 603 roots and a second round of 1.53 M hooks aimed at a few hot roots
        // (115 K at the hottest; tools/wcc_round_model.py), which k_afforest_minhook served in
        // series.  BFS bottom-up probes the hubs first for the same reason.
        const char *se = std::getenv("GX_HUB_SORT");
        if (!(se && std::atoi(se) == 0) && g->nnz) {
            DBuf<int32_t> ci2;
            DBuf<double> w2;
            GX_TRY(ci2.alloc(g->nnz, 16));
            if (g->weighted) GX_TRY(w2.alloc(g->nnz));
            int bits = 1;
            while ((1ll << bits) < n) bits++;
            GX_TRY(sort_rows_i32(c->A.rp.p, n, (int64_t)g->nnz, c->A.ci.p, ci2.p, g->weighted ? c->A.w.p : nullptr,
                                 g->weighted ? w2.p : nullptr, bits, s));
            std::swap(c->A.ci.p, ci2.p);
            std::swap(c->A.ci.n, ci2.n);
            if (g->weighted) {
                std::swap(c->A.w.p, w2.p);
                std::swap(c->A.w.n, w2.n);
            }
            GX_HIP_TRY(hipStreamSynchronize(s));   // the unsorted buffers are freed at the end of the block
            c->rows_sorted = true;
        }
    }
    GX_HIP_TRY(hipStreamSynchronize(s));   // the host vectors die at return
    GX_TRY(c->remap_tmp.alloc(std::max<int64_t>(n, 1)));
    c->live = 0;
    while (c->live < n && c->A.h_rp[c->live + 1] > c->A.h_rp[c->live]) c->live++;
    c->A.built = true;
    c->out_perm = g->hub_perm.p;
    c->out_order = g->hub_order.p;
    g->hub = c;
    return GX_SUCCESS;
}

}  // namespace

int hub_for(gx_graph *g, int calls, gx_graph **out, uint64_t *src) {
    *out = nullptr;
    if (g->directed || g->out_perm || g->n < 2) return GX_SUCCESS;
    // the copy is allocated and built on the graph's device, whatever device is current
    GX_HIP_TRY(hipSetDevice(g->ctx->device));
    const char *e = std::getenv("GX_HUB");
    const int mode = e ? std::atoi(e) : 1;
    if (!(mode == 2 || (mode == 1 && calls >= 2))) return GX_SUCCESS;
    if (!g->hub) GX_TRY(build_hub(g));
    if (src) *src = (uint64_t)g->h_hub_perm[*src];
    *out = g->hub.get();
    return GX_SUCCESS;
}

int remap_out(gx_graph *g, const void *buf, int elem, hipStream_t s, const void **res) {
    *res = buf;
    if (!g->out_perm || !g->n) return GX_SUCCESS;
    const int64_t n = (int64_t)g->n;
    void *tmp = g->remap_tmp.p;   // n words, allocated with the copy
    const unsigned grid = grid_for((uint64_t)n, 256, 8192);
    const char *re = std::getenv("GX_REMAP");
    if (!(re && std::strcmp(re, "scatter") == 0)) {
        if (elem == 8)
            hipLaunchKernelGGL(k_gather_by<uint64_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint64_t *>(buf),
                               g->out_perm, n, static_cast<uint64_t *>(tmp));
        else
            hipLaunchKernelGGL(k_gather_by<uint32_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint32_t *>(buf),
                               g->out_perm, n, static_cast<uint32_t *>(tmp));
        GX_TRY(check_launch("k_gather_by"));
        *res = tmp;
        return GX_SUCCESS;
    }
    if (elem == 8)
        hipLaunchKernelGGL(k_scatter_by<uint64_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint64_t *>(buf),
                           g->out_order, n, static_cast<uint64_t *>(tmp));
    else
        hipLaunchKernelGGL(k_scatter_by<uint32_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint32_t *>(buf),
                           g->out_order, n, static_cast<uint32_t *>(tmp));
    GX_TRY(check_launch("k_scatter_by"));
    *res = tmp;
    return GX_SUCCESS;
}

}  // namespace gx

extern "C" int gx_graph_info(gx_graph *g, uint64_t *n, uint64_t *nnz, int *directed, int *weighted) {
    if (!g) return fail(GX_NULL_POINTER, "gx_graph_info: null graph");
    if (n) *n = g->n;
    if (nnz) *nnz = g->nnz;
    if (directed) *directed = g->directed;
    if (weighted) *weighted = g->weighted;
    return GX_SUCCESS;
}

// ------------------------------------------------------------------ device transforms

namespace {

constexpr int kBuildBlock = 256;
constexpr int kEdgesPerThread = 16;

// keys[k] = (col << 32) | row for every edge k of A (one chunk of edges per thread).
__global__ void k_transpose_keys(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                 int64_t n, int64_t nnz, uint64_t *__restrict__ keys) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t e0 = t * kEdgesPerThread;
    if (e0 >= nnz) return;
    int64_t e1 = min(e0 + kEdgesPerThread, nnz);
    int64_t r = row_of_edge(rp, n, e0);
    for (int64_t e = e0; e < e1; e++) {
        while (rp[r + 1] <= e) r++;
        keys[e] = ((uint64_t)(uint32_t)ci[e] << 32) | (uint32_t)r;
    }
}

// Closure keys: both orientations of every non-loop edge, flag 1 (stored v->u) / 2 (u->v).
__global__ void k_closure_keys(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                               int64_t n, int64_t nnz, uint64_t *__restrict__ keys,
                               uint8_t *__restrict__ flags) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t e0 = t * kEdgesPerThread;
    if (e0 >= nnz) return;
    int64_t e1 = min(e0 + kEdgesPerThread, nnz);
    int64_t r = row_of_edge(rp, n, e0);
    for (int64_t e = e0; e < e1; e++) {
        while (rp[r + 1] <= e) r++;
        uint32_t u = (uint32_t)r, v = (uint32_t)ci[e];
        if (u == v) {   // self-loop: sorts to the very end, dropped by count
            keys[2 * e] = keys[2 * e + 1] = ~0ull;
            flags[2 * e] = flags[2 * e + 1] = 0;
        } else {
            keys[2 * e] = ((uint64_t)u << 32) | v;
            flags[2 * e] = 1;
            keys[2 * e + 1] = ((uint64_t)v << 32) | u;
            flags[2 * e + 1] = 2;
        }
    }
}

// rp[r] = lower_bound(keys, r << 32) for r in [0, n]; ci[k] = low word of keys[k].
__global__ void k_keys_to_csr(const uint64_t *__restrict__ keys, int64_t m, int64_t n,
                              int64_t *__restrict__ rp, int32_t *__restrict__ ci) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t <= n) {
        uint64_t target = (uint64_t)t << 32;
        int64_t lo = 0, hi = m;
        while (lo < hi) {
            int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        rp[t] = lo;
    }
    for (int64_t k = t; k < m; k += (int64_t)gridDim.x * blockDim.x)
        ci[k] = (int32_t)(uint32_t)(keys[k] & 0xffffffffu);
}

__global__ void k_outdeg(const int64_t *__restrict__ rp, int64_t n, int32_t *__restrict__ deg) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x)
        deg[v] = (int32_t)(rp[v + 1] - rp[v]);
}

struct BitOr {
    __device__ __host__ uint8_t operator()(uint8_t a, uint8_t b) const { return a | b; }
};

int key_bits(uint64_t n) {
    int b = 1;
    while ((1ull << b) < n) b++;
    return 32 + b;   // (row << 32) | col with row < n
}

}  // namespace

namespace gx {

// rocPRIM temporary storage: one grow-only buffer per device, reused by every sort and scan,
// so a call neither allocates, frees nor synchronises (the buffer outlives the stream work
// that uses it; growing frees the old one, and hipFree waits for the device).  libgx is
// driven by one host thread per device.
// (Never destroyed: a static destructor would free after the HIP runtime shut down.)
static DBuf<char> *const g_tmp = new DBuf<char>[64];

static DBuf<char> *const g_scratch = new DBuf<char>[64];

static int grow_slot(DBuf<char> *slots, size_t bytes, void **p) {
    int dev = 0;
    GX_HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(GX_NOT_IMPLEMENTED, "more than 64 devices");
    DBuf<char> &t = slots[dev];
    if (t.n < bytes) GX_TRY(t.alloc(std::max<size_t>(bytes, 1 << 20)));
    *p = t.p;
    return GX_SUCCESS;
}

// The rocPRIM temporary storage is one grow-only buffer per device, shared by every stream
// and context on it: a user on another stream than the last one first waits for the last
// use (an event recorded after each sort / scan), so two queued users never overlap in it.
struct TmpUse {
    hipStream_t last = nullptr;
    hipEvent_t done = nullptr;
};
static TmpUse *const g_tmp_use = new TmpUse[64];

static int rocprim_tmp(size_t bytes, void **p, hipStream_t s) {
    int dev = 0;
    GX_HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(GX_NOT_IMPLEMENTED, "more than 64 devices");
    TmpUse &u = g_tmp_use[dev];
    if (!u.done) GX_HIP_TRY(hipEventCreateWithFlags(&u.done, hipEventDisableTiming));
    if (u.last && u.last != s) GX_HIP_TRY(hipStreamWaitEvent(s, u.done, 0));
    return grow_slot(g_tmp, bytes, p);
}

static int rocprim_tmp_release(hipStream_t s) {
    int dev = 0;
    GX_HIP_TRY(hipGetDevice(&dev));
    TmpUse &u = g_tmp_use[dev];
    GX_HIP_TRY(hipEventRecord(u.done, s));
    u.last = s;
    return GX_SUCCESS;
}

// Plan-time scratch of the current device (the PageRank plan's sort keys and values): grow-only
// and kept, so a plan neither frees gigabytes (hipFree waits for the device) nor allocates
// them again for the next graph.  One user at a time (the plan builders, one host thread).
int plan_scratch(size_t bytes, void **p) { return grow_slot(g_scratch, bytes, p); }

int sort_keys_u64(uint64_t *k_in, uint64_t *k_out, size_t m, int end_bit, hipStream_t s) {
    if (!m) return GX_SUCCESS;
    size_t tmp_bytes = 0;
    GX_HIP_TRY(rocprim::radix_sort_keys(nullptr, tmp_bytes, k_in, k_out, m, 0, end_bit, s));
    void *tmp = nullptr;
    GX_TRY(rocprim_tmp(tmp_bytes, &tmp, s));
    GX_HIP_TRY(rocprim::radix_sort_keys(tmp, tmp_bytes, k_in, k_out, m, 0, end_bit, s));
    return rocprim_tmp_release(s);
}

template <typename K, typename V>
static int sort_pairs_kv(K *k_in, K *k_out, V *v_in, V *v_out, size_t m, int end_bit, bool desc, hipStream_t s) {
    if (!m) return GX_SUCCESS;
    size_t tmp_bytes = 0;
    if (desc)
        GX_HIP_TRY(rocprim::radix_sort_pairs_desc(nullptr, tmp_bytes, k_in, k_out, v_in, v_out, m, 0, end_bit, s));
    else
        GX_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k_in, k_out, v_in, v_out, m, 0, end_bit, s));
    void *tmp = nullptr;
    GX_TRY(rocprim_tmp(tmp_bytes, &tmp, s));
    if (desc)
        GX_HIP_TRY(rocprim::radix_sort_pairs_desc(tmp, tmp_bytes, k_in, k_out, v_in, v_out, m, 0, end_bit, s));
    else
        GX_HIP_TRY(rocprim::radix_sort_pairs(tmp, tmp_bytes, k_in, k_out, v_in, v_out, m, 0, end_bit, s));
    return rocprim_tmp_release(s);
}

int sort_pairs_u32_u16(uint32_t *k_in, uint32_t *k_out, uint16_t *v_in, uint16_t *v_out, size_t m, int end_bit,
                       hipStream_t s) {
    return sort_pairs_kv(k_in, k_out, v_in, v_out, m, end_bit, false, s);
}

int sort_pairs_u64_u16(uint64_t *k_in, uint64_t *k_out, uint16_t *v_in, uint16_t *v_out, size_t m, int end_bit,
                       hipStream_t s) {
    return sort_pairs_kv(k_in, k_out, v_in, v_out, m, end_bit, false, s);
}

int sort_pairs_u64_u32(uint64_t *k_in, uint64_t *k_out, uint32_t *v_in, uint32_t *v_out, size_t m, int end_bit,
                       hipStream_t s) {
    return sort_pairs_kv(k_in, k_out, v_in, v_out, m, end_bit, false, s);
}

int sort_pairs_desc_u32_i32(uint32_t *k_in, uint32_t *k_out, int32_t *v_in, int32_t *v_out, size_t m, hipStream_t s) {
    return sort_pairs_kv(k_in, k_out, v_in, v_out, m, 32, true, s);
}

int sort_rows_i32(const int64_t *rp, int64_t n, int64_t nnz, int32_t *ci_in, int32_t *ci_out, double *w_in,
                  double *w_out, int end_bit, hipStream_t s) {
    if (!nnz || !n) return GX_SUCCESS;
    if (nnz >= (1ll << 32) || n >= (1ll << 32)) return fail(GX_NOT_IMPLEMENTED, "sort_rows_i32: more than 2^32 entries");
    size_t tmp_bytes = 0;
    if (w_in)
        GX_HIP_TRY(rocprim::segmented_radix_sort_pairs(nullptr, tmp_bytes, ci_in, ci_out, w_in, w_out, (unsigned)nnz,
                                                       (unsigned)n, rp, rp + 1, 0, end_bit, s));
    else
        GX_HIP_TRY(rocprim::segmented_radix_sort_keys(nullptr, tmp_bytes, ci_in, ci_out, (unsigned)nnz, (unsigned)n, rp,
                                                      rp + 1, 0, end_bit, s));
    void *tmp = nullptr;
    GX_TRY(rocprim_tmp(tmp_bytes, &tmp, s));
    if (w_in)
        GX_HIP_TRY(rocprim::segmented_radix_sort_pairs(tmp, tmp_bytes, ci_in, ci_out, w_in, w_out, (unsigned)nnz,
                                                       (unsigned)n, rp, rp + 1, 0, end_bit, s));
    else
        GX_HIP_TRY(rocprim::segmented_radix_sort_keys(tmp, tmp_bytes, ci_in, ci_out, (unsigned)nnz, (unsigned)n, rp,
                                                      rp + 1, 0, end_bit, s));
    return rocprim_tmp_release(s);
}

int scan_exclusive_i64(const int64_t *in, int64_t *out, size_t m, hipStream_t s) {
    if (!m) return GX_SUCCESS;
    size_t tmp_bytes = 0;
    GX_HIP_TRY(rocprim::exclusive_scan(nullptr, tmp_bytes, in, out, (int64_t)0, m, rocprim::plus<int64_t>(), s));
    void *tmp = nullptr;
    GX_TRY(rocprim_tmp(tmp_bytes, &tmp, s));
    GX_HIP_TRY(rocprim::exclusive_scan(tmp, tmp_bytes, in, out, (int64_t)0, m, rocprim::plus<int64_t>(), s));
    return rocprim_tmp_release(s);
}

int sort_keys_to_csr(DBuf<uint64_t> &keys, DBuf<uint64_t> &scratch, size_t m, int64_t n, int64_t *rp,
                     int32_t *ci, hipStream_t s) {
    if (m) {
        const int bits = key_bits((uint64_t)n);
        size_t tmp_bytes = 0;
        GX_HIP_TRY(rocprim::radix_sort_keys(nullptr, tmp_bytes, keys.p, scratch.p, m, 0, bits, s));
        DBuf<char> tmp;
        GX_TRY(tmp.alloc(tmp_bytes));
        GX_HIP_TRY(rocprim::radix_sort_keys(tmp.p, tmp_bytes, keys.p, scratch.p, m, 0, bits, s));
        GX_HIP_TRY(hipMemcpyAsync(keys.p, scratch.p, m * 8, hipMemcpyDeviceToDevice, s));
        GX_HIP_TRY(hipStreamSynchronize(s));   // tmp is freed at return
    }
    hipLaunchKernelGGL(k_keys_to_csr, dim3(grid_for((uint64_t)n + 1, 256, 1u << 30)), dim3(256), 0, s, keys.p,
                       (int64_t)m, n, rp, ci);
    return check_launch("k_keys_to_csr");
}

int ensure_outdeg(gx_graph *g) {
    if (g->outdeg.p) return GX_SUCCESS;
    GX_TRY(g->outdeg.alloc(g->n));
    hipLaunchKernelGGL(k_outdeg, dim3(grid_for(g->n, 256, 4096)), dim3(256), 0, g->ctx->stream,
                       g->A.rp.p, (int64_t)g->n, g->outdeg.p);
    return check_launch("k_outdeg");
}

int ensure_transpose(gx_graph *g) {
    if (g->AT.built) return GX_SUCCESS;
    hipStream_t s = g->ctx->stream;
    const uint64_t n = g->n, nnz = g->nnz;
    DBuf<uint64_t> k0, k1;
    DBuf<double> w1;
    GX_TRY(k0.alloc(nnz));
    GX_TRY(k1.alloc(nnz));
    GX_TRY(g->AT.rp.alloc(n + 1));
    GX_TRY(g->AT.ci.alloc(nnz, 16));
    if (g->weighted) GX_TRY(g->AT.w.alloc(nnz));
    if (nnz) {
        unsigned grid = grid_for((nnz + kEdgesPerThread - 1) / kEdgesPerThread, kBuildBlock, 1u << 30);
        hipLaunchKernelGGL(k_transpose_keys, dim3(grid), dim3(kBuildBlock), 0, s, g->A.rp.p,
                           g->A.ci.p, (int64_t)n, (int64_t)nnz, k0.p);
        GX_TRY(check_launch("k_transpose_keys"));
        size_t tmp_bytes = 0;
        const int bits = key_bits(n);
        if (g->weighted) {
            GX_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0.p, k1.p, g->A.w.p, g->AT.w.p,
                                                 (size_t)nnz, 0, bits, s));
        } else {
            GX_HIP_TRY(rocprim::radix_sort_keys(nullptr, tmp_bytes, k0.p, k1.p, (size_t)nnz, 0, bits, s));
        }
        DBuf<char> tmp;
        GX_TRY(tmp.alloc(tmp_bytes));
        if (g->weighted) {
            GX_HIP_TRY(rocprim::radix_sort_pairs(tmp.p, tmp_bytes, k0.p, k1.p, g->A.w.p, g->AT.w.p,
                                                 (size_t)nnz, 0, bits, s));
        } else {
            GX_HIP_TRY(rocprim::radix_sort_keys(tmp.p, tmp_bytes, k0.p, k1.p, (size_t)nnz, 0, bits, s));
        }
    }
    hipLaunchKernelGGL(k_keys_to_csr, dim3(grid_for(n + 1, 256, 1u << 30)), dim3(256), 0, s, k1.p,
                       (int64_t)nnz, (int64_t)n, g->AT.rp.p, g->AT.ci.p);
    GX_TRY(check_launch("k_keys_to_csr"));
    g->AT.n = n;
    g->AT.nnz = nnz;
    g->AT.h_rp.resize(n + 1);
    GX_HIP_TRY(hipMemcpyAsync(g->AT.h_rp.data(), g->AT.rp.p, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    g->AT.built = true;
    return GX_SUCCESS;
}

int ensure_closure(gx_graph *g) {
    if (g->S.built) return GX_SUCCESS;
    hipStream_t s = g->ctx->stream;
    const uint64_t n = g->n, nnz = g->nnz, m2 = 2 * nnz;
    DBuf<uint64_t> k0, k1, uk;
    DBuf<uint8_t> f0, f1;
    DBuf<uint64_t> count;
    GX_TRY(k0.alloc(m2));
    GX_TRY(k1.alloc(m2));
    GX_TRY(f0.alloc(m2));
    GX_TRY(f1.alloc(m2));
    GX_TRY(uk.alloc(m2));
    GX_TRY(count.alloc(1));
    GX_TRY(g->S.rp.alloc(n + 1));
    uint64_t m = 0;
    if (nnz) {
        unsigned grid = grid_for((nnz + kEdgesPerThread - 1) / kEdgesPerThread, kBuildBlock, 1u << 30);
        hipLaunchKernelGGL(k_closure_keys, dim3(grid), dim3(kBuildBlock), 0, s, g->A.rp.p, g->A.ci.p,
                           (int64_t)n, (int64_t)nnz, k0.p, f0.p);
        GX_TRY(check_launch("k_closure_keys"));
        size_t tmp_sort = 0, tmp_red = 0;
        GX_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tmp_sort, k0.p, k1.p, f0.p, f1.p, (size_t)m2, 0, 64, s));
        GX_HIP_TRY(rocprim::reduce_by_key(nullptr, tmp_red, k1.p, f1.p, (size_t)m2, uk.p, f0.p, count.p,
                                          BitOr(), rocprim::equal_to<uint64_t>(), s));
        DBuf<char> tmp;
        GX_TRY(tmp.alloc(std::max(tmp_sort, tmp_red)));
        GX_HIP_TRY(rocprim::radix_sort_pairs(tmp.p, tmp_sort, k0.p, k1.p, f0.p, f1.p, (size_t)m2, 0, 64, s));
        GX_HIP_TRY(rocprim::reduce_by_key(tmp.p, tmp_red, k1.p, f1.p, (size_t)m2, uk.p, f0.p, count.p,
                                          BitOr(), rocprim::equal_to<uint64_t>(), s));
        GX_HIP_TRY(hipMemcpyAsync(&m, count.p, 8, hipMemcpyDeviceToHost, s));
        GX_HIP_TRY(hipStreamSynchronize(s));
        // a trailing ~0 key collects every self-loop
        if (m > 0) {
            uint64_t last = 0;
            GX_HIP_TRY(hipMemcpy(&last, uk.p + (m - 1), 8, hipMemcpyDeviceToHost));
            if (last == ~0ull) m--;
        }
    }
    GX_TRY(g->S.ci.alloc(m, 16));
    GX_TRY(g->S.flag.alloc(m));
    hipLaunchKernelGGL(k_keys_to_csr, dim3(grid_for(n + 1, 256, 1u << 30)), dim3(256), 0, s, uk.p,
                       (int64_t)m, (int64_t)n, g->S.rp.p, g->S.ci.p);
    GX_TRY(check_launch("k_keys_to_csr"));
    if (m) GX_HIP_TRY(hipMemcpyAsync(g->S.flag.p, f0.p, m, hipMemcpyDeviceToDevice, s));
    g->S.n = n;
    g->S.nnz = m;
    g->S.h_rp.resize(n + 1);
    GX_HIP_TRY(hipMemcpyAsync(g->S.h_rp.data(), g->S.rp.p, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    GX_HIP_TRY(hipStreamSynchronize(s));
    g->S.built = true;
    return GX_SUCCESS;
}

}  // namespace gx

GX_MODULE_WARMER(runtime)
