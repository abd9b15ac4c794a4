// gx_comm.hip -- RCCL communicator and the device-driven partitioned PageRank loop.
//
// the pull matrix is 1-D row partitioned over the GPUs (one process per GPU)
// and the rank vector is all-gathered over xGMI every iteration.  The reference has no
// distributed path; this replaces the per-iteration GrB_mxv of LAGr_PageRankGX
// (pr.cpp:61) when it runs on several GPUs.
//
// gx_pr_part_step is one iteration of one rank (or piece); driving the iterations from
// Python costs one ctypes call plus one torch.distributed collective per piece and
// iteration (~60 us of host time each, measured), more than the per-rank SpMV at 8 GPUs.
// gx_pr_dist runs a whole PageRank from here instead: every kernel and every
// ncclAllGather is enqueued by one C call, and with `use_graph` the whole run (init, all
// iterations, all gathers) is captured once into a hipGraph and replayed, so the host
// cost per run is one graph launch.
//
// Pipelining (pr_partition.local_pieces): a rank owns `npieces` virtual ranks
// p * nranks + rank.  Piece p's chunks of all ranks form one contiguous slab of the
// exchanged vector, so each piece is gathered by its own ncclAllGather on the comm
// stream while the compute stream runs the next piece's SpMV:
//
//   compute: step(0) step(1) ... step(P-1) |wait comm| step(0) ...
//   comm   :        gather(0) gather(1) ... gather(P-1)|
//
// The vector is double-buffered (x_read / x_write) so a gather never overwrites values
// that a later piece of the same iteration still reads.
//
// RCCL is opened lazily with dlopen: torch's copy when the process already has one
// (same soname, librccl.so.1), else ROCm's.  libgx itself has no link dependency on it,
// so the single-GPU executables never load RCCL.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gx_pr.h"

namespace gx {
namespace {

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                           hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    std::string error;
    bool ok = false;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // torch's, if loaded
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char *e = dlerror();
            r.error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
        r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
        r.reduce = reinterpret_cast<decltype(r.reduce)>(dlsym(h, "ncclReduce"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
        r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.error_string &&
               r.comm_init_all && r.group_start && r.group_end && r.reduce;
        if (!r.ok) r.error = "librccl.so.1 lacks an expected entry point";
    });
    return r;
}

int rccl_fail(const char *what, ncclResult_t e) {
    return fail(GX_DEVICE_ERROR, std::string(what) + ": " + rccl().error_string(e));
}

#define GX_NCCL_TRY(what, expr)                         \
    do {                                                \
        ncclResult_t _r = (expr);                       \
        if (_r != ncclSuccess) return rccl_fail(what, _r); \
    } while (0)

// ---- one-shot peer-to-peer exchange (gx_pr_dist_create_p2p) ----
// Every rank writes its chunk straight into every peer's exchanged vector (IPC-mapped over
// xGMI: one write per peer, all 7 links at once) instead of RCCL's ring, then raises an
// arrival flag in the peer's flag array.  Tokens grow monotonically across runs (a device
// run counter, so a replayed hipGraph raises new ones): token = run * kTok + step, step 0 =
// the initial exchange, it + 1 = iteration it's.  Memory model (LLVM AMDGPU, gfx942/950):
// the writer's data stores, a system-scope release, the flag store (system scope); the reader
// polls with system-scope loads and ends with a system-scope acquire, and the SpMV that
// reads x follows in stream order.  A wait gives up after `polls` polls (a dead or diverged
// peer), sets the error word and exits, so no wave spins forever.
constexpr uint64_t kTok = 1ull << 24;

__global__ void k_p2p_begin(uint64_t *seq) {
    if (threadIdx.x == 0) seq[0] += 1;
}

// chunk doubles of src into dst[q] + off for every rank q (blockIdx.y; chunk, off: multiples
// of 2), then flag[q][slot] = this run's token for `step`, raised by the workgroup that takes
// the last ticket (after every workgroup's system-scope release).  A few workgroups per peer:
// one xGMI link is ~50 GB/s, and the puts run beside the next piece's SpMV.
__global__ __launch_bounds__(256) void k_p2p_put(const double *__restrict__ src, uint64_t chunk,
                                                 double *const *__restrict__ dst, uint64_t off,
                                                 uint64_t *const *__restrict__ flags, uint64_t slot,
                                                 const uint64_t *seq, uint64_t step, uint32_t *ticket) {
    double2 *d = reinterpret_cast<double2 *>(dst[blockIdx.y] + off);
    const double2 *s = reinterpret_cast<const double2 *>(src);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < chunk / 2; i += (uint64_t)gridDim.x * 256) d[i] = s[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: the stores reach the peers first
    __syncthreads();
    if (threadIdx.x != 0) return;
    const uint32_t all = gridDim.x * gridDim.y;
    if (__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM) != all - 1) return;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint64_t tok = seq[0] * kTok + step;
    for (uint32_t q = 0; q < gridDim.y; q++) __hip_atomic_store(flags[q] + slot, tok, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// flag[q][slot] = this run's token for `step`, for every rank q < world
__global__ void k_p2p_signal(uint64_t *const *__restrict__ flags, int world, uint64_t slot, const uint64_t *seq,
                             uint64_t step) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const int q = threadIdx.x;
    if (q < world) __hip_atomic_store(flags[q] + slot, seq[0] * kTok + step, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one wave: until flags[0 .. count) all hold at least (run - prev) * kTok + step
__global__ __launch_bounds__(64) void k_p2p_wait(const uint64_t *flags, int count, const uint64_t *seq, uint64_t step,
                                                 uint64_t prev, uint64_t *err, uint32_t polls) {
    const uint64_t target = (seq[0] - prev) * kTok + step;
    // after a timeout the run's results are void: later waits of the run do not poll again
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    for (uint32_t it = 0;; it++) {
        bool ok = true;
        for (int i = threadIdx.x; i < count; i += 64)
            ok = ok && __hip_atomic_load(flags + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= target;
        if (__all(ok)) break;
        if (it >= polls) {
            if (threadIdx.x == 0) __hip_atomic_store(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope
}

}  // namespace
}  // namespace gx

using namespace gx;

struct gx_comm {
    gx_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
};

namespace {

struct PrDist {
    gx_ctx *ctx = nullptr;
    gx_comm *comm = nullptr;           // null: one rank (pieces exchanged by D2D copies)
    std::vector<PrPart *> pieces;
    int world = 1, rank = 0;           // real ranks
    uint64_t chunk = 0;
    DBuf<double> xa, xb;               // gathered vector, double-buffered
    std::vector<std::unique_ptr<DBuf<double>>> xl;   // per piece: its local chunk
    std::vector<std::unique_ptr<DBuf<double>>> ro;   // per piece: scores of its rows
    hipStream_t cs = nullptr;          // comm stream
    std::vector<hipEvent_t> ev_piece;
    hipEvent_t ev_comm = nullptr;
    hipGraphExec_t gexec = nullptr;
    hipGraph_t graph = nullptr;
    int g_iters = -1;
    hipStream_t g_stream = nullptr;
    hipStream_t last_stream = nullptr;
    // one-shot peer-to-peer exchange (gx_pr_dist_create_p2p): flags[p * world + q] = the last
    // token rank q raised here for piece p, flags[np * world + q] = q's end of its last run
    bool p2p = false, attached = false;
    DBuf<uint64_t> flags, seq;            // seq[0]: runs started; seq[1]: a wait timed out
    DBuf<double *> pxa, pxb;              // per rank: its xa / xb (ours for this rank)
    DBuf<uint64_t *> pfl;                 // per rank: its flags
    std::vector<void *> opened;           // the peers' IPC mappings
    DBuf<uint32_t> tickets;               // per piece: k_p2p_put's workgroup tickets
    uint32_t polls = 1u << 22;
    uint32_t put_blocks = 32;             // workgroups per peer (GX_P2P_BLOCKS)

    ~PrDist() {
        (void)hipSetDevice(ctx->device);
        (void)hipDeviceSynchronize();
        for (void *q : opened) (void)hipIpcCloseMemHandle(q);
        if (gexec) (void)hipGraphExecDestroy(gexec);
        if (graph) (void)hipGraphDestroy(graph);
        for (hipEvent_t e : ev_piece) (void)hipEventDestroy(e);
        if (ev_comm) (void)hipEventDestroy(ev_comm);
        if (cs) (void)hipStreamDestroy(cs);
    }

    size_t span() const { return chunk * (size_t)world; }   // one piece's slab

    int np() const { return (int)pieces.size(); }

    // exchange piece p's local chunk into slab p of `x` (after what s has enqueued so far);
    // `step` names the exchange for the peer-to-peer flags
    int gather(int p, double *x, hipStream_t s, uint64_t step) {
        double *dst = x + (size_t)p * span();
        if (p2p) {
            GX_HIP_TRY(hipEventRecord(ev_piece[p], s));
            GX_HIP_TRY(hipStreamWaitEvent(cs, ev_piece[p], 0));
            const unsigned blocks = (unsigned)std::min<uint64_t>(put_blocks, (chunk / 2 + 255) / 256);
            hipLaunchKernelGGL(k_p2p_put, dim3(std::max(blocks, 1u), world), dim3(256), 0, cs, xl[p]->p, chunk,
                               x == xa.p ? pxa.p : pxb.p, (uint64_t)p * span() + (uint64_t)rank * chunk, pfl.p,
                               (uint64_t)p * world + rank, seq.p, step, tickets.p + p);
            return check_launch("k_p2p_put");
        }
        if (!comm) {
            GX_HIP_TRY(hipMemcpyAsync(dst, xl[p]->p, chunk * sizeof(double), hipMemcpyDeviceToDevice, s));
            return GX_SUCCESS;
        }
        GX_HIP_TRY(hipEventRecord(ev_piece[p], s));
        GX_HIP_TRY(hipStreamWaitEvent(cs, ev_piece[p], 0));
        GX_NCCL_TRY("ncclAllGather", rccl().all_gather(xl[p]->p, dst, chunk, ncclFloat64, comm->comm, cs));
        return GX_SUCCESS;
    }

    // compute stream waits for every gather issued so far (peer-to-peer: and for every
    // rank's chunks of exchange `step` to have arrived here)
    int join(hipStream_t s, uint64_t step) {
        if (!comm && !p2p) return GX_SUCCESS;
        GX_HIP_TRY(hipEventRecord(ev_comm, cs));
        GX_HIP_TRY(hipStreamWaitEvent(s, ev_comm, 0));
        if (p2p) {
            hipLaunchKernelGGL(k_p2p_wait, dim3(1), dim3(64), 0, s, flags.p, np() * world, seq.p, step, (uint64_t)0,
                               seq.p + 1, polls);
            GX_TRY(check_launch("k_p2p_wait"));
        }
        return GX_SUCCESS;
    }

    int enqueue(int iters, hipStream_t s) {
        const int np = (int)pieces.size();
        const bool swap_only = !comm && !p2p && np == 1;   // one rank, one piece: no exchange at all
        double *xr = xa.p, *xw = xb.p;
        if (p2p) {
            // a new run; its first exchange overwrites the peers' xa, so every peer must have
            // finished reading it in the previous run (their end-of-run tokens)
            hipLaunchKernelGGL(k_p2p_begin, dim3(1), dim3(64), 0, s, seq.p);
            GX_TRY(check_launch("k_p2p_begin"));
            hipLaunchKernelGGL(k_p2p_wait, dim3(1), dim3(64), 0, s, flags.p + (size_t)np * world, world, seq.p,
                               (uint64_t)0, (uint64_t)1, seq.p + 1, polls);
            GX_TRY(check_launch("k_p2p_wait"));
        }
        for (int p = 0; p < np; p++) GX_TRY(pr_init(pieces[p], swap_only ? xr : xl[p]->p, s));
        if (!swap_only) {
            for (int p = 0; p < np; p++) GX_TRY(gather(p, xr, s, 0));
            GX_TRY(join(s, 0));
        }
        for (int it = 0; it < iters; it++) {
            const bool last = it == iters - 1;
            for (int p = 0; p < np; p++) {
                double *out = swap_only ? xw : xl[p]->p;
                GX_TRY(pr_step(pieces[p], xr, out, last ? ro[p]->p : nullptr, s));
                if (!last && !swap_only) GX_TRY(gather(p, xw, s, (uint64_t)it + 1));
            }
            if (last) break;
            if (!swap_only) GX_TRY(join(s, (uint64_t)it + 1));
            std::swap(xr, xw);
        }
        if (p2p) {   // this rank is done reading its vectors: the end-of-run token to every rank
            hipLaunchKernelGGL(k_p2p_signal, dim3(1), dim3(64), 0, s, pfl.p, world, (uint64_t)np * world + rank, seq.p,
                               (uint64_t)0);
            GX_TRY(check_launch("k_p2p_signal"));
        }
        return GX_SUCCESS;
    }

    int run(int iters, bool use_graph, hipStream_t s) {
        last_stream = s;
        // kernel timing brackets launches with events, which a replayed graph would not
        // refresh: timed runs go through direct launches
        if (!use_graph || ctx->timing) return enqueue(iters, s);
        if (!gexec || g_iters != iters || g_stream != s) {
            if (gexec) (void)hipGraphExecDestroy(gexec);
            if (graph) (void)hipGraphDestroy(graph);
            gexec = nullptr;
            graph = nullptr;
            GX_HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            const int rc = enqueue(iters, s);
            hipGraph_t g = nullptr;
            const hipError_t e = hipStreamEndCapture(s, &g);
            if (rc != GX_SUCCESS) {
                if (g) (void)hipGraphDestroy(g);
                return rc;
            }
            if (e != hipSuccess) return fail(GX_DEVICE_ERROR, std::string("PageRank capture: ") + hipGetErrorString(e));
            graph = g;
            GX_HIP_TRY(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
            g_iters = iters;
            g_stream = s;
        }
        GX_HIP_TRY(hipGraphLaunch(gexec, s));
        return GX_SUCCESS;
    }
};

}  // namespace

struct gx_pr_dist {
    PrDist d;
};

extern "C" int gx_comm_unique_id(uint8_t *id) {
    if (!id) return fail(GX_NULL_POINTER, "gx_comm_unique_id: null argument");
    const Rccl &r = rccl();
    if (!r.ok) return fail(GX_NOT_IMPLEMENTED, r.error);
    ncclUniqueId u;
    GX_NCCL_TRY("ncclGetUniqueId", r.get_unique_id(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return GX_SUCCESS;
}

extern "C" int gx_comm_create(gx_ctx *ctx, int nranks, int rank, const uint8_t *id, gx_comm **out) {
    if (!ctx || !id || !out) return fail(GX_NULL_POINTER, "gx_comm_create: null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(GX_INVALID_VALUE, "gx_comm_create: bad rank/nranks");
    const Rccl &r = rccl();
    if (!r.ok) return fail(GX_NOT_IMPLEMENTED, r.error);
    GX_HIP_TRY(hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t c = nullptr;
    GX_NCCL_TRY("ncclCommInitRank", r.comm_init_rank(&c, nranks, u, rank));
    auto *cm = new gx_comm();
    cm->ctx = ctx;
    cm->comm = c;
    cm->nranks = nranks;
    cm->rank = rank;
    *out = cm;
    return GX_SUCCESS;
}

extern "C" int gx_comm_free(gx_comm *comm) {
    if (!comm) return GX_SUCCESS;
    (void)hipSetDevice(comm->ctx->device);
    (void)hipDeviceSynchronize();
    if (comm->comm) (void)rccl().comm_destroy(comm->comm);
    delete comm;
    return GX_SUCCESS;
}

namespace {

int dist_create(gx_comm *comm, int world, int rank, bool p2p, gx_pr_part *const *parts, int npieces, gx_pr_dist **out) {
    if (!parts || !out || npieces < 1) return fail(GX_NULL_POINTER, "gx_pr_dist_create: null argument");
    PrPart *p0 = reinterpret_cast<PrPart *>(parts[0]);
    if (!p0) return fail(GX_NULL_POINTER, "gx_pr_dist_create: null piece");
    if (comm && comm->ctx != p0->ctx) return fail(GX_INVALID_VALUE, "gx_pr_dist_create: comm and pieces on different contexts");
    for (int p = 0; p < npieces; p++) {
        PrPart *q = reinterpret_cast<PrPart *>(parts[p]);
        if (!q) return fail(GX_NULL_POINTER, "gx_pr_dist_create: null piece");
        if (q->ctx != p0->ctx || q->chunk != p0->chunk || q->n_global != p0->n_global)
            return fail(GX_INVALID_VALUE, "gx_pr_dist_create: pieces of different partitions");
        if (q->nranks != world * npieces || q->rank != p * world + rank)
            return fail(GX_INVALID_VALUE, "gx_pr_dist_create: piece p must be virtual rank p * nranks + rank "
                                          "of a partition into nranks * npieces ranges");
    }
    gx_ctx *ctx = p0->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    auto *h = new gx_pr_dist();
    PrDist &d = h->d;
    d.ctx = ctx;
    d.comm = comm;
    d.world = world;
    d.rank = rank;
    d.chunk = p0->chunk;
    for (int p = 0; p < npieces; p++) d.pieces.push_back(reinterpret_cast<PrPart *>(parts[p]));
    const size_t full = d.chunk * (size_t)world * (size_t)npieces;
    int rc = d.xa.alloc(full);
    if (rc == GX_SUCCESS) rc = d.xb.alloc(full);
    for (int p = 0; p < npieces; p++) {
        d.xl.emplace_back(new DBuf<double>());
        d.ro.emplace_back(new DBuf<double>());
    }
    for (int p = 0; p < npieces && rc == GX_SUCCESS; p++) {
        rc = d.xl[p]->alloc(d.chunk);
        if (rc == GX_SUCCESS) rc = d.ro[p]->alloc(std::max<uint64_t>(d.pieces[p]->rows, 1));
        // the padding slots (the kernel's zero column among them) stay 0.0 through the exchange
        if (rc == GX_SUCCESS && hipMemset(d.xl[p]->p, 0, d.chunk * sizeof(double)) != hipSuccess)
            rc = fail(GX_DEVICE_ERROR, "hipMemset");
    }
    hipError_t e = hipSuccess;
    if (rc == GX_SUCCESS) e = hipMemset(d.xa.p, 0, full * sizeof(double));
    if (rc == GX_SUCCESS && e == hipSuccess) e = hipMemset(d.xb.p, 0, full * sizeof(double));
    if (rc == GX_SUCCESS && e == hipSuccess && p2p) {
        d.p2p = true;
        const size_t nf = (size_t)(npieces + 1) * world;
        rc = d.flags.alloc(nf);
        if (rc == GX_SUCCESS) rc = d.seq.alloc(2);
        if (rc == GX_SUCCESS) rc = d.pxa.alloc(world);
        if (rc == GX_SUCCESS) rc = d.pxb.alloc(world);
        if (rc == GX_SUCCESS) rc = d.pfl.alloc(world);
        if (rc == GX_SUCCESS) rc = d.tickets.alloc(npieces);
        if (rc == GX_SUCCESS) e = hipMemset(d.tickets.p, 0, npieces * sizeof(uint32_t));
        if (rc == GX_SUCCESS && e == hipSuccess) e = hipMemset(d.flags.p, 0, nf * sizeof(uint64_t));
        if (rc == GX_SUCCESS && e == hipSuccess) e = hipMemset(d.seq.p, 0, 2 * sizeof(uint64_t));
        if (const char *pl = std::getenv("GX_P2P_POLLS")) d.polls = (uint32_t)std::strtoul(pl, nullptr, 10);
        if (const char *pb = std::getenv("GX_P2P_BLOCKS")) d.put_blocks = std::max(1u, (uint32_t)std::strtoul(pb, nullptr, 10));
    }
    if (rc == GX_SUCCESS && e == hipSuccess && (comm || p2p)) {
        e = hipStreamCreateWithFlags(&d.cs, hipStreamNonBlocking);
        d.ev_piece.assign(npieces, nullptr);
        for (int p = 0; p < npieces && e == hipSuccess; p++)
            e = hipEventCreateWithFlags(&d.ev_piece[p], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&d.ev_comm, hipEventDisableTiming);
    }
    if (rc == GX_SUCCESS && e != hipSuccess)
        rc = fail(GX_DEVICE_ERROR, std::string("gx_pr_dist_create: ") + hipGetErrorString(e));
    if (rc != GX_SUCCESS) {
        delete h;
        return rc;
    }
    *out = h;
    return GX_SUCCESS;
}

}  // namespace

extern "C" int gx_pr_dist_create(gx_comm *comm, gx_pr_part *const *parts, int npieces, gx_pr_dist **out) {
    return dist_create(comm, comm ? comm->nranks : 1, comm ? comm->rank : 0, false, parts, npieces, out);
}

// IPC handles of this rank: xa, xb, flags (hipIpcMemHandle_t each)
extern "C" int gx_pr_dist_create_p2p(int nranks, int rank, gx_pr_part *const *parts, int npieces, uint8_t *handle,
                                     gx_pr_dist **out) {
    if (!handle || !out) return fail(GX_NULL_POINTER, "gx_pr_dist_create_p2p: null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks || nranks > 64)
        return fail(GX_INVALID_VALUE, "gx_pr_dist_create_p2p: bad rank/nranks (at most 64 ranks)");
    static_assert(3 * sizeof(hipIpcMemHandle_t) <= GX_P2P_HANDLE_BYTES, "handle bytes");
    gx_pr_dist *h = nullptr;
    GX_TRY(dist_create(nullptr, nranks, rank, true, parts, npieces, &h));
    PrDist &d = h->d;
    std::memset(handle, 0, GX_P2P_HANDLE_BYTES);
    hipIpcMemHandle_t m[3];
    void *bufs[3] = {d.xa.p, d.xb.p, d.flags.p};
    for (int k = 0; k < 3; k++) {
        const hipError_t e = hipIpcGetMemHandle(&m[k], bufs[k]);
        if (e != hipSuccess) {
            delete h;
            return fail(GX_DEVICE_ERROR, std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
        }
        std::memcpy(handle + k * sizeof(hipIpcMemHandle_t), &m[k], sizeof(hipIpcMemHandle_t));
    }
    *out = h;
    return GX_SUCCESS;
}

// handles: nranks * GX_P2P_HANDLE_BYTES in rank order (this rank's own entry is not opened)
extern "C" int gx_pr_dist_p2p_attach(gx_pr_dist *h, const uint8_t *handles) {
    if (!h) return fail(GX_NULL_POINTER, "gx_pr_dist_p2p_attach: null argument");
    PrDist &d = h->d;
    if (!d.p2p) return fail(GX_INVALID_OBJECT, "gx_pr_dist_p2p_attach: not a peer-to-peer runner");
    if (d.attached) return fail(GX_INVALID_OBJECT, "gx_pr_dist_p2p_attach: already attached");
    if (!handles && d.world > 1) return fail(GX_NULL_POINTER, "gx_pr_dist_p2p_attach: null handles");
    GX_HIP_TRY(hipSetDevice(d.ctx->device));
    std::vector<double *> a(d.world), b(d.world);
    std::vector<uint64_t *> f(d.world);
    for (int q = 0; q < d.world; q++) {
        if (q == d.rank) {
            a[q] = d.xa.p;
            b[q] = d.xb.p;
            f[q] = d.flags.p;
            continue;
        }
        void *ptr[3] = {nullptr, nullptr, nullptr};
        for (int k = 0; k < 3; k++) {
            hipIpcMemHandle_t m;
            std::memcpy(&m, handles + (size_t)q * GX_P2P_HANDLE_BYTES + k * sizeof(hipIpcMemHandle_t), sizeof(m));
            const hipError_t e = hipIpcOpenMemHandle(&ptr[k], m, hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess)
                return fail(GX_DEVICE_ERROR, "hipIpcOpenMemHandle (rank " + std::to_string(q) + "): " + hipGetErrorString(e));
            d.opened.push_back(ptr[k]);
        }
        a[q] = static_cast<double *>(ptr[0]);
        b[q] = static_cast<double *>(ptr[1]);
        f[q] = static_cast<uint64_t *>(ptr[2]);
    }
    GX_HIP_TRY(hipMemcpy(d.pxa.p, a.data(), d.world * sizeof(double *), hipMemcpyHostToDevice));
    GX_HIP_TRY(hipMemcpy(d.pxb.p, b.data(), d.world * sizeof(double *), hipMemcpyHostToDevice));
    GX_HIP_TRY(hipMemcpy(d.pfl.p, f.data(), d.world * sizeof(uint64_t *), hipMemcpyHostToDevice));
    d.attached = true;
    return GX_SUCCESS;
}

extern "C" int gx_pr_dist_run(gx_pr_dist *h, int iters, int use_graph, void *stream) {
    if (!h) return fail(GX_NULL_POINTER, "gx_pr_dist_run: null argument");
    if (iters < 1) return fail(GX_INVALID_VALUE, "gx_pr_dist_run: iters must be >= 1");
    PrDist &d = h->d;
    if (d.p2p && !d.attached) return fail(GX_INVALID_OBJECT, "gx_pr_dist_run: peer-to-peer runner not attached");
    // a token is run * kTok + step with step <= iters: a longer run would raise tokens that
    // satisfy the next run's waits early
    if (d.p2p && (uint64_t)iters >= kTok - 1) return fail(GX_INVALID_VALUE, "gx_pr_dist_run: at most 2^24 - 2 iterations with the peer-to-peer exchange");
    GX_HIP_TRY(hipSetDevice(d.ctx->device));
    return d.run(iters, use_graph != 0, stream ? (hipStream_t)stream : d.ctx->stream);
}

extern "C" int gx_pr_dist_scores(gx_pr_dist *h, int piece, double *scores) {
    if (!h || !scores) return fail(GX_NULL_POINTER, "gx_pr_dist_scores: null argument");
    PrDist &d = h->d;
    if (piece < 0 || piece >= (int)d.pieces.size()) return fail(GX_INVALID_INDEX, "gx_pr_dist_scores: bad piece");
    GX_HIP_TRY(hipSetDevice(d.ctx->device));
    if (d.last_stream) GX_HIP_TRY(hipStreamSynchronize(d.last_stream));
    if (d.p2p) {
        uint64_t err = 0;
        GX_HIP_TRY(hipMemcpy(&err, d.seq.p + 1, sizeof(err), hipMemcpyDeviceToHost));
        if (err) return fail(GX_DEVICE_ERROR, "gx_pr_dist_scores: a peer-to-peer wait timed out (a peer stopped or diverged)");
    }
    const uint64_t rows = d.pieces[piece]->rows;
    if (rows) GX_HIP_TRY(hipMemcpy(scores, d.ro[piece]->p, rows * sizeof(double), hipMemcpyDeviceToHost));
    return GX_SUCCESS;
}

// ---------------------------------------------------------------- one process, N GPUs

namespace {

// Adds src into dst (n words): the local reduction of Clique::reduce_sum_u64.
__global__ __launch_bounds__(256) void k_add_u64(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] += src[i];
}

bool one_device(gx_ctx *const *ctxs, int ndev) {
    for (int d = 1; d < ndev; d++)
        if (ctxs[d]->device != ctxs[0]->device) return false;
    return true;
}

// The exchange among the ndev contexts of a one-process multi-device call (gx_*_multi).
// Contexts on distinct devices form an in-process RCCL clique (ncclCommInitAll; xGMI between
// MI355X GPUs), every collective issued for all devices inside one group.  Two or more
// contexts that all sit on ONE device are virtual devices (bin/exe/* with GX_NGPUS=N and
// GX_MULTI_SIM=1): the same call, partition and kernels per virtual device, with each
// collective restated as device-to-device copies with its semantics -- every context's
// stream waits for every sender before the copies, and for every receiver after them, so a
// send buffer is never rewritten while a peer still reads it.  That runs the N > 1 code of
// gx_pagerank_multi / gx_sssp_multi / gx_lcc_multi on a one-GPU box.
// One context alone keeps a size-1 RCCL clique, so the RCCL path stays exercised there too.
struct Clique {
    static constexpr int kMaxPieces = 8;   // gx_pagerank_multi's pieces per device (events below)
    int ndev = 0;
    std::vector<gx_ctx *> ctx;
    std::vector<ncclComm_t> comm;
    bool local = false;
    std::vector<hipEvent_t> ev_in, ev_out;
    // per device: a comm stream (the pieces' exchanges overlap the next piece's SpMV on the
    // compute stream), an event per piece (its SpMV done) and one for the iteration's
    // exchanges (made here, by gx_multi_prepare, outside the processing time: creating a stream
    // cost 10-30 ms inside a call)
    std::vector<hipStream_t> cs;
    std::vector<hipEvent_t> ev_piece, ev_comm;

    ~Clique() {
        for (int d = 0; d < ndev; d++) {
            (void)hipSetDevice(ctx[d]->device);
            (void)hipStreamSynchronize(ctx[d]->stream);
            if (d < (int)cs.size() && cs[d]) (void)hipStreamSynchronize(cs[d]);
        }
        for (ncclComm_t c : comm)
            if (c) (void)rccl().comm_destroy(c);
        for (hipEvent_t e : ev_in) (void)hipEventDestroy(e);
        for (hipEvent_t e : ev_out) (void)hipEventDestroy(e);
        for (hipEvent_t e : ev_piece)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : ev_comm)
            if (e) (void)hipEventDestroy(e);
        for (int d = 0; d < (int)cs.size(); d++)
            if (cs[d]) {
                (void)hipSetDevice(ctx[d]->device);
                (void)hipStreamDestroy(cs[d]);
            }
    }

    int init(gx_ctx *const *ctxs, int n) {
        ndev = n;
        ctx.assign(ctxs, ctxs + n);
        local = n > 1 && one_device(ctxs, n);
        cs.assign(n, nullptr);
        ev_comm.assign(n, nullptr);
        ev_piece.assign((size_t)n * kMaxPieces, nullptr);
        for (int d = 0; d < n; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_HIP_TRY(hipStreamCreateWithFlags(&cs[d], hipStreamNonBlocking));
            GX_HIP_TRY(hipEventCreateWithFlags(&ev_comm[d], hipEventDisableTiming));
            for (int p = 0; p < kMaxPieces; p++)
                GX_HIP_TRY(hipEventCreateWithFlags(&ev_piece[(size_t)d * kMaxPieces + p], hipEventDisableTiming));
        }
        if (!local) {
            std::vector<int> devs(n);
            for (int d = 0; d < n; d++) devs[d] = ctxs[d]->device;
            comm.assign(n, nullptr);
            GX_NCCL_TRY("ncclCommInitAll", rccl().comm_init_all(comm.data(), n, devs.data()));
            return GX_SUCCESS;
        }
        GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
        ev_in.assign(n, nullptr);
        ev_out.assign(n, nullptr);
        for (int d = 0; d < n; d++) {
            GX_HIP_TRY(hipEventCreateWithFlags(&ev_in[d], hipEventDisableTiming));
            GX_HIP_TRY(hipEventCreateWithFlags(&ev_out[d], hipEventDisableTiming));
        }
        return GX_SUCCESS;
    }

    hipStream_t st(int d) const { return ctx[d]->stream; }

    // local mode: every stream of `sel` waits for what every such stream has enqueued so far
    template <class Sel>
    int fence_in(Sel sel) {
        for (int e = 0; e < ndev; e++) GX_HIP_TRY(hipEventRecord(ev_in[e], sel(e)));
        for (int d = 0; d < ndev; d++)
            for (int e = 0; e < ndev; e++)
                if (e != d) GX_HIP_TRY(hipStreamWaitEvent(sel(d), ev_in[e], 0));
        return GX_SUCCESS;
    }
    template <class Sel>
    int fence_out(Sel sel) {
        for (int d = 0; d < ndev; d++) GX_HIP_TRY(hipEventRecord(ev_out[d], sel(d)));
        for (int e = 0; e < ndev; e++)
            for (int d = 0; d < ndev; d++)
                if (d != e) GX_HIP_TRY(hipStreamWaitEvent(sel(e), ev_out[d], 0));
        return GX_SUCCESS;
    }
    int fence_in() {
        return fence_in([&](int d) { return st(d); });
    }
    int fence_out() {
        return fence_out([&](int d) { return st(d); });
    }

    // recv(d)[e * bytes, (e + 1) * bytes) = send(e)[0, bytes) for every pair (ncclAllGather),
    // on the compute streams
    template <class S, class R>
    int all_gather(S send, R recv, size_t bytes) {
        return all_gather_on(send, recv, bytes, [&](int d) { return st(d); });
    }

    // the same on the streams sel(d) (the comm streams for gx_pagerank_multi's pieces)
    template <class S, class R, class Sel>
    int all_gather_on(S send, R recv, size_t bytes, Sel sel) {
        if (local) {
            GX_HIP_TRY(hipSetDevice(ctx[0]->device));
            GX_TRY(fence_in(sel));
            for (int d = 0; d < ndev; d++)
                for (int e = 0; e < ndev; e++)
                    GX_HIP_TRY(hipMemcpyAsync(static_cast<char *>(recv(d)) + (size_t)e * bytes, send(e), bytes,
                                              hipMemcpyDeviceToDevice, sel(d)));
            return fence_out(sel);
        }
        const Rccl &r = rccl();
        GX_NCCL_TRY("ncclGroupStart", r.group_start());
        for (int d = 0; d < ndev; d++) {
            const ncclResult_t e = r.all_gather(send(d), recv(d), bytes, ncclUint8, comm[d], sel(d));
            if (e != ncclSuccess) {
                (void)r.group_end();
                return rccl_fail("ncclAllGather", e);
            }
        }
        GX_NCCL_TRY("ncclGroupEnd", r.group_end());
        return GX_SUCCESS;
    }

    // buf(0)[i] = sum over d of buf(d)[i], i < count (ncclReduce, root 0, in place there); the
    // other devices' buffers are left as they were in local mode, undefined under RCCL
    template <class B>
    int reduce_sum_u64(B buf, size_t count) {
        if (local) {
            GX_HIP_TRY(hipSetDevice(ctx[0]->device));
            GX_TRY(fence_in());
            for (int e = 1; e < ndev && count; e++) {
                hipLaunchKernelGGL(k_add_u64, dim3(grid_for(count, 256, 8192)), dim3(256), 0, st(0), buf(0), buf(e),
                                   (uint64_t)count);
                GX_TRY(check_launch("k_add_u64"));
            }
            return fence_out();
        }
        const Rccl &r = rccl();
        GX_NCCL_TRY("ncclGroupStart", r.group_start());
        for (int d = 0; d < ndev; d++) {
            const ncclResult_t e = r.reduce(buf(d), buf(d), count, ncclUint64, ncclSum, 0, comm[d], st(d));
            if (e != ncclSuccess) {
                (void)r.group_end();
                return rccl_fail("ncclReduce", e);
            }
        }
        GX_NCCL_TRY("ncclGroupEnd", r.group_end());
        return GX_SUCCESS;
    }
};

// The cliques of gx_*_multi, one per context list, kept until one of its contexts is freed
// (forget_cliques from gx_free): ncclCommInitAll took ~0.5 s of every call.  gx_multi_prepare
// makes one ahead of the caller's timed region, as gx_init does for a context.
struct CliqueCache {
    std::mutex mu;
    std::vector<std::pair<std::vector<gx_ctx *>, std::shared_ptr<Clique>>> list;
};
// never destroyed: an exit-time destructor would tear down communicators after the HIP runtime
CliqueCache &cliques() {
    static CliqueCache *c = new CliqueCache;
    return *c;
}

int get_clique(gx_ctx *const *ctxs, int n, std::shared_ptr<Clique> *out) {
    CliqueCache &cc = cliques();
    std::lock_guard<std::mutex> lk(cc.mu);
    const std::vector<gx_ctx *> key(ctxs, ctxs + n);
    for (auto &e : cc.list)
        if (e.first == key) {
            *out = e.second;
            return GX_SUCCESS;
        }
    auto c = std::make_shared<Clique>();
    GX_TRY(c->init(ctxs, n));
    cc.list.push_back({key, c});
    *out = c;
    return GX_SUCCESS;
}


// The in-process run of gx_pagerank_multi: per device its full vectors (xr, xw) and, per piece
// (index d * npieces + p), a PrPart, its local chunk and its scores.
struct MultiRun {
    int ndev = 0, npieces = 1;
    std::vector<gx_ctx *> ctx;
    std::vector<PrPart *> part;
    std::vector<std::unique_ptr<DBuf<double>>> xr, xw, xl, ro;
    uint64_t chunk = 0;

    ~MultiRun() {
        for (int d = 0; d < ndev; d++) {
            (void)hipSetDevice(ctx[d]->device);
            (void)hipStreamSynchronize(ctx[d]->stream);
        }
        for (int d = 0; d < ndev; d++) {
            (void)hipSetDevice(ctx[d]->device);
            for (int p = 0; p < npieces; p++) {
                const size_t k = (size_t)d * npieces + p;
                if (k < part.size()) delete part[k];
                if (k < xl.size()) xl[k].reset();
                if (k < ro.size()) ro[k].reset();
            }
            if (d < (int)xr.size()) xr[d].reset();
            if (d < (int)xw.size()) xw[d].reset();
        }
    }
};

// Run fn(d) for every device on a host thread of its own (its device current, an equal share
// of the host's OpenMP threads), so the devices' uploads and plans overlap; one device runs
// inline.  Virtual devices (every context on one device) run one after the other on the
// calling thread, each drained before the next: they share the device's grow-only sort and
// plan scratch (gx_runtime.hip), which one host thread at a time may use.  The first
// failure's code and message come back on the calling thread.
template <class F>
int per_device(gx_ctx *const *ctxs, int ndev, F fn) {
    if (ndev == 1 || one_device(ctxs, ndev)) {
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            const int rc = fn(d);
            if (rc != GX_SUCCESS)
                return ndev == 1 ? rc : fail(rc, "virtual device " + std::to_string(d) + ": " + gx_last_error());
            GX_HIP_TRY(hipStreamSynchronize(ctxs[d]->stream));
        }
        return GX_SUCCESS;
    }
    std::vector<int> rc(ndev, GX_SUCCESS);
    std::vector<std::string> msg(ndev);
    std::vector<std::thread> th;
    const int share = std::max(1, host_threads() / ndev);
    for (int d = 0; d < ndev; d++)
        th.emplace_back([&, d] {
            host_set_threads(share);
            const hipError_t e = hipSetDevice(ctxs[d]->device);
            rc[d] = e == hipSuccess ? fn(d) : fail(GX_DEVICE_ERROR, hipGetErrorString(e));
            if (rc[d] != GX_SUCCESS) msg[d] = gx_last_error();
        });
    for (auto &t : th) t.join();
    for (int d = 0; d < ndev; d++)
        if (rc[d] != GX_SUCCESS) return fail(rc[d], "device " + std::to_string(ctxs[d]->device) + ": " + msg[d]);
    return GX_SUCCESS;
}

// Contexts must be all on distinct devices (an RCCL clique) or all on one device (virtual
// devices exchanging by copies); RCCL is required for the former and for one context.
int check_ctxs(gx_ctx *const *ctxs, int ndev, const char *who);
int check_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, const char *who) {
    if (!ctxs || !A || (A->nnz && !A->colidx) || !A->rowptr) return fail(GX_NULL_POINTER, std::string(who) + ": null argument");
    return check_ctxs(ctxs, ndev, who);
}
int check_ctxs(gx_ctx *const *ctxs, int ndev, const char *who) {
    if (!ctxs) return fail(GX_NULL_POINTER, std::string(who) + ": null argument");
    if (ndev < 1) return fail(GX_INVALID_VALUE, std::string(who) + ": ndev < 1");
    for (int d = 0; d < ndev; d++)
        if (!ctxs[d]) return fail(GX_NULL_POINTER, std::string(who) + ": null context");
    for (int d = 0; d < ndev; d++)
        for (int e = 0; e < d; e++)
            if (ctxs[d] == ctxs[e]) return fail(GX_INVALID_VALUE, std::string(who) + ": a context passed twice");
    if (ndev > 1 && one_device(ctxs, ndev)) return GX_SUCCESS;
    for (int d = 0; d < ndev; d++)
        for (int e = 0; e < d; e++)
            if (ctxs[d]->device == ctxs[e]->device)
                return fail(GX_INVALID_VALUE, std::string(who) + ": contexts must be on distinct devices, or all on one");
    const Rccl &r = rccl();
    if (!r.ok) return fail(GX_NOT_IMPLEMENTED, r.error);
    return GX_SUCCESS;
}

// The graphs of a multi-device call: A on every device (gx_graph_create validates it there),
// freed with their contexts' streams drained.
struct MultiGraphs {
    std::vector<gx_graph *> g;
    ~MultiGraphs() {
        for (gx_graph *x : g) (void)gx_graph_free(x);
    }
};

}  // namespace

void gx::forget_cliques(gx_ctx *ctx) {
    std::vector<std::shared_ptr<Clique>> drop;  // destroyed outside the lock
    CliqueCache &cc = cliques();
    {
        std::lock_guard<std::mutex> lk(cc.mu);
        for (size_t i = 0; i < cc.list.size();) {
            auto &k = cc.list[i].first;
            if (std::find(k.begin(), k.end(), ctx) != k.end()) {
                drop.push_back(std::move(cc.list[i].second));
                cc.list.erase(cc.list.begin() + i);
            } else {
                i++;
            }
        }
    }
}

extern "C" int gx_multi_prepare(gx_ctx *const *ctxs, int ndev) {
    GX_TRY(check_ctxs(ctxs, ndev, "gx_multi_prepare"));
    std::shared_ptr<Clique> clique;
    return get_clique(ctxs, ndev, &clique);
}

extern "C" int gx_pagerank_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, double damping,
                                 int iters, double *rank) {
    GX_TRY(check_multi(ctxs, ndev, A, "gx_pagerank_multi"));
    if (!rank) return fail(GX_NULL_POINTER, "gx_pagerank_multi: null argument");
    if (iters < 0) return fail(GX_INVALID_VALUE, "gx_pagerank_multi: negative iteration count");
    const uint64_t n = A->n;
    if (n == 0) return GX_SUCCESS;
    if (iters == 0) {
        for (uint64_t v = 0; v < n; v++) rank[v] = 1.0 / (double)n;
        return GX_SUCCESS;
    }
    if (n >= (1ull << 31) - 64) return fail(GX_NOT_IMPLEMENTED, "gx_pagerank_multi: n >= 2^31");
    // Pieces (round 6): every device's rows are cut into P pieces, each its
    // own plan and launch.  Piece p of every device runs, then its chunks are all-gathered on
    // the comm streams while piece p + 1 runs on the compute streams, so only the last piece's
    // exchange is exposed (1/P of it) instead of all of it.  Piece p of device d is virtual rank
    // p * ndev + d of V = ndev * P ranges: x's slab p (ndev chunks) is what piece p's all-gather
    // fills, the layout PrDist uses across processes.  GX_PR_MULTI_PIECES (1..8; default 2 for
    // several devices, 1 for one: at N = 1 there is no exchange to hide).
    int P = ndev > 1 ? 2 : 1;
    if (const char *e = std::getenv("GX_PR_MULTI_PIECES")) P = std::atoi(e);
    P = std::max(1, std::min(P, Clique::kMaxPieces));
    // one device, one piece: no exchange at all, so the single-GPU call itself (upload
    // overlapped with the plan, 24-bit columns: 77 ms on SYN-8_5 where this path's upload and
    // separate plan took 149)
    if (ndev == 1 && P == 1) return gx_pagerank_csr(ctxs[0], A, directed, damping, iters, rank, nullptr);
    const int V = ndev * P;
    PlanClock clk("multi_call", ctxs[0]->stream);
    // interleaved hub-first partition (pr_partition.interleaved_relabel): hub-first position i
    // goes to virtual rank i % V as its local row i / V.  The vertices with out-edges come first
    // in that order, so virtual rank 0 holds the most live rows, ceil(nlive / V): the chunk every
    // rank exchanges (+ the zero padding slot and the dangling slot).  The pull matrix of a
    // directed graph is A', whose rows with out-edges in the PageRank sense are still A's rows
    // with out-edges: liveness is A's out-degree either way.
    // A huge graph (more than 2 Mi entries per CU, the single-GPU plan's huge-graph cut) is
    // split by blocks instead (pr_multi_blocks; pr_partition.block_relabel): every virtual
    // rank's blocks are the single-GPU plan's own, so its gathers share x lines as the whole
    // graph's do (1/8 pieces of SYN-8_5: 140 us per SpMV against 208 interleaved).
    // GX_PR_MULTI_PARTITION=blocks / interleave overrides.
    const uint64_t nlive = host_count_live(A->rowptr, n);
    MultiRun M;
    M.ndev = ndev;
    M.npieces = P;
    M.chunk = ((nlive + V - 1) / V + 2 + 31) / 32 * 32;
    bool by_blocks = V > 1 && (double)A->rowptr[n] / (double)std::max(1, ctxs[0]->num_cus) > (double)(2 << 20);
    if (const char *e = std::getenv("GX_PR_MULTI_PARTITION")) by_blocks = std::strcmp(e, "blocks") == 0;
    // Partitioned upload (round 6; GX_PR_MULTI_UPLOAD=rows, the default for
    // undirected graphs, whose pull rows are A's own): the host deals the hub-first order once,
    // and every virtual rank's rows leave the 64-bit input once, for that rank's device only,
    // picked straight into the staging buffers (pr_part_build_rows); the plan's key pass renames
    // the columns into the exchange layout through a device column map.  "whole" (and every
    // directed graph, whose pull rows are A''s) uploads A to every device and plans there
    // (pr_multi_plan).
    bool by_rows = !directed;
    if (const char *e = std::getenv("GX_PR_MULTI_UPLOAD")) by_rows = by_rows && std::strcmp(e, "whole") != 0;
    if (const char *e = std::getenv("GX_PR_KERNEL")) by_rows = by_rows && std::strcmp(e, "adaptive") != 0;   // reads raw columns
    if (by_rows) {
        if (A->rowptr[0] != 0 || A->rowptr[n] != A->nnz || !host_monotone(A->rowptr, n))
            return fail(GX_INVALID_VALUE, "gx_pagerank_multi: inconsistent row pointers");
    }
    MultiBlocks mb;
    if (by_blocks) {
        GX_TRY(pr_multi_blocks(A, directed, V, &mb));
        M.chunk = mb.chunk;
    } else if (by_rows) {
        GX_TRY(pr_multi_interleave(A, V, &mb));
        if (mb.chunk != M.chunk) return fail(GX_PANIC, "gx_pagerank_multi: interleaved chunk mismatch");
    }
    if (M.chunk * (uint64_t)V >= (1ull << 31)) return fail(GX_NOT_IMPLEMENTED, "gx_pagerank_multi: exchange too large");
    M.ctx.assign(ctxs, ctxs + ndev);
    M.part.assign((size_t)V, nullptr);
    for (int d = 0; d < ndev; d++) {
        M.xr.emplace_back(new DBuf<double>());
        M.xw.emplace_back(new DBuf<double>());
    }
    for (int k = 0; k < V; k++) {
        M.xl.emplace_back(new DBuf<double>());
        M.ro.emplace_back(new DBuf<double>());
    }
    auto piece = [&](int d, int p) { return (size_t)d * P + p; };
    MultiGraphs G;
    G.g.assign(ndev, nullptr);
    std::vector<uint64_t> rows((size_t)V);
    // by_rows: the vertex of each local row of each piece (the scores' scatter), and the column
    // map vertex -> exchange slot
    std::vector<std::vector<int32_t>> vrows(by_rows ? (size_t)V : 0);
    std::vector<int32_t> colmap;
    std::vector<uint64_t> picked((size_t)V, 0);   // input columns each piece read
    std::vector<std::unique_ptr<DBuf<int32_t>>> cmap(by_rows ? ndev : 0);
    if (by_rows) {
        colmap.resize(n);
        host_compose(mb.slot.data(), mb.perm.data(), n, colmap.data());
    }
    clk.mark("partition (host)");
    // per device, on the device: upload A, A' if directed (LAGraph_Cached_AT, pr.cpp:60), the
    // hub-first order and each piece's plan (pr_multi_plan), the exchange buffers; or (by_rows)
    // each piece's own rows, picked on the host, and its plan
    GX_TRY(per_device(ctxs, ndev, [&](int d) -> int {
        if (!by_rows) {
            GX_TRY(gx_graph_create(ctxs[d], A, directed, &G.g[d]));
            if (directed) GX_TRY(ensure_transpose(G.g[d]));
        } else {
            // the column map, once per device (the pieces' key passes rename through it)
            cmap[d].reset(new DBuf<int32_t>());
            GX_TRY(cmap[d]->alloc(n));
            bool bad = false;
            GX_TRY(upload_staged(ctxs[d], cmap[d]->p, n, 4,
                                 [&](uint64_t off, uint64_t cnt, void *buf) {
                                     host_copy(buf, colmap.data() + off, cnt * 4);
                                     return true;
                                 }, &bad));
        }
        hipStream_t s = ctxs[d]->stream;
        for (int p = 0; p < P; p++) {
            const size_t k = piece(d, p);
            const int vr = p * ndev + d;
            if (by_rows) {
                std::vector<int32_t> &vs = vrows[k];
                const std::vector<int32_t> &pos = mb.pos[vr];
                vs.resize(pos.size());
                for (size_t j = 0; j < pos.size(); j++) vs[j] = mb.order[pos[j]];
                for (int32_t v : vs) picked[k] += A->rowptr[v + 1] - A->rowptr[v];
                GX_TRY(pr_part_build_rows(ctxs[d], A, V, vr, M.chunk, vs, cmap[d]->p, damping, by_blocks, &M.part[k]));
            } else {
                GX_TRY(pr_multi_plan(G.g[d], V, vr, M.chunk, damping, by_blocks ? &mb : nullptr, &M.part[k]));
            }
            rows[k] = M.part[k]->rows;
            GX_TRY(M.xl[k]->alloc(M.chunk));
            GX_TRY(M.ro[k]->alloc(std::max<uint64_t>(rows[k], 1)));
            GX_HIP_TRY(hipMemsetAsync(M.xl[k]->p, 0, M.chunk * sizeof(double), s));
        }
        const size_t full = M.chunk * (size_t)V;
        GX_TRY(M.xr[d]->alloc(full));
        GX_TRY(M.xw[d]->alloc(full));
        GX_HIP_TRY(hipMemsetAsync(M.xr[d]->p, 0, full * sizeof(double), s));
        GX_HIP_TRY(hipMemsetAsync(M.xw[d]->p, 0, full * sizeof(double), s));
        return GX_SUCCESS;
    }));
    clk.mark("devices: upload + plans");
    if (by_rows && std::getenv("GX_PLAN_TIMES")) {
        uint64_t tot = 0;
        for (uint64_t c : picked) tot += c;
        std::fprintf(stderr, "[multi] partitioned upload: %llu of %llu input columns read (%.3fx), %d devices x %d pieces\n",
                     (unsigned long long)tot, (unsigned long long)A->nnz, A->nnz ? (double)tot / (double)A->nnz : 0.0,
                     ndev, P);
    }
    std::shared_ptr<Clique> clique;
    GX_TRY(get_clique(ctxs, ndev, &clique));
    Clique &C = *clique;
    const size_t cbytes = M.chunk * sizeof(double), span = M.chunk * (size_t)ndev;
    // piece p's chunks into slab p of every device's dst, on the compute streams (init) or,
    // after each device's piece-p SpMV, on the comm streams
    auto gather = [&](int p, std::vector<std::unique_ptr<DBuf<double>>> &dst, bool on_comm) -> int {
        auto send = [&](int d) { return (const void *)M.xl[piece(d, p)]->p; };
        auto recv = [&](int d) { return (void *)(dst[d]->p + (size_t)p * span); };
        if (!on_comm) return C.all_gather(send, recv, cbytes);
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            hipEvent_t ev = C.ev_piece[(size_t)d * Clique::kMaxPieces + p];
            GX_HIP_TRY(hipEventRecord(ev, C.st(d)));
            GX_HIP_TRY(hipStreamWaitEvent(C.cs[d], ev, 0));
        }
        return C.all_gather_on(send, recv, cbytes, [&](int d) { return C.cs[d]; });
    };
    // the compute streams wait for every exchange issued on the comm streams
    auto join = [&]() -> int {
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_HIP_TRY(hipEventRecord(C.ev_comm[d], C.cs[d]));
            GX_HIP_TRY(hipStreamWaitEvent(C.st(d), C.ev_comm[d], 0));
        }
        return GX_SUCCESS;
    };
    for (int d = 0; d < ndev; d++) {
        GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
        for (int p = 0; p < P; p++) GX_TRY(pr_init(M.part[piece(d, p)], M.xl[piece(d, p)]->p, ctxs[d]->stream));
    }
    for (int p = 0; p < P; p++) GX_TRY(gather(p, M.xr, false));
    for (int it = 0; it < iters; it++) {
        const bool last = it == iters - 1;
        for (int p = 0; p < P; p++) {
            for (int d = 0; d < ndev; d++) {
                GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
                const size_t k = piece(d, p);
                GX_TRY(pr_step(M.part[k], M.xr[d]->p, M.xl[k]->p, last ? M.ro[k]->p : nullptr, ctxs[d]->stream));
            }
            if (!last) GX_TRY(gather(p, M.xw, true));
        }
        if (last) break;
        GX_TRY(join());
        std::swap(M.xr, M.xw);
    }
    clk.mark("iterations");
    // scores back in A's vertex order: piece k's local row j is vertex order_k[j]
    for (int d = 0; d < ndev; d++) {
        GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
        std::vector<std::vector<double>> buf(P);
        std::vector<std::vector<int32_t>> who(P);
        for (int p = 0; p < P; p++) {
            const size_t k = piece(d, p);
            buf[p].resize(rows[k]);
            who[p].resize(rows[k]);
            if (rows[k]) {
                GX_HIP_TRY(hipMemcpyAsync(buf[p].data(), M.ro[k]->p, rows[k] * sizeof(double), hipMemcpyDeviceToHost,
                                          ctxs[d]->stream));
                if (by_rows)
                    std::copy(vrows[k].begin(), vrows[k].end(), who[p].begin());
                else
                    GX_HIP_TRY(hipMemcpyAsync(who[p].data(), M.part[k]->order.p, rows[k] * sizeof(int32_t),
                                              hipMemcpyDeviceToHost, ctxs[d]->stream));
            }
        }
        GX_HIP_TRY(hipStreamSynchronize(ctxs[d]->stream));
        for (int p = 0; p < P; p++)
            for (uint64_t j = 0; j < buf[p].size(); j++) rank[who[p][j]] = buf[p][j];
    }
    clk.mark("scores");
    return GX_SUCCESS;
}

// Multi-device SSSP in one process (bin/exe/sssp with GX_NGPUS; config 4's other half): the
// 1-D split of gx_sssp_split on every device, the rounds exchanged by the clique.
// Device d owns the targets [ranges[d], ranges[d+1]) (contiguous, ~nnz / ndev stored entries
// each); per round: every device relaxes into its owned vertices, the 2-word counts
// {pairs, done} are all-gathered and read by the host (the only host read of a round), then
// max-count pairs of every device are all-gathered and applied everywhere.  The decisions
// come from replicated state, so every device stops at the same round; a disagreement is an
// error, not a silent stop.
extern "C" int gx_sssp_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, uint64_t src,
                             double *dist) {
    GX_TRY(check_multi(ctxs, ndev, A, "gx_sssp_multi"));
    if (!dist) return fail(GX_NULL_POINTER, "gx_sssp_multi: null argument");
    if (!A->vals) return fail(GX_INVALID_VALUE, "gx_sssp_multi: graph has no edge weights");
    const uint64_t n = A->n, nnz = A->nnz;
    if (src >= n) return fail(GX_INVALID_INDEX, "gx_sssp_multi: source out of range");
    std::vector<uint64_t> ranges(ndev + 1, 0);
    for (int k = 1; k < ndev; k++) {   // pr_partition.partition_rows: ~nnz / ndev entries each
        const uint64_t target = nnz / ndev * k + nnz % ndev * k / ndev;
        const uint64_t r = (uint64_t)(std::lower_bound(A->rowptr, A->rowptr + n + 1, target) - A->rowptr);
        ranges[k] = std::min(std::max(r, ranges[k - 1]), n);
    }
    ranges[ndev] = n;
    uint64_t maxown = 1;
    for (int d = 0; d < ndev; d++) maxown = std::max(maxown, ranges[d + 1] - ranges[d]);
    MultiGraphs G;
    G.g.assign(ndev, nullptr);
    struct Dev {
        gx_sssp_split *sp = nullptr;
        DBuf<uint64_t> pairs, count, counts, all;
    };
    std::vector<Dev> D(ndev);
    uint64_t *hc = nullptr;
    // released in this order on every exit: the splits and buffers on their devices, the
    // pinned words (the clique is destroyed before, the graphs after, with G)
    struct Cleanup {
        gx_ctx *const *ctxs;
        std::vector<Dev> &D;
        uint64_t *&hc;
        ~Cleanup() {
            for (size_t d = 0; d < D.size(); d++) {
                (void)hipSetDevice(ctxs[d]->device);
                (void)hipStreamSynchronize(ctxs[d]->stream);
                (void)gx_sssp_split_free(D[d].sp);
                D[d].sp = nullptr;
                D[d].pairs.release();
                D[d].count.release();
                D[d].counts.release();
                D[d].all.release();
            }
            if (hc) (void)hipHostFree(hc);
        }
    } cleanup{ctxs, D, hc};
    GX_TRY(per_device(ctxs, ndev, [&](int d) -> int {
        GX_TRY(gx_graph_create(ctxs[d], A, directed, &G.g[d]));
        GX_TRY(gx_sssp_split_create(G.g[d], ranges[d], ranges[d + 1], &D[d].sp));
        GX_TRY(D[d].pairs.alloc(2 * maxown));
        GX_TRY(D[d].count.alloc(2));
        GX_TRY(D[d].counts.alloc(2 * (uint64_t)ndev));
        GX_TRY(D[d].all.alloc(2 * maxown * (uint64_t)ndev));
        return GX_SUCCESS;
    }));
    std::shared_ptr<Clique> clique;
    GX_TRY(get_clique(ctxs, ndev, &clique));
    Clique &C = *clique;
    GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
    GX_HIP_TRY(hipHostMalloc((void **)&hc, 2 * (size_t)ndev * sizeof(uint64_t), hipHostMallocDefault));
    for (int d = 0; d < ndev; d++) {
        GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
        GX_TRY(gx_sssp_split_start(D[d].sp, src, ctxs[d]->stream));
    }
    for (uint64_t round = 0;; round++) {
        if (round > 4 * (n + 16)) return fail(GX_DEVICE_ERROR, "gx_sssp_multi: no fixed point");
        for (int d = 0; d < ndev; d++)
            GX_TRY(gx_sssp_split_relax(D[d].sp, D[d].pairs.p, D[d].count.p, ctxs[d]->stream));
        GX_TRY(C.all_gather([&](int d) { return (const void *)D[d].count.p; },
                            [&](int d) { return (void *)D[d].counts.p; }, 2 * sizeof(uint64_t)));
        GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
        GX_HIP_TRY(hipMemcpyAsync(hc, D[0].counts.p, 2 * (size_t)ndev * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                  ctxs[0]->stream));
        GX_HIP_TRY(hipStreamSynchronize(ctxs[0]->stream));
        int ndone = 0;
        uint64_t m = 0;
        for (int d = 0; d < ndev; d++) {
            ndone += hc[2 * d + 1] != 0;
            m = std::max(m, hc[2 * d]);
        }
        if (ndone == ndev) break;
        if (ndone) {
            // a device that stopped alone stopped on an error (a full settled list):
            // report that cause rather than the disagreement it led to
            for (int d = 0; d < ndev; d++)
                if (hc[2 * d + 1]) {
                    GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
                    GX_TRY(sssp_split_check(D[d].sp, ctxs[d]->stream));
                }
            return fail(GX_DEVICE_ERROR, "gx_sssp_multi: devices disagree on termination");
        }
        if (m > maxown) return fail(GX_DEVICE_ERROR, "gx_sssp_multi: pair count beyond the owned range");
        if (m)
            GX_TRY(C.all_gather([&](int d) { return (const void *)D[d].pairs.p; },
                                [&](int d) { return (void *)D[d].all.p; }, 2 * m * sizeof(uint64_t)));
        for (int d = 0; d < ndev; d++)
            GX_TRY(gx_sssp_split_apply(D[d].sp, m ? D[d].all.p : D[d].pairs.p, D[d].counts.p, ndev, m,
                                       ctxs[d]->stream));
    }
    // the distance vector is replicated: device 0's, in A's vertex order
    GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
    DBuf<double> out;
    GX_TRY(out.alloc(std::max<uint64_t>(n, 1)));
    GX_TRY(gx_sssp_split_distances(D[0].sp, out.p, ctxs[0]->stream));
    GX_HIP_TRY(hipStreamSynchronize(ctxs[0]->stream));
    GX_TRY(download(ctxs[0], dist, out.p, n, Xfer::Raw64));
    return GX_SUCCESS;
}

// Multi-device LCC in one process (bin/exe/lcc with GX_NGPUS; BASELINE config 5, "LCC on
// cit-Patents, 1 -> 8 GPUs"): A is replicated, every device builds the degree orientation
// (gx_lcc_part_create) and counts the triangles whose middle vertex lies in its range of
// orientation sources, the ranges balanced by the probe work sum |O(v)| over in-neighbours
// (gx_lcc_part_ranges); the n triangle counters of all devices are summed onto device 0 by one
// reduction, which divides by the closure degree there (gx_lcc_part_finish).  The counters are
// integers, so the result is bit-identical to gx_lcc whatever the split.  Replaces LA_LCC
// (lcc.cpp:61-71) when it runs on several GPUs.
extern "C" int gx_lcc_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, double *lcc) {
    GX_TRY(check_multi(ctxs, ndev, A, "gx_lcc_multi"));
    if (!lcc) return fail(GX_NULL_POINTER, "gx_lcc_multi: null argument");
    const uint64_t n = A->n;
    if (n == 0) return GX_SUCCESS;
    if (n >= (1ull << 29)) return fail(GX_NOT_IMPLEMENTED, "gx_lcc_multi: more than 2^29 vertices (packed oriented entries)");
    MultiGraphs G;
    G.g.assign(ndev, nullptr);
    struct Dev {
        gx_lcc_part *part = nullptr;
        DBuf<uint64_t> tc;
    };
    std::vector<Dev> D(ndev);
    struct Cleanup {
        gx_ctx *const *ctxs;
        std::vector<Dev> &D;
        ~Cleanup() {
            for (size_t d = 0; d < D.size(); d++) {
                (void)hipSetDevice(ctxs[d]->device);
                (void)hipStreamSynchronize(ctxs[d]->stream);
                (void)gx_lcc_part_free(D[d].part);
                D[d].part = nullptr;
                D[d].tc.release();
            }
        }
    } cleanup{ctxs, D};
    GX_TRY(per_device(ctxs, ndev, [&](int d) -> int {
        GX_TRY(gx_graph_create(ctxs[d], A, directed, &G.g[d]));
        GX_TRY(gx_lcc_part_create(G.g[d], &D[d].part));
        GX_TRY(D[d].tc.alloc(n));
        return GX_SUCCESS;
    }));
    std::vector<uint64_t> ranges(ndev + 1);
    GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
    GX_TRY(gx_lcc_part_ranges(D[0].part, ndev, ranges.data()));
    GX_TRY(per_device(ctxs, ndev, [&](int d) -> int {
        GX_HIP_TRY(hipMemsetAsync(D[d].tc.p, 0, n * sizeof(uint64_t), ctxs[d]->stream));
        return gx_lcc_part_counts(D[d].part, ranges[d], ranges[d + 1], D[d].tc.p, ctxs[d]->stream);
    }));
    {
        std::shared_ptr<Clique> clique;
        GX_TRY(get_clique(ctxs, ndev, &clique));
        Clique &C = *clique;
        GX_TRY(C.reduce_sum_u64([&](int d) { return D[d].tc.p; }, n));
    }
    GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
    DBuf<double> out;
    GX_TRY(out.alloc(n));
    GX_TRY(gx_lcc_part_finish(D[0].part, D[0].tc.p, out.p, ctxs[0]->stream));
    GX_HIP_TRY(hipStreamSynchronize(ctxs[0]->stream));
    GX_TRY(download(ctxs[0], lcc, out.p, n, Xfer::Raw64));
    return GX_SUCCESS;
}

// ---- BFS / WCC / CDLP on several devices in one process (round 6) ----
// bin/exe/{bfs,wcc,cdlp} with GX_NGPUS: the graph replicated on every device, device d owning
// the vertex range [ranges[d], ranges[d+1]) (~nnz / ndev stored entries each), the rounds of
// distributed.py (the torch.distributed driver) restated over the in-process clique: every
// device runs its step on its own range, then only what the step changed travels as
// (v << 32 | value) words (gx_part_changes: the counts all-gathered and read by the host, the
// first max-count words of every device all-gathered, gx_part_apply on every device), or the
// dense form when the words would outweigh it.  Every device starts a round with the same
// state, so every device takes the same decisions; results are device 0's copy.
namespace {

std::vector<uint64_t> entry_ranges(const gx_csr *A, int ndev) {
    const uint64_t n = A->n, nnz = A->nnz;
    std::vector<uint64_t> ranges(ndev + 1, 0);
    for (int k = 1; k < ndev; k++) {   // pr_partition.partition_rows: ~nnz / ndev entries each
        const uint64_t target = nnz / ndev * k + nnz % ndev * k / ndev;
        const uint64_t r = (uint64_t)(std::lower_bound(A->rowptr, A->rowptr + n + 1, target) - A->rowptr);
        ranges[k] = std::min(std::max(r, ranges[k - 1]), n);
    }
    ranges[ndev] = n;
    return ranges;
}

// Per-device buffers of the word exchange; `cap` words per device (any step changes at most n
// entries), the gathered words grown on demand.
struct WordExchange {
    struct Dev {
        DBuf<uint64_t> words, gathered;
        DBuf<int64_t> count, counts;
        uint64_t gcap = 0;
    };
    std::vector<Dev> D;
    int64_t *hc = nullptr;   // pinned: the all-gathered counts (device 0's copy)
    int ndev = 0;
    gx_ctx *const *ctxs = nullptr;
    uint64_t rounds = 0, word_rounds = 0, word_bytes = 0, dense_bytes = 0;

    ~WordExchange() {
        for (int d = 0; d < ndev; d++) {
            (void)hipSetDevice(ctxs[d]->device);
            (void)hipStreamSynchronize(ctxs[d]->stream);
            D[d].words.release();
            D[d].gathered.release();
            D[d].count.release();
            D[d].counts.release();
        }
        if (hc) (void)hipHostFree(hc);
    }
    int init(gx_ctx *const *c, int nd, uint64_t cap) {
        ctxs = c;
        ndev = nd;
        D = std::vector<Dev>(nd);
        for (int d = 0; d < nd; d++) {
            GX_HIP_TRY(hipSetDevice(c[d]->device));
            GX_TRY(D[d].words.alloc(std::max<uint64_t>(cap, 1)));
            GX_TRY(D[d].count.alloc(1));
            GX_TRY(D[d].counts.alloc(nd));
        }
        GX_HIP_TRY(hipSetDevice(c[0]->device));
        GX_HIP_TRY(hipHostMalloc((void **)&hc, (size_t)nd * sizeof(int64_t), hipHostMallocDefault));
        return GX_SUCCESS;
    }
    // arr(d)'s entries in span(d) that differ from old(d) (null: from 0) -> every device's dst(d)
    // with op; dense() instead when 8 max-count ndev bytes exceed dense_bytes (GX_EXCHANGE =
    // sparse / dense forces one; dense_bytes ~0: no dense form).  *total = changes over all devices (0: none anywhere).
    template <class Arr, class Old, class Span, class Dst, class Dense>
    int run(Clique &C, Arr arr, Old old, Span span, int elem, int op, uint64_t dense_bytes, Dense dense, Dst dst,
            uint64_t *total) {
        rounds++;
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            const auto sp = span(d);
            GX_TRY(gx_part_changes(arr(d), old(d), sp.first, sp.second, elem, D[d].words.p, D[d].count.p,
                                   ctxs[d]->stream));
        }
        GX_TRY(C.all_gather([&](int d) { return (const void *)D[d].count.p; },
                            [&](int d) { return (void *)D[d].counts.p; }, sizeof(int64_t)));
        GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
        GX_HIP_TRY(hipMemcpyAsync(hc, D[0].counts.p, (size_t)ndev * sizeof(int64_t), hipMemcpyDeviceToHost,
                                  ctxs[0]->stream));
        GX_HIP_TRY(hipStreamSynchronize(ctxs[0]->stream));
        uint64_t m = 0, tot = 0;
        for (int d = 0; d < ndev; d++) {
            m = std::max<uint64_t>(m, (uint64_t)hc[d]);
            tot += (uint64_t)hc[d];
        }
        *total = tot;
        if (m == 0) return GX_SUCCESS;
        const char *ex = std::getenv("GX_EXCHANGE");
        const bool force_dense = ex && std::strcmp(ex, "dense") == 0, force_sparse = ex && std::strcmp(ex, "sparse") == 0;
        // (dense_bytes ~0: the caller has no dense form, words always)
        if (dense_bytes != ~0ull && (force_dense || (!force_sparse && 8 * m * (uint64_t)ndev > dense_bytes))) {
            dense_bytes_add(dense_bytes);
            return dense();
        }
        word_rounds++;
        word_bytes += 8 * m * (uint64_t)ndev;
        for (int d = 0; d < ndev; d++) {
            if (D[d].gcap < m * (uint64_t)ndev) {
                GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
                GX_HIP_TRY(hipStreamSynchronize(ctxs[d]->stream));   // the old buffer may still be read
                D[d].gathered.release();
                D[d].gcap = std::max<uint64_t>(m * (uint64_t)ndev, 2 * D[d].gcap);
                GX_TRY(D[d].gathered.alloc(D[d].gcap));
            }
        }
        GX_TRY(C.all_gather([&](int d) { return (const void *)D[d].words.p; },
                            [&](int d) { return (void *)D[d].gathered.p; }, m * sizeof(uint64_t)));
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_TRY(gx_part_apply(D[d].gathered.p, D[d].counts.p, ndev, m, dst(d), elem, op, ctxs[d]->stream));
        }
        return GX_SUCCESS;
    }
    void dense_bytes_add(uint64_t b) { dense_bytes += b; }
    void report(const char *who) const {
        if (std::getenv("GX_PLAN_TIMES"))
            std::fprintf(stderr, "[%s] %llu rounds, %llu as words (%.1f MB), dense %.1f MB per device\n", who,
                         (unsigned long long)rounds, (unsigned long long)word_rounds, word_bytes / 1e6 / ndev,
                         dense_bytes / 1e6);
    }
};

// A replicated per-device array of n elements (device buffers, freed on their devices).
template <class T>
struct PerDev {
    std::vector<DBuf<T>> b;
    gx_ctx *const *ctxs = nullptr;
    int ndev = 0;
    ~PerDev() {
        for (int d = 0; d < ndev; d++) {
            (void)hipSetDevice(ctxs[d]->device);
            (void)hipStreamSynchronize(ctxs[d]->stream);
            b[d].release();
        }
    }
    int alloc(gx_ctx *const *c, int nd, uint64_t n) {
        ctxs = c;
        ndev = nd;
        b = std::vector<DBuf<T>>(nd);
        for (int d = 0; d < nd; d++) {
            GX_HIP_TRY(hipSetDevice(c[d]->device));
            GX_TRY(b[d].alloc(std::max<uint64_t>(n, 1)));
        }
        return GX_SUCCESS;
    }
    T *operator[](int d) { return b[d].p; }
};

int upload_replicas(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, MultiGraphs &G) {
    G.g.assign(ndev, nullptr);
    return per_device(ctxs, ndev, [&](int d) -> int { return gx_graph_create(ctxs[d], A, directed, &G.g[d]); });
}

}  // namespace

extern "C" int gx_bfs_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, uint64_t src,
                            int64_t *level) {
    GX_TRY(check_multi(ctxs, ndev, A, "gx_bfs_multi"));
    if (!level) return fail(GX_NULL_POINTER, "gx_bfs_multi: null argument");
    const uint64_t n = A->n;
    if (src >= n) return fail(GX_INVALID_INDEX, "gx_bfs_multi: source out of range");
    const std::vector<uint64_t> ranges = entry_ranges(A, ndev);
    MultiGraphs G;
    GX_TRY(upload_replicas(ctxs, ndev, A, directed, G));
    std::shared_ptr<Clique> clique;
    GX_TRY(get_clique(ctxs, ndev, &clique));
    Clique &C = *clique;
    const uint64_t nw = (n + 31) / 32;
    PerDev<int64_t> lv, cnt;
    PerDev<uint8_t> nxt;
    PerDev<uint32_t> bits, gbits;
    GX_TRY(lv.alloc(ctxs, ndev, n));
    GX_TRY(cnt.alloc(ctxs, ndev, 1));
    GX_TRY(nxt.alloc(ctxs, ndev, (n + 15) / 16 * 16));   // 16-B multiple (gx_part_pack_bits)
    GX_TRY(bits.alloc(ctxs, ndev, nw));
    GX_TRY(gbits.alloc(ctxs, ndev, nw * (uint64_t)ndev));
    WordExchange X;
    GX_TRY(X.init(ctxs, ndev, n));
    for (int d = 0; d < ndev; d++) {
        GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
        GX_TRY(gx_bfs_part_init(G.g[d], src, lv[d], ctxs[d]->stream));
    }
    // dense form: every device's bitmap all-gathered and OR-ed (ndev n / 8 bytes < 2 n below 16)
    const uint64_t dense_bytes = (uint64_t)ndev * nw * 4;
    auto dense = [&]() -> int {
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_TRY(gx_part_pack_bits(nxt[d], n, bits[d], ctxs[d]->stream));
        }
        GX_TRY(C.all_gather([&](int d) { return (const void *)bits[d]; }, [&](int d) { return (void *)gbits[d]; },
                            nw * sizeof(uint32_t)));
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_TRY(gx_part_or_bits(gbits[d], ndev, n, nxt[d], ctxs[d]->stream));
        }
        return GX_SUCCESS;
    };
    int64_t hcount = 0;
    for (int64_t cur = 0;; cur++) {
        if ((uint64_t)cur > n + 1) return fail(GX_DEVICE_ERROR, "gx_bfs_multi: no fixed point");
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_HIP_TRY(hipMemsetAsync(nxt[d], 0, n, ctxs[d]->stream));
            GX_TRY(gx_bfs_part_expand(G.g[d], ranges[d], ranges[d + 1], lv[d], cur, nxt[d], ctxs[d]->stream));
        }
        uint64_t tot = 0;
        GX_TRY(X.run(C, [&](int d) { return (const void *)nxt[d]; }, [&](int) { return (const void *)nullptr; },
                     [&](int) { return std::make_pair((uint64_t)0, n); }, 1, 0, dense_bytes, dense,
                     [&](int d) { return (void *)nxt[d]; }, &tot));
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_HIP_TRY(hipMemsetAsync(cnt[d], 0, sizeof(int64_t), ctxs[d]->stream));   // commit adds to it
            GX_TRY(gx_bfs_part_commit(G.g[d], nxt[d], lv[d], cur, reinterpret_cast<uint64_t *>(cnt[d]),
                                      ctxs[d]->stream));
        }
        GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
        GX_HIP_TRY(hipMemcpyAsync(&hcount, cnt[0], sizeof(int64_t), hipMemcpyDeviceToHost, ctxs[0]->stream));
        GX_HIP_TRY(hipStreamSynchronize(ctxs[0]->stream));
        if (hcount == 0) break;   // identical on every device (same inputs)
    }
    X.report("bfs_multi");
    GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
    return download(ctxs[0], level, lv[0], n, Xfer::Raw64);
}

extern "C" int gx_wcc_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, uint64_t *comp) {
    GX_TRY(check_multi(ctxs, ndev, A, "gx_wcc_multi"));
    if (!comp) return fail(GX_NULL_POINTER, "gx_wcc_multi: null argument");
    const uint64_t n = A->n;
    if (n == 0) return GX_SUCCESS;
    const std::vector<uint64_t> ranges = entry_ranges(A, ndev);
    MultiGraphs G;
    GX_TRY(upload_replicas(ctxs, ndev, A, directed, G));
    std::shared_ptr<Clique> clique;
    GX_TRY(get_clique(ctxs, ndev, &clique));
    Clique &C = *clique;
    PerDev<int32_t> par, prev;
    PerDev<int> chg;
    GX_TRY(par.alloc(ctxs, ndev, n));
    GX_TRY(prev.alloc(ctxs, ndev, n));
    GX_TRY(chg.alloc(ctxs, ndev, 1));
    WordExchange X;
    GX_TRY(X.init(ctxs, ndev, n));
    for (int d = 0; d < ndev; d++) {
        GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
        GX_TRY(gx_wcc_part_init(G.g[d], par[d], ctxs[d]->stream));
    }
    // the changed parents always travel as words (applied with MIN): the dense form of the
    // torch driver is an all-reduce MIN, which the words bound from above anyway
    auto no_dense = [&]() -> int { return fail(GX_PANIC, "gx_wcc_multi: dense exchange"); };
    for (uint64_t round = 0;; round++) {
        if (round > n + 1) return fail(GX_DEVICE_ERROR, "gx_wcc_multi: no fixed point");
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_HIP_TRY(hipMemcpyAsync(prev[d], par[d], n * 4, hipMemcpyDeviceToDevice, ctxs[d]->stream));
            GX_HIP_TRY(hipMemsetAsync(chg[d], 0, sizeof(int), ctxs[d]->stream));
            GX_TRY(gx_wcc_part_hook(G.g[d], ranges[d], ranges[d + 1], par[d], chg[d], ctxs[d]->stream));
        }
        uint64_t tot = 0;
        GX_TRY(X.run(C, [&](int d) { return (const void *)par[d]; }, [&](int d) { return (const void *)prev[d]; },
                     [&](int) { return std::make_pair((uint64_t)0, n); }, 4, 1, ~0ull, no_dense,
                     [&](int d) { return (void *)par[d]; }, &tot));
        if (tot == 0) break;   // a round in which no device changed anything: the fixed point
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_TRY(gx_wcc_part_compress(G.g[d], par[d], ctxs[d]->stream));
        }
    }
    X.report("wcc_multi");
    GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
    return download(ctxs[0], comp, par[0], n, Xfer::Widen32);
}

extern "C" int gx_cdlp_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, int iters,
                             uint64_t *labels) {
    GX_TRY(check_multi(ctxs, ndev, A, "gx_cdlp_multi"));
    if (!labels) return fail(GX_NULL_POINTER, "gx_cdlp_multi: null argument");
    if (iters < 0) return fail(GX_INVALID_VALUE, "gx_cdlp_multi: negative iteration count");
    const uint64_t n = A->n;
    if (n == 0) return GX_SUCCESS;
    const std::vector<uint64_t> ranges = entry_ranges(A, ndev);
    uint64_t chunk = 1;
    for (int d = 0; d < ndev; d++) chunk = std::max(chunk, ranges[d + 1] - ranges[d]);
    MultiGraphs G;
    GX_TRY(upload_replicas(ctxs, ndev, A, directed, G));
    std::shared_ptr<Clique> clique;
    GX_TRY(get_clique(ctxs, ndev, &clique));
    Clique &C = *clique;
    PerDev<int32_t> lab, nxt, send, gath;
    PerDev<int> chg;
    GX_TRY(lab.alloc(ctxs, ndev, n));
    GX_TRY(nxt.alloc(ctxs, ndev, n));
    GX_TRY(send.alloc(ctxs, ndev, chunk));
    GX_TRY(gath.alloc(ctxs, ndev, chunk * (uint64_t)ndev));
    GX_TRY(chg.alloc(ctxs, ndev, 1));
    std::vector<gx_cdlp_part *> part(ndev, nullptr);
    struct Parts {
        gx_ctx *const *ctxs;
        std::vector<gx_cdlp_part *> &p;
        ~Parts() {
            for (size_t d = 0; d < p.size(); d++) {
                (void)hipSetDevice(ctxs[d]->device);
                (void)gx_cdlp_part_free(p[d]);
            }
        }
    } parts_cleanup{ctxs, part};
    WordExchange X;
    GX_TRY(X.init(ctxs, ndev, n));
    for (int d = 0; d < ndev; d++) {
        GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
        GX_TRY(gx_cdlp_part_create(G.g[d], ranges[d], ranges[d + 1], &part[d]));
        GX_TRY(gx_cdlp_part_init(part[d], lab[d], ctxs[d]->stream));
    }
    // dense form: the owned slices all-gathered (padded to the largest range) into every labels
    auto dense = [&]() -> int {
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            const uint64_t own = ranges[d + 1] - ranges[d];
            if (own)
                GX_HIP_TRY(hipMemcpyAsync(send[d], nxt[d] + ranges[d], own * 4, hipMemcpyDeviceToDevice,
                                          ctxs[d]->stream));
        }
        GX_TRY(C.all_gather([&](int d) { return (const void *)send[d]; }, [&](int d) { return (void *)gath[d]; },
                            chunk * 4));
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            for (int e = 0; e < ndev; e++) {
                const uint64_t own = ranges[e + 1] - ranges[e];
                if (own)
                    GX_HIP_TRY(hipMemcpyAsync(lab[d] + ranges[e], gath[d] + (uint64_t)e * chunk, own * 4,
                                              hipMemcpyDeviceToDevice, ctxs[d]->stream));
            }
        }
        return GX_SUCCESS;
    };
    for (int it = 0; it < iters; it++) {
        for (int d = 0; d < ndev; d++) {
            GX_HIP_TRY(hipSetDevice(ctxs[d]->device));
            GX_HIP_TRY(hipMemsetAsync(chg[d], 0, sizeof(int), ctxs[d]->stream));
            GX_TRY(gx_cdlp_part_step(part[d], lab[d], nxt[d], chg[d], ctxs[d]->stream));
        }
        uint64_t tot = 0;
        // the owned labels that changed, set into every device's labels; the owned slices
        // all-gathered when that is smaller
        GX_TRY(X.run(C, [&](int d) { return (const void *)nxt[d]; }, [&](int d) { return (const void *)lab[d]; },
                     [&](int d) { return std::make_pair(ranges[d], ranges[d + 1]); }, 4, 0, 4 * n, dense,
                     [&](int d) { return (void *)lab[d]; }, &tot));
        if (tot == 0) break;   // fixed point (LAGraph_cdlp.c:328-332)
    }
    X.report("cdlp_multi");
    GX_HIP_TRY(hipSetDevice(ctxs[0]->device));
    return download(ctxs[0], labels, lab[0], n, Xfer::Widen32);
}

extern "C" int gx_pr_dist_free(gx_pr_dist *h) {
    if (!h) return GX_SUCCESS;
    (void)hipSetDevice(h->d.ctx->device);
    (void)hipDeviceSynchronize();
    delete h;
    return GX_SUCCESS;
}
