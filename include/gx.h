/*
 * gx.h -- C ABI of the MI355X-native GraphBLAS execution layer (libgx.so).
 *
 * Drop-in boundary for the LDBC Graphalytics algorithm hot path of the reference
 * platform driver.  The reference wrapper executables (src/main/c/src/algorithms/<alg>.cpp)
 * load `graph.grb` + `graph.vtb`, call ONE LAGraph function between the
 * "Processing starts/ends at" markers and serialise the result.  libgx replaces that
 * LAGraph/SuiteSparse:GraphBLAS call with hand-written HIP kernels for gfx950; the
 * executables under bin/exe keep the CLI and file contract (execute-job.sh:68-145).
 *
 * Conventions
 *   - Every entry point returns an int status with GrB_Info numbering: 0 = success,
 *     < 0 = error (GX_* below mirror GrB_NULL_POINTER, GrB_INVALID_VALUE, ...).  The
 *     executables keep the reference's OK()-throws convention on top (utils.h:45-55).
 *     gx_last_error() returns a message for the last failure on that thread.
 *   - Host arrays are owned by the caller; libgx copies them to HBM.  Outputs are
 *     caller-allocated host arrays of length n.  Device memory is owned by libgx until
 *     gx_graph_free / gx_free.
 *   - Vertex ids are internal 0-based indices (the .grb row order = .vtb order); the
 *     caller maps them to original ids exactly as the reference serialisers do.
 *   - One gx_ctx per device per process; calls on one ctx come from one host thread.
 *   - There is no CPU fallback: if no gfx950 device is usable gx_init fails.
 */
#ifndef GX_H
#define GX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (GrB_Info numbering) */
#define GX_SUCCESS 0
#define GX_NO_VALUE 1
#define GX_UNINITIALIZED_OBJECT (-1)
#define GX_NULL_POINTER (-2)
#define GX_INVALID_VALUE (-3)
#define GX_INVALID_INDEX (-4)
#define GX_NOT_IMPLEMENTED (-101)
#define GX_OUT_OF_MEMORY (-102)
#define GX_INVALID_OBJECT (-104)
#define GX_PANIC (-103)
#define GX_IO_ERROR (-1001)       /* LAGRAPH_IO_ERROR / binread FREAD CATCH(-1001), graphio.h:43-49 */
#define GX_DEVICE_ERROR (-2000)   /* HIP runtime error */

typedef struct gx_ctx gx_ctx;
typedef struct gx_graph gx_graph;

/* ---------------------------------------------------------------------------------
 * Host CSR exactly as the `.grb` file provides it (graphio.h:88-137, binread).
 * rowptr[n+1], colidx[nnz] are GrB_Index (uint64); vals is NULL for iso/boolean
 * (unweighted) graphs, else nnz fp64 weights.  Row i = out-edges of vertex i.
 * ------------------------------------------------------------------------------- */
typedef struct gx_csr {
    uint64_t n;
    uint64_t nnz;
    uint64_t *rowptr;
    uint64_t *colidx;
    double *vals;
} gx_csr;

/* ---- runtime ---------------------------------------------------------------- */

/* Replaces LAGraph_Init + GxB_Global_Option_set(GxB_GLOBAL_NTHREADS) (bfs.cpp:88-89). */
int gx_init(int device, gx_ctx **ctx);
int gx_free(gx_ctx *ctx);
const char *gx_last_error(void);
int gx_device_count(int *count);
/* Device name / CU count of the context's device (for logs and bench metadata). */
int gx_device_info(gx_ctx *ctx, char *name, size_t name_len, int *num_cus);

/* ---- graph I/O (host, no SuiteSparse) --------------------------------------- */

/* Replaces ReadMatrixMarket -> binread (graphio.cpp:10-15, graphio.h:49-285).
 * Reads every kind binread reads (graphio.h:114-117): sparse, hypersparse, bitmap and
 * full, CSR or CSC, any GrB type; bool/integer values are treated as structure,
 * FP32/FP64 values become fp64 weights (an iso FP64 matrix -- all weights equal -- gives
 * every entry that weight).  Output arrays are allocated by libgx; release with
 * gx_csr_release. */
int gx_read_grb(const char *path, gx_csr *out);
/* Replaces binwrite (graphio.h:310-615): writes a SuiteSparse-compatible sparse CSR
 * `.grb` (BOOL iso when vals == NULL, else FP64). */
int gx_write_grb(const char *path, const gx_csr *csr);
/* Replaces ReadMapping for `.vtb` (graphio.cpp:39-49): raw uint64 original ids. */
int gx_read_vtb(const char *path, uint64_t **ids, uint64_t *count);
int gx_write_vtb(const char *path, const uint64_t *ids, uint64_t count);
/* Replaces LAGraph_MMRead (graphio.cpp:16-24; converter.cpp:38): Matrix Market
 * coordinate file as written by relabel.py:64-79 (integer|real|pattern,
 * general|symmetric; the `%%GraphBLAS <type>` line is honoured).  Symmetric files are
 * expanded to both directions; rows come out sorted; duplicate entries keep the last. */
int gx_read_mtx(const char *path, gx_csr *out);
/* Replaces ReadMapping for `.vtx` (graphio.cpp:50-57): one original id per line. */
int gx_read_vtx(const char *path, uint64_t **ids, uint64_t *count);
void gx_csr_release(gx_csr *csr);
void gx_host_free(void *p);

/* Synthetic inputs (bench / tests): R-MAT edge list with probabilities
 * (a,b,c, d=1-a-b-c), 2^scale vertices, edgefactor*2^scale generated edges, seeded and
 * independent of thread count; self-loops and duplicates removed; vertex ids permuted by
 * a seeded permutation; `undirected` stores both directions.  weighted != 0 attaches
 * U(0,1] fp64 weights (symmetric for undirected graphs).  Result is a sorted CSR. */
int gx_rmat_csr(int scale, int edgefactor, double a, double b, double c, uint64_t seed,
                int undirected, int weighted, gx_csr *out);

/* ---- device graph ------------------------------------------------------------ */

/* Uploads A to HBM (int64 row pointers, int32 column indices when n < 2^31).
 * Replaces LAGraph_New(&G, &A, kind) (bfs.cpp:78).  A row must not hold the same column
 * twice (a GrB_Matrix cannot; gx_read_grb/_mtx and gx_rmat_csr never produce it): CDLP's first
 * iteration on an undirected graph relies on it. */
int gx_graph_create(gx_ctx *ctx, const gx_csr *A, int directed, gx_graph **g);
int gx_graph_free(gx_graph *g);
int gx_graph_info(gx_graph *g, uint64_t *n, uint64_t *nnz, int *directed, int *weighted);

/* ---- algorithm-level entry points (one per reference executable) -------------- */

/* LAGr_BreadthFirstSearch(&level, NULL, G, src) (bfs.cpp:80).  level[v] = hop count
 * over out-edges, INT64_MAX when unreachable (bfs.cpp:53-61). */
int gx_bfs(gx_graph *g, uint64_t src, int64_t *level);

/* LAGr_PageRankGX(&r, &iters, G, damping, itermax) incl. LAGraph_Cached_OutDegree /
 * LAGraph_Cached_AT (pr.cpp:58-61).  Graphalytics PR with dangling redistribution,
 * exactly `iters` iterations, fp64. */
int gx_pagerank(gx_graph *g, double damping, int iters, double *rank);
/* The whole of bin/exe/pr's processing (pr.cpp:77-79: LAGraph_New .. LAGr_PageRankGX between the
 * markers) in one call: upload of the host CSR A, plan, iterations.  For an undirected graph the
 * columns cross the host link chunk by chunk on a host thread while the device builds the plan
 * from the row pointers and takes each chunk as it lands, and the weights (unused by PageRank) are
 * not uploaded.  Same result as gx_graph_create + gx_pagerank + gx_graph_free (which directed
 * graphs and GX_PR_FUSED=0 run); a column >= n fails with GX_INVALID_INDEX.  keep != NULL: the
 * device graph (with its cached plan; its weights are absent) is handed to the caller, who
 * frees it with gx_graph_free (bin/exe/pr does so after its end marker); NULL: freed here. */
int gx_pagerank_csr(gx_ctx *ctx, const gx_csr *A, int directed, double damping, int iters, double *rank,
                    gx_graph **keep);

/* Diagonal fill + LAGraph_Cached_EMin + LAGr_SingleSourceShortestPath(Delta = 2.5)
 * (sssp.cpp:53-81).  dist[v] fp64, +INFINITY when unreachable (printed `infinity`,
 * sssp.cpp:44-46).  Requires a weighted graph. */
int gx_sssp(gx_graph *g, uint64_t src, double *dist);

/* A LOR A' (directed) + LAGr_ConnectedComponents (wcc.cpp:39-66).  comp[v] = the
 * smallest internal vertex index of v's weakly connected component. */
int gx_wcc(gx_graph *g, uint64_t *comp);

/* LAGraph_cdlp / CUDA_CDLP::LAGraph_cdlp_gpu (cdlp.cpp:54-81; cdlp_cuda.cu:118-251).
 * labels[v] = internal index of v's community label after at most `iters` synchronous
 * min-mode iterations (in + out neighbours for directed graphs). */
int gx_cdlp(gx_graph *g, int iters, uint64_t *labels);

/* LAGraph_lcc(&d, A, symmetric = !directed) (lcc.cpp:61-71). */
int gx_lcc(gx_graph *g, double *lcc);

/* ---- op-level GraphBLAS entry points (unit parity) ------------------
 * The operations the reference's LAGraph calls are built from, on the device graph g
 * (A = its adjacency; the matrix value of an entry is its fp64 weight, 1 when unweighted).
 * Vectors are dense host arrays of length n with an optional presence byte per entry
 * (NULL = every entry present); absent entries hold the monoid identity.
 *   semiring              u / w types          reference use
 *   GX_PLUS_SECOND_FP64   double / double      GrB_mxv(t, .., plus_second_fp64, AT, w), pr.cpp:61
 *                                              (LAGr_PageRankGX): mxv with GX_DESC_T0 runs the
 *                                              PageRank kernel itself
 *   GX_MIN_SECOND_UINT64  uint64 / uint64      GrB_mxm(S, .., GrB_MIN_SECOND_SEMIRING_UINT64, ..),
 *                                              LAGraph_cdlp.c:272-281; FastSV (wcc.cpp:61)
 *   GX_ANY_PAIR_BOOL      (presence) / uint8   BFS frontier vxm (bfs.cpp:80)
 *   GX_MIN_PLUS_FP64      double / double      SSSP relaxation vxm (sssp.cpp:78)
 *   GX_PLUS_PAIR_INT64    (presence) / int64   triangle counts (lcc.cpp:68)
 * gx_mxv: t(i) = (+)_j mult(M(i,j), u(j)) over stored M(i,j) and present u(j), M = A (A' with
 *         GX_DESC_T0);  gx_vxm: t(j) = (+)_i mult(u(i), A(i,j)) (A' with GX_DESC_T0);
 *         SECOND(x,y) = y, PLUS(x,y) = x+y, PAIR = 1; t(i) present iff a term exists.  Then
 *         w<mask> = t, or w (+)= t with GX_DESC_ACCUM (old w present per w_present, or all
 *         when it is NULL); mask = n structural bytes or NULL, complemented by
 *         GX_DESC_MASK_COMP; masked-out entries are kept, or cleared by GX_DESC_REPLACE.
 *         w is read (for the kept / accumulated entries) and written; w_present, if given,
 *         likewise.  u may be NULL for the PAIR semirings and vxm's SECOND ones.
 * gx_mxm_masked: C<A> = A (+).(x) A' with GX_PLUS_PAIR_INT64 and desc 0: c[e] for the stored
 *         entry e = (i, j) of A (in A's entry order, nnz values) is |{k : A(i,k), A(j,k)}|,
 *         the dot product of rows i and j (rows must not repeat a column).  Other semirings
 *         and descriptors: GX_NOT_IMPLEMENTED.
 * ------------------------------------------------------------------------------- */
#define GX_PLUS_SECOND_FP64 0
#define GX_MIN_SECOND_UINT64 1
#define GX_ANY_PAIR_BOOL 2
#define GX_MIN_PLUS_FP64 3
#define GX_PLUS_PAIR_INT64 4
#define GX_DESC_T0 1          /* GrB_INP0 = GrB_TRAN */
#define GX_DESC_MASK_COMP 2   /* GrB_MASK = GrB_COMP (structural mask) */
#define GX_DESC_REPLACE 4     /* GrB_OUTP = GrB_REPLACE */
#define GX_DESC_ACCUM 8       /* accum = the semiring's monoid */
int gx_mxv(gx_graph *g, int semiring, int desc, const uint8_t *mask, const void *u, const uint8_t *u_present,
           void *w, uint8_t *w_present);
int gx_vxm(gx_graph *g, int semiring, int desc, const uint8_t *mask, const void *u, const uint8_t *u_present,
           void *w, uint8_t *w_present);
int gx_mxm_masked(gx_graph *g, int semiring, int desc, int64_t *c);

/* ---- timing ---------------------------------------------------------------------
 * Kernel-level timing with hipEvents on the stream the kernels run on.  When enabled,
 * every launch of a named hot kernel is bracketed by events; gx_kernel_stats reports
 * the number of launches and the summed device time since the last reset. */
int gx_set_kernel_timing(gx_ctx *ctx, int enable);
int gx_kernel_stats(gx_ctx *ctx, const char *kernel, uint64_t *launches, double *total_ms);
int gx_reset_kernel_stats(gx_ctx *ctx);
/* Device time (ms) of the last algorithm call, from hipEvents around its device work
 * (excludes the host->device upload of the graph and the device->host result copy). */
int gx_last_device_ms(gx_ctx *ctx, double *ms);

/* ---- PageRank row partition (1-D row blocks, one process per GPU) ----------------
 * The pull matrix (A' for directed graphs, A for undirected) is split into row blocks;
 * each rank owns rows [row_begin, row_end).  Rank vectors are exchanged in a padded
 * layout of `nranks` chunks of `chunk` doubles: rows of rank k occupy
 * [k*chunk, k*chunk + rows_k) and the rank's dangling-score sum sits at
 * k*chunk + chunk - 1.  The caller all-gathers the local chunk each iteration
 * (RCCL over xGMI); libgx only touches device memory on the context's stream.
 *
 *   gx_pr_part_create   : local pull rows (global column ids, sorted), global out-degree
 *                         of every local row, and the row ranges of all ranks.
 *   gx_pr_part_chunk    : doubles per chunk (buffers are nranks*chunk long).
 *   gx_pr_part_init     : writes the iteration-0 local chunk into x_local (device).
 *   gx_pr_part_step     : one iteration: reads the gathered x_full (device), writes the
 *                         next local chunk into x_local (device); if rank_out (device,
 *                         rows_local long) is non-NULL also writes the scores.
 *   stream              : hipStream_t to launch on (NULL = the context's stream).
 * ------------------------------------------------------------------------------- */
typedef struct gx_pr_part gx_pr_part;
int gx_pr_part_create(gx_ctx *ctx, uint64_t n_global, int nranks, int rank,
                      const uint64_t *row_ranges /* nranks+1 */,
                      const uint64_t *rowptr_local /* rows_local+1, starting at 0 */,
                      const uint64_t *colidx_local, const uint64_t *outdeg_local,
                      double damping, gx_pr_part **part);
/* As gx_pr_part_create, with live_rows[k] (nranks entries) = the leading rows of rank k
 * that have out-edges; every later row of rank k has out-degree 0, so no rank ever gathers
 * it.  Only the live prefix of each rank goes in the chunk (chunk = max live + 1, rounded
 * up), which cuts the all-gather by the share of vertices without out-edges (29.5 % of
 * SYN-7_5).  The x values of the other rows stay in the part.  NULL = all rows live. */
int gx_pr_part_create_live(gx_ctx *ctx, uint64_t n_global, int nranks, int rank,
                           const uint64_t *row_ranges /* nranks+1 */, const uint64_t *live_rows /* nranks */,
                           const uint64_t *rowptr_local, const uint64_t *colidx_local,
                           const uint64_t *outdeg_local, double damping, gx_pr_part **part);
int gx_pr_part_chunk(gx_pr_part *part, uint64_t *chunk);
int gx_pr_part_init(gx_pr_part *part, double *x_local, void *stream);
int gx_pr_part_step(gx_pr_part *part, const double *x_full, double *x_local,
                    double *rank_out, void *stream);
int gx_pr_part_free(gx_pr_part *part);

/* ---- device-driven multi-GPU PageRank (RCCL inside libgx) --------------------------
 * The same partition, but the whole run -- init, every iteration's SpMV and every
 * all-gather -- is enqueued by one call (optionally captured once into a hipGraph and
 * replayed), instead of one host round trip per iteration and rank.
 * Replaces the per-iteration GrB_mxv of LAGr_PageRankGX (pr.cpp:61) on N GPUs.
 *
 *   gx_comm_unique_id : rank 0 creates the RCCL id (128 opaque bytes); the caller
 *                       shares it with every rank (e.g. torch.distributed broadcast).
 *   gx_comm_create    : collective over the `nranks` processes (ncclCommInitRank); rank
 *                       numbering must equal the partition's.
 *   gx_pr_dist_create : `npieces` pieces of this rank, piece p = virtual rank
 *                       p*nranks + rank of a gx_pr_part partition into nranks*npieces
 *                       ranges (pr_partition.local_pieces).  comm == NULL means one rank
 *                       (pieces exchanged by device copies).  Borrows the pieces.
 *   gx_pr_dist_run    : `iters` iterations; use_graph != 0 captures the run into a
 *                       hipGraph on first use (re-captured when iters/stream change) and
 *                       replays it.  Asynchronous on `stream` (NULL = context stream).
 *                       With kernel timing on (gx_set_kernel_timing) launches are direct.
 *   gx_pr_dist_scores : waits for the last run, copies piece `piece`'s scores (its rows,
 *                       in the partition's row order) to host memory.
 * ------------------------------------------------------------------------------- */
typedef struct gx_comm gx_comm;
typedef struct gx_pr_dist gx_pr_dist;
int gx_comm_unique_id(uint8_t *id /* 128 bytes */);
int gx_comm_create(gx_ctx *ctx, int nranks, int rank, const uint8_t *id, gx_comm **comm);
int gx_comm_free(gx_comm *comm);
int gx_pr_dist_create(gx_comm *comm, gx_pr_part *const *pieces, int npieces, gx_pr_dist **dist);
int gx_pr_dist_run(gx_pr_dist *dist, int iters, int use_graph, void *stream);
int gx_pr_dist_scores(gx_pr_dist *dist, int piece, double *scores);
int gx_pr_dist_free(gx_pr_dist *dist);

/* ---- one-shot peer-to-peer exchange (no RCCL) -----
 * EXPERIMENTAL: tested only with two processes sharing one GPU (IPC mappings on one device);
 * the cross-device case (puts over xGMI into another GPU's coarse-grained memory, polled by the
 * owner) has not run on a multi-GPU node yet -- tests/test_distributed.py::
 * test_gpu_p2p_exchange_world2_two_devices is that check, skipped on a one-GPU box.  RCCL
 * (gx_pr_dist_create) is the supported exchange.
 * The same runner, but each exchange is direct: every rank writes its chunk into every
 * peer's exchanged vector (IPC-mapped over xGMI, one write per peer and piece, all links at
 * once) and raises an arrival flag there; the next SpMV waits for every rank's flag.
 *   gx_pr_dist_create_p2p : rank `rank` of `nranks` processes (<= 64), pieces as for
 *                           gx_pr_dist_create; writes GX_P2P_HANDLE_BYTES of IPC handles
 *                           of this rank's buffers to `handle`.
 *   gx_pr_dist_p2p_attach : `handles` = every rank's handle in rank order (an all-gather
 *                           of `handle`; NULL allowed for one rank); collective in effect,
 *                           required before gx_pr_dist_run.
 * A wait that never sees a peer's flag gives up after GX_P2P_POLLS polls (default 2^22,
 * seconds) and gx_pr_dist_scores then fails with GX_DEVICE_ERROR.  At most 2^24 - 2 iterations
 * per run (tokens are run * 2^24 + step).  Before any rank calls gx_pr_dist_free, every rank must
 * have stopped issuing runs and passed a barrier (e.g. MPI_Barrier after its last
 * gx_pr_dist_scores): free unmaps this rank's vectors, which a peer's next run would write.
 * ------------------------------------------------------------------------------- */
#define GX_P2P_HANDLE_BYTES 192
int gx_pr_dist_create_p2p(int nranks, int rank, gx_pr_part *const *pieces, int npieces, uint8_t *handle,
                          gx_pr_dist **dist);
int gx_pr_dist_p2p_attach(gx_pr_dist *dist, const uint8_t *handles);

/* ---- one process, N GPUs (the executables' GX_NGPUS switch) ------------------------
 * gx_pagerank_multi: Graphalytics PageRank of the host CSR A on the ndev devices of `ctxs`
 * (one gx_ctx per distinct device, or virtual devices: see gx_lcc_multi).  The pull matrix
 * (A' built on each device for a directed graph) is 1-D row partitioned: the hub-first order is
 * dealt round-robin over the devices (gx_pr_partition; each device derives it by the same
 * device sort), each device gets its rows with columns already in the exchange layout,
 * and every iteration is one SpMV per device (k_pr_pull_units) plus one grouped in-process
 * RCCL all-gather (ncclCommInitAll over the devices, xGMI) of the live rows and dangling
 * slots.  rank[v] in A's vertex order.  Replaces LA_PR (pr.cpp:47-66) when bin/exe/pr runs with
 * GX_NGPUS=N: execute-job.sh cannot pass new flags (execute-job.sh:68-151), and the CLI stays
 * one process.
 * gx_pr_partition (host only, no GPU): order[i] = the vertex at hub-first position i
 * (out-degree descending, ties by id); part k owns positions k, k + nparts, ... as its local
 * rows 0, 1, ...: rows[k] of them, the first live[k] with out-edges (nparts entries each).
 * ------------------------------------------------------------------------------- */
int gx_pagerank_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, double damping, int iters,
                      double *rank);
int gx_pr_partition(uint64_t n, const uint64_t *rowptr, int nparts, uint32_t *order, uint64_t *rows, uint64_t *live);
/* gx_sssp_multi: single-source shortest paths of the weighted host CSR A (vals = fp64) from
 * src on the ndev devices of `ctxs`, in one process (bin/exe/sssp with GX_NGPUS=N; config 4 is
 * "PageRank + SSSP on datagen-8_5-fb, 8 GPUs, 1-D row partition + RCCL allgather").  Every
 * device holds A and owns a contiguous target range of ~nnz / ndev entries (gx_sssp_split);
 * per round the 2-word counts and then the improved (vertex, distance) pairs are all-gathered
 * by an in-process RCCL clique.  dist[v] in A's vertex order, +inf = unreached, bit-identical
 * to gx_sssp.  Replaces LA_SSSP (sssp.cpp:53-81) when it runs on several GPUs. */
int gx_sssp_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, uint64_t src, double *dist);
/* gx_lcc_multi: LAGraph_lcc of the host CSR A on the ndev devices of `ctxs`, in one process
 * (bin/exe/lcc with GX_NGPUS=N; BASELINE config 5, "LCC on cit-Patents, 1 -> 8 GPUs").  Every
 * device holds A and its degree orientation and counts the triangles of a range of middle
 * vertices balanced by probe work (gx_lcc_part_ranges); the n integer counters are summed onto
 * the first device by one reduction (in-process RCCL ncclReduce).  lcc[v] in A's vertex order,
 * bit-identical to gx_lcc.  Replaces LA_LCC (lcc.cpp:61-71) when it runs on several GPUs.
 *
 * Virtual devices: the three gx_*_multi calls also accept ndev >= 2 contexts that are ALL on
 * one device (gx_init(d) called ndev times).  Each is then planned and run exactly as a
 * separate GPU would be, and every collective becomes device-to-device copies (reduce: device
 * adds) with the collective's ordering, so the N > 1 path runs, and is tested, on one GPU.
 * Mixed layouts (some contexts sharing a device, some not) are GX_INVALID_VALUE. */
int gx_lcc_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, double *lcc);
/* gx_multi_prepare: creates the collective clique of the ndev contexts (ncclCommInitAll, or the
 * copy events of virtual devices) that the gx_*_multi calls on the same context list reuse, so
 * a caller pays it ahead of its timed region, as it pays gx_init.  Optional: the first
 * gx_*_multi call on a list creates it otherwise.  The clique lives until gx_free of any of
 * its contexts.  Same argument rules as gx_lcc_multi. */
int gx_multi_prepare(gx_ctx *const *ctxs, int ndev);
/* gx_bfs_multi / gx_wcc_multi / gx_cdlp_multi: BFS levels (int64, INT64_MAX = unreached), WCC
 * labels (the smallest vertex id of each component) and CDLP labels (vertex ids) of the host
 * CSR A on the ndev devices of `ctxs`, in one process (bin/exe/{bfs,wcc,cdlp} with GX_NGPUS=N).
 * The graph is replicated (gx_graph_create on every device); device d owns a contiguous vertex
 * range of ~nnz / ndev entries and runs the gx_*_part_* steps below on it; per round only what
 * the step changed crosses the clique (gx_part_changes words, counts read by the host), or the
 * dense form when smaller (BFS: bitmaps OR-ed; CDLP: the owned label slices).  Results equal
 * gx_bfs / gx_wcc / gx_cdlp bit for bit.  Replace LA_BFS (bfs.cpp:70-83), WeaklyConnectedComponents
 * (wcc.cpp:39-66) and LA_CDLP (cdlp.cpp:54-81) when they run on several GPUs.  Same context
 * rules (distinct devices or virtual devices) as gx_lcc_multi. */
int gx_bfs_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, uint64_t src, int64_t *level);
int gx_wcc_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, uint64_t *comp);
int gx_cdlp_multi(gx_ctx *const *ctxs, int ndev, const gx_csr *A, int directed, int iters, uint64_t *labels);

/* ---------------------------------------------------------------------------------
 * Multi-GPU steps for the other algorithms.  The graph is replicated on
 * every rank (gx_graph_create on each device); rank k owns the vertex range
 * [v0, v1) = [ranges[k], ranges[k+1]).  All array arguments are DEVICE pointers of full
 * length n (caller-allocated, e.g. torch tensors); the caller runs the collective named
 * below between steps (torch.distributed / RCCL).  `stream` is the hipStream_t to launch
 * on; unlike gx_pr_part_*, NULL here means the null (default) stream -- torch's default
 * stream -- so the steps order with tensors and collectives issued there.
 * The reference has no distributed path; these replace LA_BFS / LA_CDLP_CPU / LA_LCC /
 * LA_SSSP / WeaklyConnectedComponents (bfs.cpp:70-83, cdlp.cpp:54-67, lcc.cpp:61-71,
 * sssp.cpp:53-81, wcc.cpp:39-66) when they run on several GPUs.
 *
 * BFS  : init(level); per level cur = 0, 1, ...: zero next (n bytes); expand(owned rows);
 *        all-reduce MAX(next); zero count; commit -> count = vertices at level cur+1;
 *        stop when count == 0.  level: INT64_MAX = unreached.
 * WCC  : init(parent); per round: zero changed; hook(owned rows' edges, then compress);
 *        all-reduce MIN(parent); compress; all-reduce MAX(changed); stop when 0.
 *        parent[v] is then the smallest vertex id of v's component.
 * SSSP : split_create(owned targets [v0, v1)) once -- the edges into owned vertices, by
 *        source, light first; split_start(src); per round: split_relax(-> this rank's
 *        improved owned vertices as (vertex, fp64 bits) pairs + count[2] = {pairs, done});
 *        all-gather the count words; stop when done; all-gather the first 2 max-count words
 *        of every rank's pairs; split_apply(all ranks' pairs, the gathered counts, nranks,
 *        stride = max count).  The distance vector is replicated: every rank applies every
 *        improvement and takes the same delta-stepping decisions.  split_distances copies it
 *        out (fp64, +inf = unreached).  split_run: one rank owning every vertex, rounds on the
 *        device with no exchange.
 * CDLP : part_create(range) once; part_init(labels); per iteration: zero changed;
 *        part_step(labels -> next, owned range written); exchange the owned slices of next
 *        into every rank's labels (all-gather); all-reduce MAX(changed); stop when 0 or
 *        after `iters`.  labels are int32 vertex ids.
 * LCC  : part_create once (orientation); part_ranges -> balanced ranges (same on every
 *        rank); zero tc (n uint64); part_counts(owned range); all-reduce SUM(tc);
 *        part_finish(tc -> lcc).
 * ------------------------------------------------------------------------------- */
int gx_bfs_part_init(gx_graph *g, uint64_t src, int64_t *level, void *stream);
int gx_bfs_part_expand(gx_graph *g, uint64_t v0, uint64_t v1, const int64_t *level, int64_t cur,
                       uint8_t *next, void *stream);
int gx_bfs_part_commit(gx_graph *g, const uint8_t *next, int64_t *level, int64_t cur, uint64_t *count,
                       void *stream);

/* Sparse exchange of a step's updates (BFS / WCC / CDLP at N > 1, distributed.py): the
 * entries v in [v0, v1) of a whose value differs from b[v] (b null: from 0) are appended to
 * words as (v << 32 | value) -- one 64-bit word each, *count (device int64, zeroed here) of
 * them, in no particular order; elem_bytes 1 (uint8) or 4 (int32).  After an all-gather of
 * the counts and of the first max-count words of every rank, gx_part_apply writes every
 * rank's words (rank k's counts[k] words at words + k stride) into arr: op 0 set, 1 min, 2 max
 * (min / max for 4-byte elements).  No gx_graph: runs on the current device, on `stream`. */
int gx_part_changes(const void *a, const void *b, uint64_t v0, uint64_t v1, int elem_bytes, uint64_t *words,
                    int64_t *count, void *stream);
int gx_part_apply(const uint64_t *words, const int64_t *counts, int nranks, uint64_t stride, void *arr,
                  int elem_bytes, int op, void *stream);
/* BFS's dense exchange as bits: next (n bytes, 16-B aligned) -> bits (ceil(n / 32) words); after
 * an all-gather of every rank's words (rank r at gathered + r ceil(n / 32)), next[v] = 1 where
 * any rank's bit v is set (1 / N the bytes of an all-reduce MAX of next at N ranks over 8). */
int gx_part_pack_bits(const uint8_t *next, uint64_t n, uint32_t *bits, void *stream);
int gx_part_or_bits(const uint32_t *gathered, int nranks, uint64_t n, uint8_t *next, void *stream);

int gx_wcc_part_init(gx_graph *g, int32_t *parent, void *stream);
int gx_wcc_part_hook(gx_graph *g, uint64_t v0, uint64_t v1, int32_t *parent, int *changed, void *stream);
int gx_wcc_part_compress(gx_graph *g, int32_t *parent, void *stream);

typedef struct gx_sssp_split gx_sssp_split;
int gx_sssp_split_create(gx_graph *g, uint64_t v0, uint64_t v1, gx_sssp_split **part);
int gx_sssp_split_delta(gx_sssp_split *part, double *delta);
int gx_sssp_split_start(gx_sssp_split *part, uint64_t src, void *stream);
/* pairs: device buffer of 2 (v1 - v0) uint64; count: device uint64[2] */
int gx_sssp_split_relax(gx_sssp_split *part, uint64_t *pairs, uint64_t *count, void *stream);
/* rank r's pairs at pairs + 2 r stride, its count words at counts + 2 r */
int gx_sssp_split_apply(gx_sssp_split *part, const uint64_t *pairs, const uint64_t *counts, int nranks,
                        uint64_t stride, void *stream);
int gx_sssp_split_distances(gx_sssp_split *part, double *dist, void *stream);
int gx_sssp_split_run(gx_sssp_split *part, uint64_t src, double *dist);
int gx_sssp_split_free(gx_sssp_split *part);

typedef struct gx_cdlp_part gx_cdlp_part;
int gx_cdlp_part_create(gx_graph *g, uint64_t v0, uint64_t v1, gx_cdlp_part **part);
int gx_cdlp_part_init(gx_cdlp_part *part, int32_t *labels, void *stream);
int gx_cdlp_part_step(gx_cdlp_part *part, const int32_t *labels, int32_t *next, int *changed, void *stream);
int gx_cdlp_part_free(gx_cdlp_part *part);

typedef struct gx_lcc_part gx_lcc_part;
int gx_lcc_part_create(gx_graph *g, gx_lcc_part **part);
int gx_lcc_part_ranges(gx_lcc_part *part, int nranks, uint64_t *ranges /* nranks+1, host */);
int gx_lcc_part_counts(gx_lcc_part *part, uint64_t v0, uint64_t v1, uint64_t *tc, void *stream);
int gx_lcc_part_finish(gx_lcc_part *part, const uint64_t *tc, double *lcc, void *stream);
int gx_lcc_part_free(gx_lcc_part *part);

#ifdef __cplusplus
}
#endif

#endif /* GX_H */
