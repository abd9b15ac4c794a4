/*
 * gx_oracle.c -- CPU restatement of the six LDBC Graphalytics algorithm kernels.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle for the HIP hot path in
 * ldbc_graphalytics_platforms_graphblas_amd/csrc.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / the CPU
 * baseline -- never as the thing measured or shipped.
 *
 * What it restates (the reference calls these through LAGraph / SuiteSparse:GraphBLAS,
 * which are third-party and not vendored in the reference):
 *   - SuiteSparse:GraphBLAS v7.4.4 (pinned tag, bin/sh/install-graphblas.sh:8)
 *   - LAGraph `dev` branch (unpinned, bin/sh/install-lagraph.sh:8)
 * Call sites in the reference wrapper executables:
 *   BFS  LAGr_BreadthFirstSearch        src/main/c/src/algorithms/bfs.cpp:80
 *   PR   LAGr_PageRankGX                src/main/c/src/algorithms/pr.cpp:61
 *   SSSP LAGr_SingleSourceShortestPath  src/main/c/src/algorithms/sssp.cpp:78
 *   WCC  LAGr_ConnectedComponents       src/main/c/src/algorithms/wcc.cpp:61
 *   LCC  LAGraph_lcc                    src/main/c/src/algorithms/lcc.cpp:68
 *   CDLP LAGraph_cdlp                   src/main/c/src/algorithms/cdlp.cpp:63
 *                                       (vendored text: LAGraph_cdlp.c:37-121, 264-333)
 * The restatement follows the published Graphalytics definitions those calls implement.
 * Pinning: tests/test_oracle_fixtures.py checks every function below against the 24
 * Graphalytics validation outputs shipped in the reference (example-data-sets/graphs/,
 * copied to tests/golden/graphalytics/) and against scipy/networkx on synthetic graphs.
 *
 * Graph representation: the `.grb` CSR exactly as the reference reads it
 * (graphio.h:88-137): rowptr[n+1] and colidx[nnz] as 64-bit GrB_Index, row i = out-edges
 * of internal vertex i, optional fp64 weights.  Undirected graphs are stored with both
 * directions (symmetric .mtx expanded by LAGraph_MMRead, relabel.py:47-50).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_OK 0
#define ORC_OOM (-102)        /* GrB_OUT_OF_MEMORY */
#define ORC_INVALID (-3)      /* GrB_INVALID_VALUE */

static void orc_set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------------------------
 * Transpose by counting sort.  Stable, so every row of the result is sorted by column
 * when the input rows are (LAGraph_Cached_AT, pr.cpp:60; GrB_transpose, LAGraph_cdlp.c:258).
 * Caller frees *rpT, *ciT, *wT with orc_free.
 * ---------------------------------------------------------------------------------- */
int orc_transpose(int64_t n, const int64_t *rp, const int64_t *ci, const double *w,
                  int64_t **rpT, int64_t **ciT, double **wT) {
    int64_t nnz = rp[n];
    int64_t *tp = (int64_t *)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t *tc = (int64_t *)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int64_t));
    double *tw = w ? (double *)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(double)) : NULL;
    int64_t *cur = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
    if (!tp || !tc || !cur || (w && !tw)) {
        free(tp); free(tc); free(tw); free(cur);
        return ORC_OOM;
    }
    for (int64_t k = 0; k < nnz; k++) tp[ci[k] + 1]++;
    for (int64_t i = 0; i < n; i++) tp[i + 1] += tp[i];
    memcpy(cur, tp, (size_t)(n + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) {
        for (int64_t k = rp[i]; k < rp[i + 1]; k++) {
            int64_t dst = cur[ci[k]]++;
            tc[dst] = i;
            if (w) tw[dst] = w[k];
        }
    }
    free(cur);
    *rpT = tp;
    *ciT = tc;
    if (wT) *wT = tw; else free(tw);
    return ORC_OK;
}

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------------------------
 * BFS: level-synchronous traversal over out-edges from internal vertex `src`
 * (LAGr_BreadthFirstSearch(&level, NULL, G, src), bfs.cpp:70-83).  level[src] = 0;
 * unreachable vertices get INT64_MAX, the value SerializeBFSResult prints for vertices
 * absent from LAGraph's sparse result (bfs.cpp:53-61).
 * ---------------------------------------------------------------------------------- */
int orc_bfs(int64_t n, const int64_t *rp, const int64_t *ci, int64_t src, int64_t *level) {
    if (src < 0 || src >= n) return ORC_INVALID;
    int64_t *queue = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    if (!queue) return ORC_OOM;
    for (int64_t i = 0; i < n; i++) level[i] = INT64_MAX;
    int64_t head = 0, tail = 0;
    level[src] = 0;
    queue[tail++] = src;
    while (head < tail) {
        int64_t u = queue[head++];
        for (int64_t k = rp[u]; k < rp[u + 1]; k++) {
            int64_t v = ci[k];
            if (level[v] == INT64_MAX) {
                level[v] = level[u] + 1;
                queue[tail++] = v;
            }
        }
    }
    free(queue);
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------
 * PageRank, Graphalytics definition with dangling redistribution, fixed `iters`
 * iterations (LA_PR -> LAGr_PageRankGX(&r, &iters, G, damping, itermax), pr.cpp:47-66):
 *   PR_0(v)   = 1/n
 *   PR_i(v)   = (1-d)/n + (d/n) * sum_{w: outdeg(w)=0} PR_{i-1}(w)
 *               + sum_{u in in(v)} PR_{i-1}(u) / (outdeg(u)/d)
 * Arithmetic order follows LAGraph's GX variant: the damping is folded into the
 * out-degree divisor, teleport = (1-d)/n + d/n * dangling, r = teleport + A'*w.
 * Pull over in-edges: for an undirected graph in(v) = out(v) and the CSR is used as is;
 * for a directed graph the transpose is built first (LAGraph_Cached_AT, pr.cpp:60).
 * OpenMP over rows; the per-row sum order (ascending column) does not depend on the
 * thread count, so the result is bitwise independent of nthreads.
 * ---------------------------------------------------------------------------------- */
static double dangling_sum(const int64_t *rp, const double *x, int64_t lo, int64_t hi) {
    if (hi - lo <= 1024) {
        double s = 0.0;
        for (int64_t i = lo; i < hi; i++)
            if (rp[i + 1] == rp[i]) s += x[i];
        return s;
    }
    const int64_t mid = lo + (hi - lo) / 2;
    return dangling_sum(rp, x, lo, mid) + dangling_sum(rp, x, mid, hi);
}

int orc_pagerank(int64_t n, const int64_t *rp, const int64_t *ci, int directed,
                 double damping, int iters, double *rank, int nthreads) {
    if (n <= 0) return ORC_OK;
    orc_set_threads(nthreads);
    const int64_t *prp = rp, *pci = ci;
    int64_t *trp = NULL, *tci = NULL;
    if (directed) {
        int rc = orc_transpose(n, rp, ci, NULL, &trp, &tci, NULL);
        if (rc) return rc;
        prp = trp;
        pci = tci;
    }
    double *bufA = (double *)malloc((size_t)n * sizeof(double));
    double *w = (double *)malloc((size_t)n * sizeof(double));
    double *dsc = (double *)malloc((size_t)n * sizeof(double));
    if (!bufA || !w || !dsc) {
        free(bufA); free(w); free(dsc); free(trp); free(tci);
        return ORC_OOM;
    }
    const double dn = (double)n;
    double *cur = rank, *prev = bufA;
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        cur[i] = 1.0 / dn;
        dsc[i] = (double)(rp[i + 1] - rp[i]) / damping;   /* d_out / damping */
    }
    const double teleport0 = (1.0 - damping) / dn;
    const double damping_over_n = damping / dn;
    for (int it = 0; it < iters; it++) {
        double *tmp = prev; prev = cur; cur = tmp;   /* prev = previous scores */
        /* sum of sink scores: blocked pairwise reduction (GrB_reduce of SuiteSparse is a
         * blocked parallel reduction, not a left-to-right sum); deterministic */
        const double dangling = dangling_sum(rp, prev, 0, n);
        const double teleport = teleport0 + damping_over_n * dangling;
        #pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; i++) w[i] = (rp[i + 1] > rp[i]) ? prev[i] / dsc[i] : 0.0;
        #pragma omp parallel for schedule(dynamic, 1024)
        for (int64_t v = 0; v < n; v++) {
            double s = 0.0;
            for (int64_t k = prp[v]; k < prp[v + 1]; k++) s += w[pci[k]];
            cur[v] = teleport + s;
        }
    }
    if (cur != rank) memcpy(rank, cur, (size_t)n * sizeof(double));
    free(bufA); free(w); free(dsc); free(trp); free(tci);
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------
 * SSSP: Dijkstra over out-edges with non-negative fp64 weights (LA_SSSP ->
 * LAGr_SingleSourceShortestPath(&d, G, src, Delta=2.5), sssp.cpp:53-81).  The reference
 * first stores an explicit 0.0 diagonal (sssp.cpp:60-62); a zero self-loop never shortens
 * a path, so it is not materialised here.  Unreachable vertices get +infinity, which
 * SerializeSSSPResult prints as the literal `infinity` (sssp.cpp:44-46).
 * dist[v] = min over paths of the left-to-right fp64 sum of the path's weights; the
 * relaxation d[v] = min(d[v], d[u] + w) reaches that same fixed point in any order
 * because fp64 addition is monotone, so any correct label-correcting algorithm
 * (delta-stepping, Bellman-Ford) produces bitwise the same distances.
 * Binary heap with lazy deletion.
 * ---------------------------------------------------------------------------------- */
typedef struct { double d; int64_t v; } orc_heap_item;

static void heap_push(orc_heap_item *h, int64_t *sz, double d, int64_t v) {
    int64_t i = (*sz)++;
    h[i].d = d; h[i].v = v;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (h[p].d <= h[i].d) break;
        orc_heap_item t = h[p]; h[p] = h[i]; h[i] = t;
        i = p;
    }
}

static orc_heap_item heap_pop(orc_heap_item *h, int64_t *sz) {
    orc_heap_item top = h[0];
    h[0] = h[--(*sz)];
    int64_t i = 0;
    for (;;) {
        int64_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < *sz && h[l].d < h[m].d) m = l;
        if (r < *sz && h[r].d < h[m].d) m = r;
        if (m == i) break;
        orc_heap_item t = h[m]; h[m] = h[i]; h[i] = t;
        i = m;
    }
    return top;
}

int orc_sssp(int64_t n, const int64_t *rp, const int64_t *ci, const double *w,
             int64_t src, double *dist) {
    if (src < 0 || src >= n) return ORC_INVALID;
    int64_t nnz = rp[n];
    orc_heap_item *h = (orc_heap_item *)malloc((size_t)(nnz + 2) * sizeof(orc_heap_item));
    if (!h) return ORC_OOM;
    for (int64_t i = 0; i < n; i++) dist[i] = INFINITY;
    int64_t sz = 0;
    dist[src] = 0.0;
    heap_push(h, &sz, 0.0, src);
    while (sz > 0) {
        orc_heap_item it = heap_pop(h, &sz);
        if (it.d > dist[it.v]) continue;
        for (int64_t k = rp[it.v]; k < rp[it.v + 1]; k++) {
            double nd = it.d + w[k];
            if (nd < dist[ci[k]]) {
                dist[ci[k]] = nd;
                heap_push(h, &sz, nd, ci[k]);
            }
        }
    }
    free(h);
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------
 * WCC: weakly connected components (WeaklyConnectedComponents -> symmetrize with
 * A LOR A' for directed graphs, then LAGr_ConnectedComponents, wcc.cpp:39-66).
 * Union-find over every stored edge (either direction joins), so no explicit
 * symmetrisation is needed.  Label = minimum internal vertex index of the component:
 * a canonical labelling (Graphalytics validates WCC by equivalence); the
 * wrapper prints mapping[label], which equals the fixtures' min-original-id labels
 * when the .v file is sorted (all shipped fixtures are).
 * ---------------------------------------------------------------------------------- */
static int64_t uf_find(int64_t *p, int64_t x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

int orc_wcc(int64_t n, const int64_t *rp, const int64_t *ci, uint64_t *comp) {
    int64_t *p = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    if (!p) return ORC_OOM;
    for (int64_t i = 0; i < n; i++) p[i] = i;
    for (int64_t u = 0; u < n; u++) {
        for (int64_t k = rp[u]; k < rp[u + 1]; k++) {
            int64_t a = uf_find(p, u), b = uf_find(p, ci[k]);
            if (a == b) continue;
            if (a < b) p[b] = a; else p[a] = b;   /* smaller index stays the root */
        }
    }
    for (int64_t i = 0; i < n; i++) comp[i] = (uint64_t)uf_find(p, i);
    free(p);
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------
 * CDLP: synchronous label propagation (LAGraph_cdlp, LAGraph_cdlp.c:37-121 semantics,
 * 264-333 loop; called from cdlp.cpp:63).  Initial label = internal vertex index
 * (LAGraph_cdlp.c:242-252).  Each iteration every vertex takes the minimum of the most
 * frequent labels among its neighbours: for directed graphs the multiset is the labels
 * of out-neighbours PLUS the labels of in-neighbours, so a reciprocal edge counts twice
 * (LAGraph_cdlp.c:47-50, 113-121).  A vertex without neighbours keeps its label
 * (Graphalytics definition).  The loop stops early at a fixed point
 * (LAGraph_cdlp.c:328-332), which does not change the result.
 * The wrapper prints mapping[label] (cdlp.cpp:48).
 * ---------------------------------------------------------------------------------- */
static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return (x > y) - (x < y);
}

int orc_cdlp(int64_t n, const int64_t *rp, const int64_t *ci, int directed, int iters,
             uint64_t *labels, int nthreads) {
    orc_set_threads(nthreads);
    int64_t *trp = NULL, *tci = NULL;
    if (directed) {
        int rc = orc_transpose(n, rp, ci, NULL, &trp, &tci, NULL);
        if (rc) return rc;
    }
    uint64_t *prev = (uint64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(uint64_t));
    if (!prev) { free(trp); free(tci); return ORC_OOM; }
    int64_t maxdeg = 0;
    for (int64_t v = 0; v < n; v++) {
        int64_t d = rp[v + 1] - rp[v] + (directed ? trp[v + 1] - trp[v] : 0);
        if (d > maxdeg) maxdeg = d;
    }
    for (int64_t v = 0; v < n; v++) labels[v] = (uint64_t)v;
    int oom = 0;
    for (int it = 0; it < iters; it++) {
        memcpy(prev, labels, (size_t)n * sizeof(uint64_t));
        int changed = 0;
        #pragma omp parallel reduction(|:changed) reduction(|:oom)
        {
            uint64_t *buf = (uint64_t *)malloc((size_t)(maxdeg > 0 ? maxdeg : 1) * sizeof(uint64_t));
            if (!buf) oom = 1;
            #pragma omp for schedule(dynamic, 256)
            for (int64_t v = 0; v < n; v++) {
                if (!buf) continue;
                int64_t m = 0;
                for (int64_t k = rp[v]; k < rp[v + 1]; k++) buf[m++] = prev[ci[k]];
                if (directed)
                    for (int64_t k = trp[v]; k < trp[v + 1]; k++) buf[m++] = prev[tci[k]];
                if (m == 0) { labels[v] = prev[v]; continue; }
                qsort(buf, (size_t)m, sizeof(uint64_t), cmp_u64);
                uint64_t best = buf[0];
                int64_t bestc = 0, run = 0;
                for (int64_t k = 0; k < m; k++) {
                    run = (k > 0 && buf[k] == buf[k - 1]) ? run + 1 : 1;
                    if (run > bestc) { bestc = run; best = buf[k]; }  /* strict: min label wins ties */
                }
                labels[v] = best;
                if (best != prev[v]) changed = 1;
            }
            free(buf);
        }
        if (oom) break;
        if (!changed) break;
    }
    free(prev); free(trp); free(tci);
    return oom ? ORC_OOM : ORC_OK;
}

/* ------------------------------------------------------------------------------------
 * LCC: local clustering coefficient (LA_LCC -> LAGraph_lcc(&d, A, symmetric=!directed),
 * lcc.cpp:61-71).  N(v) = in(v) U out(v) as a set, without v; k = |N(v)|;
 *   LCC(v) = #{(u,w) in E : u, w in N(v)} / (k (k-1)),   0 when k < 2.
 * For undirected graphs E holds both directions, which gives 2 t(v) / (k (k-1)).
 * The numerator is an exact integer; the division is one fp64 operation.
 * ---------------------------------------------------------------------------------- */
int orc_lcc(int64_t n, const int64_t *rp, const int64_t *ci, int directed, double *lcc,
            int nthreads) {
    orc_set_threads(nthreads);
    /* S = sorted, deduplicated undirected closure without self-loops */
    int64_t *trp = NULL, *tci = NULL;
    const int64_t *irp = rp, *ici = ci;
    if (directed) {
        int rc = orc_transpose(n, rp, ci, NULL, &trp, &tci, NULL);
        if (rc) return rc;
        irp = trp; ici = tci;
    }
    int64_t *srp = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
    int64_t cap = rp[n] + irp[n];
    int64_t *sci = (int64_t *)malloc((size_t)(cap > 0 ? cap : 1) * sizeof(int64_t));
    /* sorted copy of out-rows for membership tests (input rows may be unsorted) */
    int64_t *oci = (int64_t *)malloc((size_t)(rp[n] > 0 ? rp[n] : 1) * sizeof(int64_t));
    if (!srp || !sci || !oci) {
        free(srp); free(sci); free(oci); free(trp); free(tci);
        return ORC_OOM;
    }
    memcpy(oci, ci, (size_t)rp[n] * sizeof(int64_t));
    srp[0] = 0;
    for (int64_t v = 0; v < n; v++) {
        int64_t m = srp[v];
        for (int64_t k = rp[v]; k < rp[v + 1]; k++) if (ci[k] != v) sci[m++] = ci[k];
        if (directed)
            for (int64_t k = irp[v]; k < irp[v + 1]; k++) if (ici[k] != v) sci[m++] = ici[k];
        qsort(sci + srp[v], (size_t)(m - srp[v]), sizeof(int64_t), cmp_u64);
        int64_t u = srp[v];
        for (int64_t k = srp[v]; k < m; k++)
            if (k == srp[v] || sci[k] != sci[k - 1]) sci[u++] = sci[k];
        srp[v + 1] = u;
        qsort(oci + rp[v], (size_t)(rp[v + 1] - rp[v]), sizeof(int64_t), cmp_u64);
    }
    #pragma omp parallel for schedule(dynamic, 64)
    for (int64_t v = 0; v < n; v++) {
        int64_t k = srp[v + 1] - srp[v];
        if (k < 2) { lcc[v] = 0.0; continue; }
        int64_t num = 0;
        for (int64_t a = srp[v]; a < srp[v + 1]; a++) {
            int64_t u = sci[a];
            /* |out(u) \ {u} intersect N(v)|, both sorted: merge */
            int64_t i = rp[u], j = srp[v];
            while (i < rp[u + 1] && j < srp[v + 1]) {
                int64_t x = oci[i], y = sci[j];
                if (x < y) i++;
                else if (x > y) j++;
                else { if (x != u) num++; i++; j++; }
            }
        }
        lcc[v] = (double)num / ((double)k * (double)(k - 1));
    }
    free(srp); free(sci); free(oci); free(trp); free(tci);
    return ORC_OK;
}

/* ====================================================================================
 * Parallel CPU baselines (bench.py's cpu_baseline leg).  The functions above are the
 * checkers; these compute the same results with every host core, so that the GPU/CPU ratio
 * is against a multithreaded CPU implementation like SuiteSparse's (GxB_GLOBAL_NTHREADS =
 * --threadnum, bfs.cpp:88-89).  Each returns bitwise the result of its serial counterpart
 * (tests/test_oracle_parallel.py): BFS levels and min-id WCC labels are unique, and SSSP's
 * relaxation fixed point does not depend on the order (see orc_sssp).
 * ==================================================================================== */

/* BFS, direction-optimising (Beamer et al.; LAGr_BreadthFirstSearch is push/pull too):
 * top-down levels claim vertices with a CAS on level[]; when the frontier's out-edges pass
 * 1/14 of the unexplored edges a level is run bottom-up (only for symmetric graphs, whose
 * in-edges are the out-edges: the reference never builds A' for BFS, bfs.cpp:76-80). */
int orc_bfs_par(int64_t n, const int64_t *rp, const int64_t *ci, int64_t src, int symmetric,
                int64_t *level, int nthreads) {
    if (src < 0 || src >= n) return ORC_INVALID;
    orc_set_threads(nthreads);
    int64_t *front = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    int64_t *next = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    if (!front || !next) { free(front); free(next); return ORC_OOM; }
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) level[i] = INT64_MAX;
    level[src] = 0;
    front[0] = src;
    int64_t nf = 1, depth = 0;
    int64_t edges_unexplored = rp[n];
    int bottom_up = 0;
    while (nf > 0) {
        int64_t mf = 0;
        #pragma omp parallel for reduction(+:mf) schedule(static)
        for (int64_t i = 0; i < nf; i++) mf += rp[front[i] + 1] - rp[front[i]];
        edges_unexplored -= mf;
        if (symmetric && !bottom_up && mf > edges_unexplored / 14) bottom_up = 1;
        else if (bottom_up && nf < n / 24) bottom_up = 0;
        int64_t nn = 0;
        if (bottom_up) {
            #pragma omp parallel for reduction(+:nn) schedule(dynamic, 1024)
            for (int64_t v = 0; v < n; v++) {
                if (level[v] != INT64_MAX) continue;
                for (int64_t k = rp[v]; k < rp[v + 1]; k++)
                    if (level[ci[k]] == depth) { level[v] = depth + 1; nn++; break; }
            }
            /* the next frontier: vertices just reached (one pass, in vertex order) */
            int64_t m = 0;
            for (int64_t v = 0; v < n; v++) if (level[v] == depth + 1) next[m++] = v;
            nn = m;
        } else {
            #pragma omp parallel
            {
                int64_t buf[256];
                int nb = 0;
                #pragma omp for schedule(dynamic, 64)
                for (int64_t i = 0; i < nf; i++) {
                    const int64_t u = front[i];
                    for (int64_t k = rp[u]; k < rp[u + 1]; k++) {
                        const int64_t v = ci[k];
                        if (level[v] == INT64_MAX &&
                            __sync_bool_compare_and_swap(&level[v], INT64_MAX, depth + 1)) {
                            buf[nb++] = v;
                            if (nb == 256) {
                                const int64_t at = __sync_fetch_and_add(&nn, 256);
                                memcpy(next + at, buf, sizeof(buf));
                                nb = 0;
                            }
                        }
                    }
                }
                if (nb) {
                    const int64_t at = __sync_fetch_and_add(&nn, nb);
                    memcpy(next + at, buf, (size_t)nb * sizeof(int64_t));
                }
            }
        }
        int64_t *t = front; front = next; next = t;
        nf = nn;
        depth++;
    }
    free(front); free(next);
    return ORC_OK;
}

/* WCC: lock-free union-find (min-root linking by CAS, path halving), every stored edge
 * joins its endpoints, so directed graphs need no explicit A LOR A' (wcc.cpp:54-55).  Roots
 * are component minima, so the labels equal orc_wcc's. */
static int64_t par_find(int64_t *p, int64_t x) {
    for (;;) {
        int64_t y = __atomic_load_n(&p[x], __ATOMIC_RELAXED);
        if (y == x) return x;
        int64_t z = __atomic_load_n(&p[y], __ATOMIC_RELAXED);
        if (z != y) __sync_bool_compare_and_swap(&p[x], y, z);   /* halving */
        x = y;
    }
}

int orc_wcc_par(int64_t n, const int64_t *rp, const int64_t *ci, uint64_t *comp, int nthreads) {
    orc_set_threads(nthreads);
    int64_t *p = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    if (!p) return ORC_OOM;
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) p[i] = i;
    #pragma omp parallel for schedule(dynamic, 256)
    for (int64_t u = 0; u < n; u++) {
        for (int64_t k = rp[u]; k < rp[u + 1]; k++) {
            int64_t a = u, b = ci[k];
            for (;;) {
                a = par_find(p, a);
                b = par_find(p, b);
                if (a == b) break;
                if (a < b) { int64_t t = a; a = b; b = t; }      /* link the larger root */
                if (__sync_bool_compare_and_swap(&p[a], a, b)) break;
            }
        }
    }
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) comp[i] = (uint64_t)par_find(p, i);
    free(p);
    return ORC_OK;
}

/* SSSP: parallel delta-stepping (Meyer & Sanders; the GAP benchmark's shared-frontier form),
 * distances as fp64 bit patterns lowered by CAS (non-negative doubles order like their
 * bits).  Per-thread bins; the smallest non-empty bin of any thread is the next frontier;
 * a thread keeps processing its own current bin while it stays small (bin fusion).  The
 * result is the relaxation fixed point, bitwise equal to orc_sssp's Dijkstra. */
typedef struct { int64_t *v; int64_t len, cap; } orc_vec;

static int vec_push(orc_vec *b, int64_t x) {
    if (b->len == b->cap) {
        int64_t nc = b->cap ? 2 * b->cap : 64;
        int64_t *nv = (int64_t *)realloc(b->v, (size_t)nc * sizeof(int64_t));
        if (!nv) return 0;
        b->v = nv;
        b->cap = nc;
    }
    b->v[b->len++] = x;
    return 1;
}

static int relax_min(double *dist, int64_t v, double nd) {
    uint64_t *slot = (uint64_t *)&dist[v];
    uint64_t old = __atomic_load_n(slot, __ATOMIC_RELAXED);
    uint64_t nb;
    memcpy(&nb, &nd, 8);
    while (nb < old) {
        if (__atomic_compare_exchange_n(slot, &old, nb, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return 1;
    }
    return 0;
}

int orc_sssp_par(int64_t n, const int64_t *rp, const int64_t *ci, const double *w, int64_t src,
                 double delta, double *dist, int nthreads) {
    if (src < 0 || src >= n) return ORC_INVALID;
    if (!(delta > 0)) return ORC_INVALID;
    orc_set_threads(nthreads);
    const int64_t nnz = rp[n];
    const int64_t kMaxBin = INT64_MAX / 2;
    int64_t *frontier = (int64_t *)malloc((size_t)(nnz + n + 1) * sizeof(int64_t));
    if (!frontier) return ORC_OOM;
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) dist[i] = INFINITY;
    dist[src] = 0.0;
    frontier[0] = src;
    int64_t shared_bin[2] = {0, kMaxBin}, tails[2] = {1, 0};
    int oom = 0;
    #pragma omp parallel reduction(|:oom)
    {
        orc_vec *bins = NULL;
        int64_t nbins = 0;
        int64_t iter = 0;
        while (__atomic_load_n(&shared_bin[iter & 1], __ATOMIC_ACQUIRE) != kMaxBin) {
            int64_t *cur_bin = &shared_bin[iter & 1], *next_bin = &shared_bin[(iter + 1) & 1];
            int64_t *cur_tail = &tails[iter & 1], *next_tail = &tails[(iter + 1) & 1];
            const int64_t b = *cur_bin;
            const int64_t ct = *cur_tail;
            #define ORC_RELAX(u_)                                                              \
                do {                                                                           \
                    const int64_t uu = (u_);                                                   \
                    const double du = dist[uu];                                                \
                    for (int64_t k = rp[uu]; k < rp[uu + 1]; k++) {                             \
                        const double nd = du + w[k];                                           \
                        if (relax_min(dist, ci[k], nd)) {                                      \
                            const int64_t db = (int64_t)(nd / delta);                          \
                            if (db >= nbins) {                                                 \
                                orc_vec *nbs = (orc_vec *)realloc(bins, (size_t)(db + 1) * sizeof(orc_vec)); \
                                if (!nbs) { oom = 1; break; }                                  \
                                memset(nbs + nbins, 0, (size_t)(db + 1 - nbins) * sizeof(orc_vec)); \
                                bins = nbs;                                                    \
                                nbins = db + 1;                                                \
                            }                                                                  \
                            if (!vec_push(&bins[db], ci[k])) { oom = 1; break; }               \
                        }                                                                      \
                    }                                                                          \
                } while (0)
            #pragma omp for schedule(dynamic, 64) nowait
            for (int64_t i = 0; i < ct; i++) {
                const int64_t u = frontier[i];
                if (dist[u] >= delta * (double)b) ORC_RELAX(u);
            }
            /* bin fusion: keep going on this thread's own small current bin */
            while (b < nbins && bins[b].len > 0 && bins[b].len < 1000) {
                int64_t len = bins[b].len;
                int64_t *copy = (int64_t *)malloc((size_t)len * sizeof(int64_t));
                if (!copy) { oom = 1; break; }
                memcpy(copy, bins[b].v, (size_t)len * sizeof(int64_t));
                bins[b].len = 0;
                for (int64_t i = 0; i < len; i++) ORC_RELAX(copy[i]);
                free(copy);
            }
            #undef ORC_RELAX
            for (int64_t j = b; j < nbins; j++) {
                if (bins[j].len > 0) {
                    int64_t cur = __atomic_load_n(next_bin, __ATOMIC_RELAXED);
                    while (j < cur && !__atomic_compare_exchange_n(next_bin, &cur, j, 0, __ATOMIC_RELAXED,
                                                                   __ATOMIC_RELAXED)) {}
                    break;
                }
            }
            #pragma omp barrier
            #pragma omp single
            {
                *cur_bin = kMaxBin;
                *cur_tail = 0;
            }
            const int64_t nb = __atomic_load_n(next_bin, __ATOMIC_RELAXED);
            if (nb < nbins && bins[nb].len > 0) {
                const int64_t at = __atomic_fetch_add(next_tail, bins[nb].len, __ATOMIC_RELAXED);
                if (at + bins[nb].len <= nnz + n + 1)   /* a bin's pushes never exceed its edges in practice */
                    memcpy(frontier + at, bins[nb].v, (size_t)bins[nb].len * sizeof(int64_t));
                else
                    oom = 1;
                bins[nb].len = 0;
            }
            iter++;
            #pragma omp barrier
        }
        for (int64_t j = 0; j < nbins; j++) free(bins[j].v);
        free(bins);
    }
    free(frontier);
    return oom ? ORC_OOM : ORC_OK;
}

/* ====================================================================================
 * Op-level GraphBLAS restatements, the checkers of gx_mxv / gx_vxm / gx_mxm_masked
 * (include/gx.h).  The built-in semirings the reference's LAGraph calls use:
 *   PLUS_SECOND_FP64   GrB_mxv(t, .., LAGraph_plus_second_fp64, AT, w) in LAGr_PageRankGX
 *                      (pr.cpp:61)
 *   MIN_SECOND_UINT64  GrB_mxm(S, .., GrB_MIN_SECOND_SEMIRING_UINT64, S, L)
 *                      (LAGraph_cdlp.c:272-281); FastSV's mxv (LAGr_ConnectedComponents, wcc.cpp:61)
 *   ANY_PAIR_BOOL      the BFS frontier vxm (LAGr_BreadthFirstSearch, bfs.cpp:80)
 *   MIN_PLUS_FP64      the SSSP relaxation vxm (LAGr_SingleSourceShortestPath, sssp.cpp:78)
 *   PLUS_PAIR_INT64    triangle counts, masked mxm (LAGraph_lcc, lcc.cpp:68)
 * Semantics (GraphBLAS C API 2.0, dense vectors with a presence byte per entry):
 *   mxv: t(i) = (+)_{j : M(i,j) stored, u(j) present} mult(M(i,j), u(j)),  M = A, or A' with T0
 *   vxm: t(j) = (+)_{i : A(i,j) stored, u(i) present} mult(u(i), A(i,j)),  A' with T0
 *   (SECOND(x, y) = y, PLUS(x, y) = x + y, PAIR = 1; the matrix value is the fp64 weight, 1 for
 *   an unweighted graph); t(i) is present iff some term exists.  Then w<mask> (+)= t:
 *   where the (structural, optionally complemented) mask is false, w is kept (cleared with
 *   REPLACE); elsewhere w = t, or w (+) t with ACCUM.  Absent entries hold the monoid identity
 *   (0, UINT64_MAX, false, +inf, 0).
 *   mxm_masked: C<A> = A (+).(x) A' with PLUS_PAIR: c(e) for the stored entry e = (i, j) of A
 *   is |{k : A(i,k) and A(j,k) stored}| (the dot product of rows i and j; rows must not repeat a
 *   column), in A's entry order.
 * ==================================================================================== */
enum { ORC_PLUS_SECOND_FP64 = 0, ORC_MIN_SECOND_UINT64 = 1, ORC_ANY_PAIR_BOOL = 2, ORC_MIN_PLUS_FP64 = 3,
       ORC_PLUS_PAIR_INT64 = 4 };
#define ORC_DESC_T0 1
#define ORC_DESC_MASK_COMP 2
#define ORC_DESC_REPLACE 4
#define ORC_DESC_ACCUM 8

int orc_mxv(int64_t n, const int64_t *rp, const int64_t *ci, const double *wt, int sr, int vxm, int desc,
            const uint8_t *mask, const void *u, const uint8_t *u_present, void *out, uint8_t *out_present) {
    if (sr < 0 || sr > 4) return ORC_INVALID;
    const int use_t = (vxm != 0) ^ ((desc & ORC_DESC_T0) != 0);
    const int64_t *mrp = rp, *mci = ci;
    const double *mw = wt;
    int64_t *trp = NULL, *tci = NULL;
    double *tw = NULL;
    if (use_t) {
        int rc = orc_transpose(n, rp, ci, wt, &trp, &tci, wt ? &tw : NULL);
        if (rc) return rc;
        mrp = trp; mci = tci; mw = tw;
    }
    const double *ud = (const double *)u;
    const uint64_t *uu = (const uint64_t *)u;
    for (int64_t i = 0; i < n; i++) {
        double accd = (sr == ORC_MIN_PLUS_FP64) ? INFINITY : 0.0;
        uint64_t accu = UINT64_MAX;
        int64_t acci = 0;
        int hit = 0;
        for (int64_t k = mrp[i]; k < mrp[i + 1]; k++) {
            const int64_t j = mci[k];
            if (u_present && !u_present[j]) continue;
            const double a = mw ? mw[k] : 1.0;
            hit = 1;
            switch (sr) {
                case ORC_PLUS_SECOND_FP64: accd += vxm ? a : ud[j]; break;
                case ORC_MIN_SECOND_UINT64: {
                    /* GraphBLAS's fp64 -> uint64 typecast (GB_cast_to_uint64_t): saturating */
                    const uint64_t v = vxm ? (!(a > 0.0) ? 0 : a >= 18446744073709551616.0 ? UINT64_MAX : (uint64_t)a) : uu[j];
                    if (v < accu) accu = v;
                    break;
                }
                case ORC_MIN_PLUS_FP64: {
                    const double v = vxm ? ud[j] + a : a + ud[j];
                    if (v < accd) accd = v;
                    break;
                }
                case ORC_PLUS_PAIR_INT64: acci++; break;
                default: break;   /* ANY_PAIR: the hit itself */
            }
        }
        const int allowed = !mask || ((mask[i] != 0) != ((desc & ORC_DESC_MASK_COMP) != 0));
        const int old = out_present ? out_present[i] != 0 : 1;
        int present = hit;
        if (!allowed) {
            if (!(desc & ORC_DESC_REPLACE)) continue;
            present = 0;
            hit = 0;
        } else if ((desc & ORC_DESC_ACCUM) && old) {
            present = 1;
            if (hit) {
                switch (sr) {
                    case ORC_PLUS_SECOND_FP64: accd = ((double *)out)[i] + accd; break;
                    case ORC_MIN_SECOND_UINT64: if (((uint64_t *)out)[i] < accu) accu = ((uint64_t *)out)[i]; break;
                    case ORC_MIN_PLUS_FP64: if (((double *)out)[i] < accd) accd = ((double *)out)[i]; break;
                    case ORC_PLUS_PAIR_INT64: acci += ((int64_t *)out)[i]; break;
                    default: break;
                }
            } else {
                if (out_present) out_present[i] = 1;
                continue;   /* w(i) kept */
            }
        }
        if (out_present) out_present[i] = (uint8_t)present;
        switch (sr) {
            case ORC_PLUS_SECOND_FP64: ((double *)out)[i] = present ? accd : 0.0; break;
            case ORC_MIN_SECOND_UINT64: ((uint64_t *)out)[i] = present ? accu : UINT64_MAX; break;
            case ORC_ANY_PAIR_BOOL: ((uint8_t *)out)[i] = (uint8_t)(present ? 1 : 0); break;
            case ORC_MIN_PLUS_FP64: ((double *)out)[i] = present ? accd : INFINITY; break;
            default: ((int64_t *)out)[i] = present ? acci : 0; break;
        }
    }
    free(trp); free(tci); free(tw);
    return ORC_OK;
}

int orc_mxm_masked(int64_t n, const int64_t *rp, const int64_t *ci, int sr, int desc, int64_t *c) {
    if (sr != ORC_PLUS_PAIR_INT64 || desc != 0) return ORC_INVALID;
    const int64_t nnz = rp[n];
    int64_t *s = (int64_t *)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int64_t));
    if (!s) return ORC_OOM;
    memcpy(s, ci, (size_t)nnz * sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) qsort(s + rp[i], (size_t)(rp[i + 1] - rp[i]), sizeof(int64_t), cmp_u64);
    #pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < n; i++) {
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            const int64_t j = ci[e];
            int64_t a = rp[i], b = rp[j], cnt = 0;
            while (a < rp[i + 1] && b < rp[j + 1]) {
                if (s[a] < s[b]) a++;
                else if (s[a] > s[b]) b++;
                else { cnt++; a++; b++; }
            }
            c[e] = cnt;
        }
    }
    free(s);
    return ORC_OK;
}
