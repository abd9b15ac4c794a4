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
