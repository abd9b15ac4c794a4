// gx_wcc.hip -- weakly connected components: Afforest (undirected) / min-label hooking
// (directed), with pointer jumping.
//
// Replaces WeaklyConnectedComponents -> GrB_eWiseAdd(A, LOR, A, A') + LAGr_ConnectedComponents
// (wcc.cpp:39-66).  Every stored edge (u, v) is treated as undirected, so the explicit
// symmetrisation the reference performs inside processing time is not needed.
// Undirected graphs (every edge stored at both endpoints), Afforest (Sutton et al.):
//   sample   : two rounds linking each vertex with its r-th neighbour (CAS hooking), each
//              followed by pointer jumping;
//   giant    : the most frequent root among 1024 hashed vertices;
//   finish   : one wave per vertex outside the giant component links its remaining neighbours.
// Directed graphs (an edge is seen from one endpoint only): the same two sampling rounds over
//   out-neighbours, then one edge-balanced pass (kWccEdgesPerThread entries per thread) links
//   every remaining entry with the CAS link -- no vertex can be skipped -- and pointer
//   jumping until every vertex points at its root.  (Min-label hooking repeated until no
//   change took 2.48 ms on SYN-cit.)
// parent[v] <= v always holds, so the root of each final tree is the smallest vertex index
// of the component: comp[v] is canonical and equals the oracle's union-find labels exactly.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "gx_device.h"

namespace gx {
namespace {

constexpr int kWccBlock = 256;
constexpr int kWccEdgesPerThread = 16;

__device__ __forceinline__ int32_t find_root(const int32_t *parent, int32_t v) {
    int32_t p = parent[v];
    while (p != v) {
        v = p;
        p = parent[v];
    }
    return v;
}

__global__ __launch_bounds__(kWccBlock) void k_wcc_compress(int32_t *parent, int64_t n) {
    for (int64_t v = (int64_t)blockIdx.x * kWccBlock + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * kWccBlock) {
        int32_t p = parent[v];
        int32_t pp = parent[p];
        while (p != pp) {
            p = pp;
            pp = parent[p];
        }
        parent[v] = p;
    }
}

// Afforest link (Sutton et al., IPDPS'18): hook the higher of the two roots below the lower
// one with a CAS; parent[x] <= x is kept, so roots stay component minima.
__device__ __forceinline__ void link(int32_t *parent, int32_t u, int32_t v) {
    int32_t p1 = __hip_atomic_load(&parent[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int32_t p2 = __hip_atomic_load(&parent[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (p1 != p2) {
        const int32_t high = max(p1, p2), low = min(p1, p2);
        const int32_t ph = __hip_atomic_load(&parent[high], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ph == low) break;
        if (ph == high && atomicCAS(&parent[high], high, low) == high) break;
        p1 = __hip_atomic_load(&parent[ph], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        p2 = __hip_atomic_load(&parent[low], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Afforest sampling round 0 from the identity forest without atomics: a vertex whose first
// neighbour is smaller points at it (plain store of its own entry; pointers only go down, so
// no cycle), and only the vertices whose first neighbour is larger link in a second pass.
__global__ __launch_bounds__(kWccBlock) void k_afforest_hook0(const int64_t *__restrict__ rp,
                                                              const int32_t *__restrict__ ci, int64_t n,
                                                              int32_t *parent) {
    for (int64_t v = (int64_t)blockIdx.x * kWccBlock + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * kWccBlock) {
        const int64_t k = rp[v];
        if (k < rp[v + 1]) {
            const int32_t u = ci[k];
            if (u < (int32_t)v) parent[v] = u;
        }
    }
}

__global__ __launch_bounds__(kWccBlock) void k_afforest_link0(const int64_t *__restrict__ rp,
                                                              const int32_t *__restrict__ ci, int64_t n,
                                                              int32_t *parent) {
    for (int64_t v = (int64_t)blockIdx.x * kWccBlock + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * kWccBlock) {
        const int64_t k = rp[v];
        if (k < rp[v + 1]) {
            const int32_t u = ci[k];
            if (u > (int32_t)v) link(parent, (int32_t)v, u);
        }
    }
}

// Afforest sampling round r >= 1, first pass, on a compressed forest: the roots of v and of its
// r-th neighbour are joined by an atomicMin of the higher root's parent (issued only if it
// lowers it).  Many pairs target the same root, and there CAS links retried in series (534 us
// of a 1.1 ms WCC on SYN-g500-22); here the lowest wins at once and the pairs whose union was
// lost are few and retried by k_afforest_sample with distinct targets.  Pointers only go
// down, so no cycle; only pointers of roots change, so earlier unions stand.
__global__ __launch_bounds__(kWccBlock) void k_afforest_minhook(const int64_t *__restrict__ rp,
                                                                const int32_t *__restrict__ ci, int64_t n, int r,
                                                                int32_t *parent) {
    // wave-uniform trip count: the ballots and shuffles below see every lane
    for (int64_t base = (int64_t)blockIdx.x * kWccBlock + (threadIdx.x & ~(kWave - 1)); base < n;
         base += (int64_t)gridDim.x * kWccBlock) {
        const int64_t v = base + (threadIdx.x & (kWave - 1));
        const int64_t k = v < n ? rp[v] + r : 0;
        int32_t high = 0, low = 0;
        bool want = false;
        if (v < n && k < rp[v + 1]) {
            const int32_t r1 = __hip_atomic_load(&parent[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int32_t r2 = __hip_atomic_load(&parent[ci[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            high = max(r1, r2);
            low = min(r1, r2);
            want = r1 != r2 && low < __hip_atomic_load(&parent[high], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // lanes aiming at the same root as the first remaining lane send one atomic with their
        // smallest low (two rounds): a few hot roots drew most of the atomics, in series
        const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
        for (int round = 0; round < 2; round++) {
            const unsigned long long act = __ballot(want);
            if (!act) break;
            const int first = __ffsll((long long)act) - 1;
            const int32_t lead = __shfl(high, first, kWave);
            const bool same = want && high == lead;
            int32_t m = same ? low : 0x7fffffff;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) m = min(m, __shfl_xor(m, off, kWave));
            if (lane == first) __hip_atomic_fetch_min(&parent[lead], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            want = want && !same;
        }
        if (want) __hip_atomic_fetch_min(&parent[high], low, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Afforest sampling round r: link every vertex with its r-th neighbour.
__global__ __launch_bounds__(kWccBlock) void k_afforest_sample(const int64_t *__restrict__ rp,
                                                               const int32_t *__restrict__ ci, int64_t n,
                                                               int r, int32_t *parent) {
    for (int64_t v = (int64_t)blockIdx.x * kWccBlock + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * kWccBlock) {
        const int64_t k = rp[v] + r;
        if (k < rp[v + 1]) link(parent, (int32_t)v, ci[k]);
    }
}

// Afforest finish: every vertex outside the sampled giant component links all its remaining
// neighbours (undirected graphs store every edge at both endpoints, so an edge between the
// giant component and another vertex is seen from the other vertex).  One wave per vertex.
__global__ __launch_bounds__(kWccBlock) void k_afforest_finish(const int64_t *__restrict__ rp,
                                                               const int32_t *__restrict__ ci, int64_t n,
                                                               int skip, const int32_t *giant_p, int32_t *parent) {
    const int lane = threadIdx.x & (kWave - 1);
    const int32_t giant = *giant_p;
    const int64_t w0 = ((int64_t)blockIdx.x * kWccBlock + threadIdx.x) / kWave;
    const int64_t nw = (int64_t)gridDim.x * (kWccBlock / kWave);
    // the giant-component test for 64 vertices at once (one per lane, coalesced), then the
    // wave links the rows of the few outside it (a wave walking its vertices one by one spent
    // a dependent root lookup per vertex)
    for (int64_t base = w0 * kWave; base < n; base += nw * kWave) {
        const int64_t v = base + lane;
        int64_t b = 0, e = 0;
        bool need = false;
        if (v < n) {
            b = rp[v] + skip;
            e = rp[v + 1];
            need = b < e && find_root(parent, (int32_t)v) != giant;
        }
        unsigned long long m = __ballot(need);
        while (m) {
            const int l = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int64_t vb = __shfl(b, l, kWave), ve = __shfl(e, l, kWave);
            for (int64_t k = vb + lane; k < ve; k += kWave) link(parent, (int32_t)(base + l), ci[k]);
        }
    }
}

// Directed graphs: an edge is stored at its source only, so no vertex may skip its row (the
// giant-component shortcut above relies on seeing every edge from both ends).  After the two
// sampling rounds, one edge-balanced pass links every remaining entry (row position >= 2):
// Afforest's CAS link is a complete concurrent union, so one pass suffices.
__global__ __launch_bounds__(kWccBlock) void k_wcc_link_edges(const int64_t *__restrict__ rp,
                                                              const int32_t *__restrict__ ci, int64_t n,
                                                              int64_t nnz, int skip, int32_t *parent) {
    const int64_t t = (int64_t)blockIdx.x * kWccBlock + threadIdx.x;
    const int64_t e0 = t * kWccEdgesPerThread;
    if (e0 >= nnz) return;
    const int64_t e1 = min(e0 + kWccEdgesPerThread, nnz);
    int64_t r = row_of_edge(rp, n, e0);
    for (int64_t e = e0; e < e1; e++) {
        while (rp[r + 1] <= e) r++;
        if (e - rp[r] >= skip) link(parent, (int32_t)r, ci[e]);
    }
}

// Afforest's giant component: the most frequent root among kSamples sampled vertices (ties:
// the smallest root), chosen by one workgroup, so the host does not wait for the samples
// between the passes.  The roots are counted in an LDS hash table (linear probing, CAS-claimed
// keys, atomic counts).  Each thread scanning all samples (O(kSamples^2) LDS reads on one CU)
// took 20 us of a 169 us WCC run.  Any root would be correct (the finish links every edge of
// the vertices outside it); the most frequent one skips the most.
constexpr int kSamples = 1024;
constexpr int kGiantSlots = 2 * kSamples;

__global__ __launch_bounds__(kSamples) void k_pick_giant(const int32_t *parent, const int32_t *__restrict__ ids,
                                                         int32_t *giant) {
    __shared__ int32_t keys[kGiantSlots];
    __shared__ uint32_t cnts[kGiantSlots];
    __shared__ unsigned long long best[kSamples / kWave];
    const int t = threadIdx.x;
    for (int i = t; i < kGiantSlots; i += kSamples) {
        keys[i] = -1;
        cnts[i] = 0;
    }
    const int32_t r = find_root(parent, ids[t]);
    __syncthreads();
    uint32_t h = ((uint32_t)r * 2654435761u) >> 21;   // 11 bits: kGiantSlots
    for (;;) {
        const int32_t k = atomicCAS(&keys[h], -1, r);
        if (k == -1 || k == r) break;
        h = (h + 1) & (kGiantSlots - 1);
    }
    atomicAdd(&cnts[h], 1u);
    __syncthreads();
    const uint32_t c = cnts[h];
    unsigned long long key = ((unsigned long long)c << 32) | (uint32_t)(0x7fffffff - r);
    for (int off = kWave / 2; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, kWave);
        key = o > key ? o : key;
    }
    if ((t & (kWave - 1)) == 0) best[t / kWave] = key;
    __syncthreads();
    if (t == 0) {
        for (int w = 1; w < kSamples / kWave; w++) key = best[w] > key ? best[w] : key;
        *giant = 0x7fffffff - (int32_t)(uint32_t)key;
    }
}

__global__ void k_iota(int32_t *a, int64_t n) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x)
        a[v] = (int32_t)v;
}

// Afforest's sampling rounds (each vertex with its first, then its second neighbour), each
// followed by pointer jumping: round 0 by k_afforest_hook0/link0, round 1 by min-hook passes
// before the CAS links (GX_WCC_HOOK0=0 / GX_WCC_MINHOOK=0: CAS links only).
int afforest_sample(gx_graph *g, int32_t *parent, unsigned vgrid, int rounds, hipStream_t s) {
    gx_ctx *ctx = g->ctx;
    const int64_t n = (int64_t)g->n;
    // default on for undirected graphs only: on SYN-cit (directed, out-neighbours) the
    // passes cost more than the CAS links they spare (1.21 vs 1.09 ms)
    const bool und = !g->directed;
    const bool hook0 = std::getenv("GX_WCC_HOOK0") ? std::atoi(std::getenv("GX_WCC_HOOK0")) != 0 : und;
    const int minhook = std::getenv("GX_WCC_MINHOOK") ? std::atoi(std::getenv("GX_WCC_MINHOOK")) : (und ? 1 : 0);
    for (int r = 0; r < rounds; r++) {
        for (int pass = 0; r > 0 && pass < minhook; pass++) {
            KTimer kt(ctx, "wcc_sample", s);
            hipLaunchKernelGGL(k_afforest_minhook, dim3(vgrid), dim3(kWccBlock), 0, s, g->A.rp.p, g->A.ci.p, n, r,
                               parent);
            hipLaunchKernelGGL(k_wcc_compress, dim3(vgrid), dim3(kWccBlock), 0, s, parent, n);
        }
        {
            KTimer kt(ctx, "wcc_sample", s);
            if (r == 0 && hook0) {
                hipLaunchKernelGGL(k_afforest_hook0, dim3(vgrid), dim3(kWccBlock), 0, s, g->A.rp.p, g->A.ci.p, n,
                                   parent);
                hipLaunchKernelGGL(k_afforest_link0, dim3(vgrid), dim3(kWccBlock), 0, s, g->A.rp.p, g->A.ci.p, n,
                                   parent);
            } else {
                hipLaunchKernelGGL(k_afforest_sample, dim3(vgrid), dim3(kWccBlock), 0, s, g->A.rp.p, g->A.ci.p, n,
                                   r, parent);
            }
        }
        GX_TRY(check_launch("k_afforest_sample"));
        {
            KTimer kt(ctx, "wcc_compress", s);
            hipLaunchKernelGGL(k_wcc_compress, dim3(vgrid), dim3(kWccBlock), 0, s, parent, n);
        }
        GX_TRY(check_launch("k_wcc_compress"));
    }
    return GX_SUCCESS;
}

// Labels of a run on the hub-first copy (gx_graph::out_perm): a component's label is its
// smallest vertex id in the caller's numbering, the min of order[] over its members.  The
// giant component's members (root `giant`) meet in a workgroup min first, since one word
// taking an atomic per member would serialise millions of them; the rest take one each.
__global__ __launch_bounds__(kWccBlock) void k_wcc_min_orig(const int32_t *__restrict__ parent,
                                                            const int32_t *__restrict__ order, int64_t n,
                                                            const int32_t *giant_p, int32_t *__restrict__ minorig) {
    __shared__ int32_t wmin[kWccBlock / kWave];
    const int32_t giant = giant_p ? *giant_p : -1;
    int32_t lm = 0x7fffffff;
    for (int64_t x = (int64_t)blockIdx.x * kWccBlock + threadIdx.x; x < n; x += (int64_t)gridDim.x * kWccBlock) {
        const int32_t r = parent[x], o = order[x];
        if (r == giant) lm = min(lm, o);
        else atomicMin(&minorig[r], o);
    }
    for (int off = kWave / 2; off > 0; off >>= 1) lm = min(lm, __shfl_xor(lm, off, kWave));
    if ((threadIdx.x & (kWave - 1)) == 0) wmin[threadIdx.x / kWave] = lm;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kWccBlock / kWave; w++) lm = min(lm, wmin[w]);
        // one atomic per workgroup on one word serialised (2 048 of them, 26 us per run on
        // SYN-g500-22): only a workgroup whose minimum beats the word's current value sends one
        if (giant >= 0 && lm != 0x7fffffff &&
            lm < __hip_atomic_load(&minorig[giant], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(&minorig[giant], lm);
    }
}

// out[v] = the label of v's component, gathered through perm (x = perm[v], the hub-first
// position of caller vertex v); vertices past `live` have no edges and are their own component.
// Coalesced stores: the scatter below took 30 us per run on SYN-g500-22 (r05_wcc_kernel_stats.csv).
__global__ void k_wcc_label_gather(const int32_t *__restrict__ parent, const int32_t *__restrict__ perm,
                                   const int32_t *__restrict__ minorig, int64_t n, int64_t live,
                                   int32_t *__restrict__ out) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const int32_t x = perm[v];
        out[v] = x < live ? minorig[parent[x]] : (int32_t)v;
    }
}

// The same as a scatter through order (GX_REMAP=scatter): streaming reads, random stores.
__global__ void k_wcc_label_orig(const int32_t *__restrict__ parent, const int32_t *__restrict__ order,
                                 const int32_t *__restrict__ minorig, int64_t n, int64_t live,
                                 int32_t *__restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t o = order[x];
        out[o] = x < live ? minorig[parent[x]] : o;
    }
}

}  // namespace
}  // namespace gx

using namespace gx;

extern "C" int gx_wcc(gx_graph *g, uint64_t *comp) {
    if (!g || !comp) return fail(GX_NULL_POINTER, "gx_wcc: null argument");
    gx_ctx *ctx = g->ctx;
    GX_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t n = (int64_t)g->n, nnz = (int64_t)g->nnz;
    if (n == 0) return GX_SUCCESS;
    {
        gx_graph *h = nullptr;   // hub-first copy from the second call (gx_runtime.hip hub_for)
        GX_TRY(hub_for(g, ++g->wcc_calls, &h, nullptr));
        if (h) return gx_wcc(h, comp);
    }
    int32_t *giant_d = nullptr;   // device word holding the giant component's root
    DBuf<int32_t> parent;
    GX_TRY(parent.alloc(n));
    GX_TRY(device_begin(ctx));
    hipLaunchKernelGGL(k_iota, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, parent.p, n);
    GX_TRY(check_launch("k_iota"));
    const unsigned vgrid = grid_for(n, kWccBlock, 8192);
    if (!g->directed && nnz) {
        // ---- Afforest: sample two neighbours per vertex, find the giant component from
        // 1024 sampled roots, then link only the remaining edges of the other vertices.  On the
        // hub-first copy with sorted rows one round suffices: every first neighbour is the
        // vertex's largest hub, so that round already joins the giant component (build_hub,
        // gx_runtime.hip); GX_WCC_ROUNDS overrides (1 or 2).
        int rounds = g->rows_sorted ? 1 : 2;
        if (const char *e = std::getenv("GX_WCC_ROUNDS")) rounds = std::max(1, std::min(2, std::atoi(e)));
        GX_TRY(afforest_sample(g, parent.p, vgrid, rounds, s));
        // sample ids: a fixed hash sequence, uploaded once per graph size
        if (!g->wcc_ids.p || g->wcc_ids_n != n) {
            std::vector<int32_t> ids(kSamples);
            uint64_t h = 0x9E3779B97F4A7C15ull;
            for (int i = 0; i < kSamples; i++) {
                h ^= h >> 31;
                h *= 0xBF58476D1CE4E5B9ull;
                h ^= h >> 29;
                ids[i] = (int32_t)(h % (uint64_t)n);
            }
            GX_TRY(g->wcc_ids.alloc(kSamples + 1));   // + the chosen root
            GX_HIP_TRY(hipMemcpy(g->wcc_ids.p, ids.data(), kSamples * 4, hipMemcpyHostToDevice));
            g->wcc_ids_n = n;
        }
        giant_d = g->wcc_ids.p + kSamples;
        hipLaunchKernelGGL(k_pick_giant, dim3(1), dim3(kSamples), 0, s, parent.p, g->wcc_ids.p, giant_d);
        GX_TRY(check_launch("k_pick_giant"));
        {
            KTimer kt(ctx, "wcc_hook", s);
            hipLaunchKernelGGL(k_afforest_finish, dim3(grid_for((uint64_t)n, kWccBlock, 8192)),
                               dim3(kWccBlock), 0, s, g->A.rp.p, g->A.ci.p, n, rounds, giant_d, parent.p);
        }
        GX_TRY(check_launch("k_afforest_finish"));
        {
            KTimer kt(ctx, "wcc_compress", s);
            hipLaunchKernelGGL(k_wcc_compress, dim3(vgrid), dim3(kWccBlock), 0, s, parent.p, n);
        }
        GX_TRY(check_launch("k_wcc_compress"));
    }
    if (g->directed && nnz) {
        GX_TRY(afforest_sample(g, parent.p, vgrid, 2, s));
        {
            KTimer kt(ctx, "wcc_hook", s);
            hipLaunchKernelGGL(k_wcc_link_edges,
                               dim3(grid_for((uint64_t)((nnz + kWccEdgesPerThread - 1) / kWccEdgesPerThread),
                                             kWccBlock, 1u << 30)),
                               dim3(kWccBlock), 0, s, g->A.rp.p, g->A.ci.p, n, nnz, 2, parent.p);
        }
        GX_TRY(check_launch("k_wcc_link_edges"));
        {
            KTimer kt(ctx, "wcc_compress", s);
            hipLaunchKernelGGL(k_wcc_compress, dim3(vgrid), dim3(kWccBlock), 0, s, parent.p, n);
        }
        GX_TRY(check_launch("k_wcc_compress"));
    }
    const int32_t *res = parent.p;
    if (g->out_perm) {
        int32_t *minorig = reinterpret_cast<int32_t *>(g->remap_tmp.p), *lab = minorig + n;   // 2n int32
        const int64_t live = g->live;   // roots of components with edges are below it
        if (live) {
            GX_HIP_TRY(hipMemsetAsync(minorig, 0x7f, (size_t)live * 4, s));
            hipLaunchKernelGGL(k_wcc_min_orig, dim3(grid_for((uint64_t)live, kWccBlock, 2048)), dim3(kWccBlock), 0,
                               s, parent.p, g->out_order, live, giant_d, minorig);
        }
        const char *re = std::getenv("GX_REMAP");
        if (re && std::strcmp(re, "scatter") == 0)
            hipLaunchKernelGGL(k_wcc_label_orig, dim3(vgrid), dim3(256), 0, s, parent.p, g->out_order, minorig, n,
                               live, lab);
        else
            hipLaunchKernelGGL(k_wcc_label_gather, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, parent.p,
                               g->out_perm, minorig, n, live, lab);
        GX_TRY(check_launch("k_wcc_label_orig"));
        res = lab;
    }
    GX_TRY(device_end(ctx));
    GX_TRY(download(ctx, comp, res, (uint64_t)n, Xfer::Widen32));
    return GX_SUCCESS;
}

GX_MODULE_WARMER(wcc)
