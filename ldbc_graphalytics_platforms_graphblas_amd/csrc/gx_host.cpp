// gx_host.cpp -- host side of libgx that needs no GPU: `.grb`/`.vtb` I/O without
// SuiteSparse and the seeded R-MAT generator used by the bench and the tests.
//
// .grb layout (reference include/graphio.h:49-285 binread, :310-615 binwrite; format of
// SuiteSparse:GraphBLAS v7 serialisation as written by LAGraph's binwrite):
//   char header[512]                       informational ASCII
//   int32  fmt        GxB_BY_ROW=0 / GxB_BY_COL=1
//   int32  kind       1 hyper, 2 sparse (0 legacy sparse), 4 bitmap, 8 full; +100 if iso
//   double hyper      hyper switch
//   uint64 nrows, ncols
//   int64  nonempty
//   uint64 nvec, nvals
//   int32  typecode   0 BOOL ... 8 UINT64, 9 FP32, 10 FP64
//   size_t typesize
//   then Ap[nvec+1], [Ah[nvec]], Ai[nvals] (uint64), Ax[iso ? 1 : nvals] (typesize each)
//   (bitmap: Ab[nrows*ncols] int8 presence bytes, then Ax[iso ? 1 : nrows*ncols];
//    full: Ax[iso ? 1 : nrows*ncols] only -- graphio.h:175-186, 211-216)
#include <algorithm>
#include <cctype>
#include <cinttypes>
#include <emmintrin.h>
#include <smmintrin.h>
#include <tmmintrin.h>
#include <cmath>
#include <cstring>
#include <memory>
#include <numeric>
#include <vector>

#include <omp.h>

#include "gx_internal.h"

namespace gx {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg) {
    set_error(msg);
    return code;
}

}  // namespace gx

using gx::fail;

extern "C" const char *gx_last_error(void) { return gx::g_last_error.c_str(); }

extern "C" void gx_host_free(void *p) { std::free(p); }

extern "C" void gx_csr_release(gx_csr *csr) {
    if (!csr) return;
    std::free(csr->rowptr);
    std::free(csr->colidx);
    std::free(csr->vals);
    csr->rowptr = nullptr;
    csr->colidx = nullptr;
    csr->vals = nullptr;
    csr->n = csr->nnz = 0;
}

namespace {

struct FileCloser {
    void operator()(FILE *f) const {
        if (f) std::fclose(f);
    }
};
using FilePtr = std::unique_ptr<FILE, FileCloser>;

template <typename T>
bool read_n(FILE *f, T *p, size_t n) {
    return n == 0 || std::fread(p, sizeof(T), n, f) == n;
}

template <typename T>
T *xmalloc(size_t n) {
    return static_cast<T *>(std::malloc(std::max<size_t>(n, 1) * sizeof(T)));
}

// Convert one stored value of GrB type `typecode` to fp64.
double value_as_double(const unsigned char *p, int32_t typecode) {
    switch (typecode) {
        case 0: return *reinterpret_cast<const bool *>(p) ? 1.0 : 0.0;
        case 1: return *reinterpret_cast<const int8_t *>(p);
        case 2: return *reinterpret_cast<const int16_t *>(p);
        case 3: return *reinterpret_cast<const int32_t *>(p);
        case 4: return (double)*reinterpret_cast<const int64_t *>(p);
        case 5: return *reinterpret_cast<const uint8_t *>(p);
        case 6: return *reinterpret_cast<const uint16_t *>(p);
        case 7: return *reinterpret_cast<const uint32_t *>(p);
        case 8: return (double)*reinterpret_cast<const uint64_t *>(p);
        case 9: return *reinterpret_cast<const float *>(p);
        case 10: return *reinterpret_cast<const double *>(p);
        default: return 0.0;
    }
}

// Build a row-major CSR (sorted rows) from a column-major one: a counting-sort transpose.
void csc_to_csr(uint64_t nrows, uint64_t ncols, const uint64_t *cp, const uint64_t *ri,
                const double *cx, uint64_t *rp, uint64_t *ci, double *rx) {
    std::fill(rp, rp + nrows + 1, 0);
    uint64_t nnz = cp[ncols];
    for (uint64_t k = 0; k < nnz; k++) rp[ri[k] + 1]++;
    for (uint64_t i = 0; i < nrows; i++) rp[i + 1] += rp[i];
    std::vector<uint64_t> cur(rp, rp + nrows);
    for (uint64_t j = 0; j < ncols; j++)
        for (uint64_t k = cp[j]; k < cp[j + 1]; k++) {
            uint64_t d = cur[ri[k]]++;
            ci[d] = j;
            if (rx) rx[d] = cx[k];
        }
}

}  // namespace

extern "C" int gx_read_grb(const char *path, gx_csr *out) {
    if (!path || !out) return fail(GX_NULL_POINTER, "gx_read_grb: null argument");
    std::memset(out, 0, sizeof(*out));
    FilePtr f(std::fopen(path, "rb"));
    if (!f) return fail(GX_IO_ERROR, std::string("cannot open ") + path);
    char header[512];
    int32_t fmt = 0, kind = 0, typecode = 0;
    double hyper = 0;
    uint64_t nrows = 0, ncols = 0, nvec = 0, nvals = 0;
    int64_t nonempty = 0;
    uint64_t typesize = 0;   // size_t on the LP64 writer
    FILE *fp = f.get();
    if (!read_n(fp, header, 512) || !read_n(fp, &fmt, 1) || !read_n(fp, &kind, 1) ||
        !read_n(fp, &hyper, 1) || !read_n(fp, &nrows, 1) || !read_n(fp, &ncols, 1) ||
        !read_n(fp, &nonempty, 1) || !read_n(fp, &nvec, 1) || !read_n(fp, &nvals, 1) ||
        !read_n(fp, &typecode, 1) || !read_n(fp, &typesize, 1))
        return fail(GX_IO_ERROR, std::string("truncated .grb header: ") + path);
    bool iso = false;
    if (kind > 100) {
        iso = true;
        kind -= 100;
    }
    // kinds as binread decodes them (graphio.h:114-117): 1 hyper, 0/2 sparse, 4 bitmap, 8 full
    const bool is_hyper = kind == 1;
    const bool is_sparse = kind == 0 || kind == 2;
    const bool is_bitmap = kind == 4;
    const bool is_full = kind == 8;
    if (!is_hyper && !is_sparse && !is_bitmap && !is_full)
        return fail(GX_NOT_IMPLEMENTED, "unknown .grb matrix kind");
    if (typecode < 0 || typecode > 10 || typesize == 0 || typesize > 16)
        return fail(GX_NOT_IMPLEMENTED, "unsupported .grb value type");
    if (fmt != 0 && fmt != 1) return fail(GX_INVALID_VALUE, "bad .grb format field");
    if (nrows != ncols) return fail(GX_INVALID_VALUE, "adjacency matrix must be square");
    const uint64_t nmajor = fmt == 0 ? nrows : ncols;
    const uint64_t nminor = fmt == 0 ? ncols : nrows;
    // Weighted iff the values are floating point (relabel.py:11-16 writes FP64 for weighted
    // graphs and BOOL iso for unweighted ones).  An iso FP32/FP64 matrix -- SuiteSparse stores
    // one when every weight is equal -- is weighted too, each entry carrying the one value.
    const bool weighted = typecode == 9 || typecode == 10;

    // The major dimension as a full pointer array P, the minor index of every entry in Ai and,
    // for weighted graphs, its value in X.
    std::vector<uint64_t> P(nmajor + 1, 0), Ai;
    std::vector<double> X;
    if (is_hyper || is_sparse) {
        if (is_sparse && nvec != nmajor) nvec = nmajor;   // sparse: nvec = vdim
        std::vector<uint64_t> Ap(nvec + 1), Ah(is_hyper ? nvec : 0);
        Ai.resize(nvals);
        if (!read_n(fp, Ap.data(), nvec + 1)) return fail(GX_IO_ERROR, "truncated Ap");
        if (is_hyper && !read_n(fp, Ah.data(), nvec)) return fail(GX_IO_ERROR, "truncated Ah");
        if (!read_n(fp, Ai.data(), nvals)) return fail(GX_IO_ERROR, "truncated Ai");
        const uint64_t nx = iso ? 1 : nvals;
        std::vector<unsigned char> Ax(nx * typesize);
        if (!read_n(fp, Ax.data(), Ax.size())) return fail(GX_IO_ERROR, "truncated Ax");
        if (Ap[0] != 0 || Ap[nvec] != nvals) return fail(GX_INVALID_VALUE, "corrupt Ap");
        for (uint64_t k = 0; k < nvals; k++)
            if (Ai[k] >= nminor) return fail(GX_INVALID_INDEX, "column index out of range");
        if (is_hyper) {
            for (uint64_t k = 0; k < nvec; k++) {
                if (Ah[k] >= nmajor) return fail(GX_INVALID_INDEX, "hyper index out of range");
                P[Ah[k] + 1] = Ap[k + 1] - Ap[k];
            }
            for (uint64_t i = 0; i < nmajor; i++) P[i + 1] += P[i];
        } else {
            P.assign(Ap.begin(), Ap.end());
        }
        if (weighted) {
            X.resize(nvals);
            for (uint64_t k = 0; k < nvals; k++) X[k] = value_as_double(&Ax[(iso ? 0 : k) * typesize], typecode);
        }
    } else {
        // bitmap / full (graphio.h:175-186, 211-216): nrows*ncols cells in major order, a
        // presence byte per cell for bitmap (full: every cell present), then the values.
        if (nrows > (1ull << 20)) return fail(GX_NOT_IMPLEMENTED, "dense .grb kind too large for a graph");
        const uint64_t cells = nrows * ncols;
        std::vector<int8_t> Ab(is_bitmap ? cells : 0);
        if (is_bitmap && !read_n(fp, Ab.data(), cells)) return fail(GX_IO_ERROR, "truncated Ab");
        const uint64_t nx = iso ? 1 : cells;
        std::vector<unsigned char> Ax(nx * typesize);
        if (!read_n(fp, Ax.data(), Ax.size())) return fail(GX_IO_ERROR, "truncated Ax");
        for (uint64_t m = 0; m < nmajor; m++) {
            for (uint64_t j = 0; j < nminor; j++) {
                const uint64_t cell = m * nminor + j;
                if (is_bitmap && !Ab[cell]) continue;
                Ai.push_back(j);
                if (weighted) X.push_back(value_as_double(&Ax[(iso ? 0 : cell) * typesize], typecode));
            }
            P[m + 1] = Ai.size();
        }
        nvals = Ai.size();
    }

    out->n = nrows;
    out->nnz = nvals;
    out->rowptr = xmalloc<uint64_t>(nrows + 1);
    out->colidx = xmalloc<uint64_t>(nvals);
    out->vals = weighted ? xmalloc<double>(nvals) : nullptr;
    if (!out->rowptr || !out->colidx || (weighted && !out->vals)) {
        gx_csr_release(out);
        return fail(GX_OUT_OF_MEMORY, "gx_read_grb: out of memory");
    }
    if (fmt == 0) {
        std::memcpy(out->rowptr, P.data(), (nrows + 1) * sizeof(uint64_t));
        if (nvals) std::memcpy(out->colidx, Ai.data(), nvals * sizeof(uint64_t));
        if (weighted && nvals) std::memcpy(out->vals, X.data(), nvals * sizeof(double));
        // SuiteSparse may leave rows jumbled; sort every row (values follow).
        #pragma omp parallel for schedule(dynamic, 1024)
        for (int64_t i = 0; i < (int64_t)nrows; i++) {
            uint64_t b = out->rowptr[i], e = out->rowptr[i + 1];
            if (std::is_sorted(out->colidx + b, out->colidx + e)) continue;
            std::vector<std::pair<uint64_t, double>> row;
            for (uint64_t k = b; k < e; k++) row.push_back({out->colidx[k], weighted ? out->vals[k] : 0.0});
            std::sort(row.begin(), row.end());
            for (uint64_t k = b; k < e; k++) {
                out->colidx[k] = row[k - b].first;
                if (weighted) out->vals[k] = row[k - b].second;
            }
        }
    } else {
        csc_to_csr(nrows, ncols, P.data(), Ai.data(), weighted ? X.data() : nullptr,
                   out->rowptr, out->colidx, out->vals);
    }
    return GX_SUCCESS;
}

extern "C" int gx_write_grb(const char *path, const gx_csr *csr) {
    if (!path || !csr || !csr->rowptr || (!csr->colidx && csr->nnz))
        return fail(GX_NULL_POINTER, "gx_write_grb: null argument");
    FilePtr f(std::fopen(path, "wb"));
    if (!f) return fail(GX_IO_ERROR, std::string("cannot create ") + path);
    const bool weighted = csr->vals != nullptr;
    const uint64_t n = csr->n, nnz = csr->nnz;
    int32_t fmt = 0;                              // GxB_BY_ROW
    int32_t kind = weighted ? 2 : 102;            // sparse (+100 iso)
    double hyper = 0.0625;                        // GxB_HYPER_DEFAULT
    int64_t nonempty = -1;
    uint64_t nvec = n;
    int32_t typecode = weighted ? 10 : 0;         // GrB_FP64 / GrB_BOOL
    uint64_t typesize = weighted ? 8 : 1;
    char header[512];
    int len = std::snprintf(header, sizeof(header),
                            "SuiteSparse:GraphBLAS matrix\nv%-25s\n"
                            "nrows:  %-18" PRIu64 "\nncols:  %-18" PRIu64 "\n"
                            "nvec:   %-18" PRIu64 "\nnvals:  %-18" PRIu64 "\n"
                            "format: %-8s\nsize:   %-18" PRIu64 "\ntype:   %-72s\n"
                            "iso:    %1d\n%-210s\n\n",
                            "7.4.4 (gx)", n, n, nvec, nnz, "CSR ", typesize,
                            weighted ? "GrB_FP64  " : "GrB_BOOL  ", weighted ? 0 : 1, "\n");
    if (len < 0) len = 0;
    for (int k = len; k < 512; k++) header[k] = ' ';
    header[511] = '\0';
    FILE *fp = f.get();
    bool ok = std::fwrite(header, 1, 512, fp) == 512;
    ok = ok && std::fwrite(&fmt, 4, 1, fp) == 1 && std::fwrite(&kind, 4, 1, fp) == 1;
    ok = ok && std::fwrite(&hyper, 8, 1, fp) == 1 && std::fwrite(&n, 8, 1, fp) == 1;
    ok = ok && std::fwrite(&n, 8, 1, fp) == 1 && std::fwrite(&nonempty, 8, 1, fp) == 1;
    ok = ok && std::fwrite(&nvec, 8, 1, fp) == 1 && std::fwrite(&nnz, 8, 1, fp) == 1;
    ok = ok && std::fwrite(&typecode, 4, 1, fp) == 1 && std::fwrite(&typesize, 8, 1, fp) == 1;
    ok = ok && std::fwrite(csr->rowptr, 8, n + 1, fp) == n + 1;
    ok = ok && (nnz == 0 || std::fwrite(csr->colidx, 8, nnz, fp) == nnz);
    if (weighted) {
        ok = ok && (nnz == 0 || std::fwrite(csr->vals, 8, nnz, fp) == nnz);
    } else {
        const bool one = true;
        ok = ok && std::fwrite(&one, 1, 1, fp) == 1;
    }
    if (!ok) return fail(GX_IO_ERROR, std::string("write failed: ") + path);
    return GX_SUCCESS;
}

extern "C" int gx_read_vtb(const char *path, uint64_t **ids, uint64_t *count) {
    if (!path || !ids || !count) return fail(GX_NULL_POINTER, "gx_read_vtb: null argument");
    FilePtr f(std::fopen(path, "rb"));
    if (!f) return fail(GX_IO_ERROR, std::string("cannot open ") + path);
    std::fseek(f.get(), 0, SEEK_END);
    long bytes = std::ftell(f.get());
    std::fseek(f.get(), 0, SEEK_SET);
    if (bytes < 0 || bytes % 8) return fail(GX_IO_ERROR, "bad .vtb size");
    uint64_t n = (uint64_t)bytes / 8;
    uint64_t *p = xmalloc<uint64_t>(n);
    if (!p) return fail(GX_OUT_OF_MEMORY, "gx_read_vtb: out of memory");
    if (!read_n(f.get(), p, n)) {
        std::free(p);
        return fail(GX_IO_ERROR, "truncated .vtb");
    }
    *ids = p;
    *count = n;
    return GX_SUCCESS;
}

extern "C" int gx_write_vtb(const char *path, const uint64_t *ids, uint64_t count) {
    if (!path || (!ids && count)) return fail(GX_NULL_POINTER, "gx_write_vtb: null argument");
    FilePtr f(std::fopen(path, "wb"));
    if (!f) return fail(GX_IO_ERROR, std::string("cannot create ") + path);
    if (count && std::fwrite(ids, 8, count, f.get()) != count)
        return fail(GX_IO_ERROR, "write failed");
    return GX_SUCCESS;
}

// ------------------------------------------------------------------------------------
// Seeded R-MAT (SURVEY.md 8d synthetic inputs).  Every random draw is a pure function
// of (seed, edge index, level), so the graph does not depend on the thread count.
// ------------------------------------------------------------------------------------
namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

// U(0,1] weight of the unordered pair {u, v}: symmetric by construction.
inline double pair_weight(uint64_t seed, uint32_t u, uint32_t v) {
    uint32_t lo = std::min(u, v), hi = std::max(u, v);
    uint64_t h = splitmix64(seed ^ 0x5851F42D4C957F2Dull ^ (((uint64_t)lo << 32) | hi));
    return 1.0 - u01(h);   // in (0, 1]
}

}  // namespace

extern "C" int gx_rmat_csr(int scale, int edgefactor, double a, double b, double c,
                           uint64_t seed, int undirected, int weighted, gx_csr *out) {
    if (!out) return fail(GX_NULL_POINTER, "gx_rmat_csr: null out");
    std::memset(out, 0, sizeof(*out));
    if (scale < 1 || scale > 30 || edgefactor < 1)
        return fail(GX_INVALID_VALUE, "gx_rmat_csr: bad scale/edgefactor");
    if (a < 0 || b < 0 || c < 0 || a + b + c > 1.0)
        return fail(GX_INVALID_VALUE, "gx_rmat_csr: bad probabilities");
    const uint64_t n = 1ull << scale;
    const uint64_t m = (uint64_t)edgefactor << scale;

    // seeded vertex permutation (Fisher-Yates)
    std::vector<uint32_t> perm(n);
    std::iota(perm.begin(), perm.end(), 0u);
    for (uint64_t i = n - 1; i > 0; i--) {
        uint64_t j = splitmix64(seed ^ 0xA24BAED4963EE407ull ^ i) % (i + 1);
        std::swap(perm[i], perm[j]);
    }

    // edge generation
    const uint64_t mult = undirected ? 2 : 1;
    std::vector<uint32_t> src(m * mult), dst(m * mult);
    const double ab = a + b, abc = a + b + c;
    #pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < (int64_t)m; e++) {
        uint64_t u = 0, v = 0;
        uint64_t state = splitmix64(seed * 0x100000001B3ull + (uint64_t)e);
        for (int l = 0; l < scale; l++) {
            state = splitmix64(state);
            double r = u01(state);
            u <<= 1;
            v <<= 1;
            if (r < a) {
            } else if (r < ab) {
                v |= 1;
            } else if (r < abc) {
                u |= 1;
            } else {
                u |= 1;
                v |= 1;
            }
        }
        uint32_t pu = perm[u], pv = perm[v];
        src[e] = pu;
        dst[e] = pv;
        if (undirected) {
            src[m + e] = pv;
            dst[m + e] = pu;
        }
    }
    const uint64_t me = m * mult;

    // counting sort by source (self-loops dropped)
    std::vector<uint64_t> rp(n + 1, 0);
    for (uint64_t e = 0; e < me; e++)
        if (src[e] != dst[e]) rp[src[e] + 1]++;
    for (uint64_t i = 0; i < n; i++) rp[i + 1] += rp[i];
    std::vector<uint32_t> col(rp[n]);
    {
        std::vector<uint64_t> cur(rp.begin(), rp.end() - 1);
        for (uint64_t e = 0; e < me; e++)
            if (src[e] != dst[e]) col[cur[src[e]]++] = dst[e];
    }
    std::vector<uint32_t>().swap(src);
    std::vector<uint32_t>().swap(dst);

    // sort + dedup each row
    std::vector<uint64_t> deg(n);
    #pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        uint32_t *bgn = col.data() + rp[i], *end = col.data() + rp[i + 1];
        std::sort(bgn, end);
        deg[i] = (uint64_t)(std::unique(bgn, end) - bgn);
    }
    uint64_t *orp = xmalloc<uint64_t>(n + 1);
    if (!orp) return fail(GX_OUT_OF_MEMORY, "gx_rmat_csr: out of memory");
    orp[0] = 0;
    for (uint64_t i = 0; i < n; i++) orp[i + 1] = orp[i] + deg[i];
    const uint64_t nnz = orp[n];
    uint64_t *oci = xmalloc<uint64_t>(nnz);
    double *ow = weighted ? xmalloc<double>(nnz) : nullptr;
    if (!oci || (weighted && !ow)) {
        std::free(orp);
        std::free(oci);
        std::free(ow);
        return fail(GX_OUT_OF_MEMORY, "gx_rmat_csr: out of memory");
    }
    #pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        const uint32_t *row = col.data() + rp[i];
        for (uint64_t k = 0; k < deg[i]; k++) {
            oci[orp[i] + k] = row[k];
            if (weighted) ow[orp[i] + k] = pair_weight(seed, (uint32_t)i, row[k]);
        }
    }
    out->n = n;
    out->nnz = nnz;
    out->rowptr = orp;
    out->colidx = oci;
    out->vals = ow;
    return GX_SUCCESS;
}

// ------------------------------------------------------------------------------------
// Text formats written by relabel.py (Matrix Market + one-id-per-line mapping).
// ------------------------------------------------------------------------------------
extern "C" int gx_read_vtx(const char *path, uint64_t **ids, uint64_t *count) {
    if (!path || !ids || !count) return fail(GX_NULL_POINTER, "gx_read_vtx: null argument");
    FilePtr f(std::fopen(path, "r"));
    if (!f) return fail(GX_IO_ERROR, std::string("cannot open ") + path);
    std::vector<uint64_t> v;
    unsigned long long x;
    while (std::fscanf(f.get(), "%llu", &x) == 1) v.push_back(x);
    uint64_t *p = xmalloc<uint64_t>(v.size());
    if (!p) return fail(GX_OUT_OF_MEMORY, "gx_read_vtx: out of memory");
    std::memcpy(p, v.data(), v.size() * 8);
    *ids = p;
    *count = v.size();
    return GX_SUCCESS;
}

extern "C" int gx_read_mtx(const char *path, gx_csr *out) {
    if (!path || !out) return fail(GX_NULL_POINTER, "gx_read_mtx: null argument");
    std::memset(out, 0, sizeof(*out));
    FilePtr f(std::fopen(path, "r"));
    if (!f) return fail(GX_IO_ERROR, std::string("cannot open Matrix Market file: ") + path);
    char line[1024];
    if (!std::fgets(line, sizeof line, f.get())) return fail(GX_IO_ERROR, "empty .mtx");
    char banner[64] = {0}, object[64] = {0}, format[64] = {0}, field[64] = {0}, symmetry[64] = {0};
    if (std::sscanf(line, "%63s %63s %63s %63s %63s", banner, object, format, field, symmetry) != 5 ||
        std::strcmp(banner, "%%MatrixMarket") != 0)
        return fail(GX_IO_ERROR, "bad Matrix Market banner");
    auto lower = [](char *s) {
        for (; *s; s++) *s = (char)std::tolower((unsigned char)*s);
    };
    lower(object);
    lower(format);
    lower(field);
    lower(symmetry);
    if (std::strcmp(object, "matrix") != 0 || std::strcmp(format, "coordinate") != 0)
        return fail(GX_NOT_IMPLEMENTED, "only coordinate matrices are supported");
    const bool symmetric = std::strcmp(symmetry, "symmetric") == 0;
    if (!symmetric && std::strcmp(symmetry, "general") != 0)
        return fail(GX_NOT_IMPLEMENTED, "only general/symmetric Matrix Market files are supported");
    const bool pattern = std::strcmp(field, "pattern") == 0;
    bool weighted = std::strcmp(field, "real") == 0 || std::strcmp(field, "double") == 0;
    // %%GraphBLAS <type> (relabel.py:68) overrides the Matrix Market field
    uint64_t nr = 0, nc = 0, ne = 0;
    for (;;) {
        if (!std::fgets(line, sizeof line, f.get())) return fail(GX_IO_ERROR, "missing size line");
        if (line[0] == '%') {
            char tag[64] = {0}, type[64] = {0};
            if (std::sscanf(line, "%63s %63s", tag, type) == 2 && std::strcmp(tag, "%%GraphBLAS") == 0)
                weighted = std::strcmp(type, "GrB_FP64") == 0 || std::strcmp(type, "GrB_FP32") == 0;
            continue;
        }
        unsigned long long a, b, c;
        if (std::sscanf(line, "%llu %llu %llu", &a, &b, &c) != 3) return fail(GX_IO_ERROR, "bad size line");
        nr = a;
        nc = b;
        ne = c;
        break;
    }
    if (nr != nc) return fail(GX_INVALID_VALUE, "adjacency matrix must be square");
    struct Ent {
        uint64_t r, c;
        double v;
    };
    std::vector<Ent> ents;
    ents.reserve(symmetric ? 2 * ne : ne);
    for (uint64_t k = 0; k < ne; k++) {
        unsigned long long i, j;
        double v = 1.0;
        int got = pattern ? std::fscanf(f.get(), "%llu %llu", &i, &j)
                          : std::fscanf(f.get(), "%llu %llu %lf", &i, &j, &v);
        if (got != (pattern ? 2 : 3)) return fail(GX_IO_ERROR, "truncated Matrix Market entries");
        if (i < 1 || j < 1 || i > nr || j > nc) return fail(GX_INVALID_INDEX, "entry out of range");
        ents.push_back({i - 1, j - 1, v});
        if (symmetric && i != j) ents.push_back({j - 1, i - 1, v});
    }
    std::stable_sort(ents.begin(), ents.end(),
                     [](const Ent &x, const Ent &y) { return x.r != y.r ? x.r < y.r : x.c < y.c; });
    // duplicates: keep the last occurrence
    std::vector<Ent> uniq;
    uniq.reserve(ents.size());
    for (size_t k = 0; k < ents.size(); k++) {
        if (!uniq.empty() && uniq.back().r == ents[k].r && uniq.back().c == ents[k].c) uniq.back() = ents[k];
        else uniq.push_back(ents[k]);
    }
    const uint64_t nnz = uniq.size();
    out->n = nr;
    out->nnz = nnz;
    out->rowptr = xmalloc<uint64_t>(nr + 1);
    out->colidx = xmalloc<uint64_t>(nnz);
    out->vals = weighted ? xmalloc<double>(nnz) : nullptr;
    if (!out->rowptr || !out->colidx || (weighted && !out->vals)) {
        gx_csr_release(out);
        return fail(GX_OUT_OF_MEMORY, "gx_read_mtx: out of memory");
    }
    std::fill(out->rowptr, out->rowptr + nr + 1, 0);
    for (uint64_t k = 0; k < nnz; k++) {
        out->rowptr[uniq[k].r + 1]++;
        out->colidx[k] = uniq[k].c;
        if (weighted) out->vals[k] = uniq[k].v;
    }
    for (uint64_t i = 0; i < nr; i++) out->rowptr[i + 1] += out->rowptr[i];
    return GX_SUCCESS;
}

// ---------------------------------------------------------------- host helpers (OpenMP)

namespace gx {

bool host_narrow(const uint64_t *in, uint64_t count, uint64_t limit, int32_t *out, bool nt) {
    int bad = 0;
    if (!nt || (reinterpret_cast<uintptr_t>(out) & 15)) {
#pragma omp parallel for schedule(static) reduction(| : bad)
        for (int64_t k = 0; k < (int64_t)count; k++) {
            const uint64_t c = in[k];
            bad |= c >= limit;
            out[k] = (int32_t)c;
        }
        return bad == 0;
    }
    // streaming stores: the staging buffer is read next by the DMA engine, not by this core,
    // so its lines are not fetched for ownership first
    const int64_t nq = (int64_t)(count / 4);
#pragma omp parallel reduction(| : bad)
    {
#pragma omp for schedule(static)
        for (int64_t q = 0; q < nq; q++) {
            const uint64_t *p = in + 4 * q;
            const uint64_t c0 = p[0], c1 = p[1], c2 = p[2], c3 = p[3];
            bad |= (c0 >= limit) | (c1 >= limit) | (c2 >= limit) | (c3 >= limit);
            _mm_stream_si128(reinterpret_cast<__m128i *>(out + 4 * q),
                             _mm_set_epi32((int32_t)c3, (int32_t)c2, (int32_t)c1, (int32_t)c0));
        }
        _mm_sfence();
    }
    for (uint64_t k = (uint64_t)nq * 4; k < count; k++) {
        bad |= in[k] >= limit;
        out[k] = (int32_t)in[k];
    }
    return bad == 0;
}

// Columns < limit <= 2^24 as packed 24-bit little-endian values: entry k in bytes [3k, 3k+3)
// of out, 16 entries = 12 words = three streaming 16-B stores (the upload's host->device bytes
// fall by a quarter; k_unpack24 widens them on the device).  out holds ceil(3 count / 4) words.
// SSE4.1 / SSSE3 body (EPYC hosts; checked at run time): per 4 entries the low dwords by two
// shuffles, the unsigned max for the range check, a byte shuffle to 12 bytes, and four 12-byte
// groups merged into three 16-byte streaming stores.
__attribute__((target("sse4.1,ssse3"))) static bool pack24_simd(const uint64_t *in, int64_t ng, uint64_t limit,
                                                                uint32_t *out) {
    const __m128i sq = _mm_setr_epi8(0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -1, -1, -1, -1);
    int bad = 0;
#pragma omp parallel reduction(| : bad)
    {
        __m128i mx = _mm_setzero_si128(), hi = _mm_setzero_si128();
#pragma omp for schedule(static)
        for (int64_t q = 0; q < ng; q++) {
            const __m128i *p = reinterpret_cast<const __m128i *>(in + 16 * q);
            __m128i g[4];
            for (int k = 0; k < 4; k++) {
                const __m128i a = _mm_loadu_si128(p + 2 * k), b = _mm_loadu_si128(p + 2 * k + 1);
                // dwords: a0lo a0hi a1lo a1hi | b0lo b0hi b1lo b1hi
                const __m128i lo = _mm_unpacklo_epi64(_mm_shuffle_epi32(a, 0x08), _mm_shuffle_epi32(b, 0x08));
                const __m128i h = _mm_unpacklo_epi64(_mm_shuffle_epi32(a, 0x0d), _mm_shuffle_epi32(b, 0x0d));
                mx = _mm_max_epu32(mx, lo);
                hi = _mm_or_si128(hi, h);
                g[k] = _mm_shuffle_epi8(lo, sq);
            }
            __m128i *o = reinterpret_cast<__m128i *>(out + 12 * q);
            _mm_stream_si128(o, _mm_or_si128(g[0], _mm_slli_si128(g[1], 12)));
            _mm_stream_si128(o + 1, _mm_or_si128(_mm_srli_si128(g[1], 4), _mm_slli_si128(g[2], 8)));
            _mm_stream_si128(o + 2, _mm_or_si128(_mm_srli_si128(g[2], 8), _mm_slli_si128(g[3], 4)));
        }
        _mm_sfence();
        alignas(16) uint32_t m[4], h[4];
        _mm_store_si128(reinterpret_cast<__m128i *>(m), mx);
        _mm_store_si128(reinterpret_cast<__m128i *>(h), hi);
        for (int k = 0; k < 4; k++) bad |= (h[k] != 0) | ((uint64_t)m[k] >= limit);
    }
    return bad == 0;
}

bool host_pack24(const uint64_t *in, uint64_t count, uint64_t limit, uint32_t *out) {
    int bad = 0;
    const int64_t ng = (int64_t)(count / 16);
    const bool aligned = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    static const bool simd = __builtin_cpu_supports("sse4.1") && __builtin_cpu_supports("ssse3");
    if (aligned && simd && ng > 0) {
        bad |= !pack24_simd(in, ng, limit, out);
        unsigned char *b = reinterpret_cast<unsigned char *>(out);
        for (uint64_t k = (uint64_t)ng * 16; k < count; k++) {
            bad |= in[k] >= limit;
            const uint32_t c = (uint32_t)in[k];
            b[3 * k] = (unsigned char)c;
            b[3 * k + 1] = (unsigned char)(c >> 8);
            b[3 * k + 2] = (unsigned char)(c >> 16);
        }
        return bad == 0;
    }
#pragma omp parallel reduction(| : bad)
    {
#pragma omp for schedule(static)
        for (int64_t q = 0; q < ng; q++) {
            const uint64_t *p = in + 16 * q;
            uint32_t c[16];
            uint64_t any = 0;
            for (int j = 0; j < 16; j++) {
                any |= p[j] >= limit;
                c[j] = (uint32_t)p[j];
            }
            bad |= (int)any;
            uint32_t w[12];
            for (int g = 0; g < 4; g++) {
                const uint32_t c0 = c[4 * g], c1 = c[4 * g + 1], c2 = c[4 * g + 2], c3 = c[4 * g + 3];
                w[3 * g] = (c0 & 0xffffffu) | (c1 << 24);
                w[3 * g + 1] = ((c1 >> 8) & 0xffffu) | (c2 << 16);
                w[3 * g + 2] = ((c2 >> 16) & 0xffu) | (c3 << 8);
            }
            uint32_t *o = out + 12 * q;
            if (aligned) {
                _mm_stream_si128(reinterpret_cast<__m128i *>(o), _mm_loadu_si128(reinterpret_cast<const __m128i *>(w)));
                _mm_stream_si128(reinterpret_cast<__m128i *>(o + 4), _mm_loadu_si128(reinterpret_cast<const __m128i *>(w + 4)));
                _mm_stream_si128(reinterpret_cast<__m128i *>(o + 8), _mm_loadu_si128(reinterpret_cast<const __m128i *>(w + 8)));
            } else {
                std::memcpy(o, w, sizeof w);
            }
        }
        _mm_sfence();
    }
    unsigned char *b = reinterpret_cast<unsigned char *>(out);
    for (uint64_t k = (uint64_t)ng * 16; k < count; k++) {
        bad |= in[k] >= limit;
        const uint32_t c = (uint32_t)in[k];
        b[3 * k] = (unsigned char)c;
        b[3 * k + 1] = (unsigned char)(c >> 8);
        b[3 * k + 2] = (unsigned char)(c >> 16);
    }
    return bad == 0;
}

void host_copy(void *dst, const void *src, size_t bytes) {
    constexpr size_t kBlock = 1 << 20;
    const int64_t nb = (int64_t)((bytes + kBlock - 1) / kBlock);
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; b++) {
        const size_t off = (size_t)b * kBlock;
        std::memcpy(static_cast<char *>(dst) + off, static_cast<const char *>(src) + off,
                    std::min(kBlock, bytes - off));
    }
}

void host_prefault(void *p, size_t bytes) {
    constexpr size_t kPage = 4096;
    char *c = static_cast<char *>(p);
    const int64_t np = (int64_t)((bytes + kPage - 1) / kPage);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < np; i++) *reinterpret_cast<volatile char *>(c + i * kPage) = 0;
}

int host_threads() { return omp_get_max_threads(); }

void host_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

bool host_monotone(const uint64_t *rp, uint64_t n) {
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int64_t i = 0; i < (int64_t)n; i++) bad |= rp[i + 1] < rp[i];
    return bad == 0;
}

void host_levels(const int32_t *in, uint64_t n, int64_t *out) {
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < (int64_t)n; v++) out[v] = in[v] < 0 ? INT64_MAX : (int64_t)in[v];
}

void host_widen(const int32_t *in, uint64_t n, uint64_t *out) {
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < (int64_t)n; v++) out[v] = (uint64_t)(uint32_t)in[v];
}

int host_chunk_columns(const uint64_t *ci, uint64_t nnz, const uint64_t *ranges, int nranks, const uint64_t *live,
                       uint64_t chunk, uint64_t n, int32_t *out) {
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int64_t k = 0; k < (int64_t)nnz; k++) {
        const uint64_t c = ci[k];
        if (c >= n) {
            bad |= 1;
            continue;
        }
        int owner = 0;   // nranks is small: the last range starting at or before c
        while (owner + 1 < nranks && ranges[owner + 1] <= c) owner++;
        const uint64_t local = c - ranges[owner];
        if (local >= live[owner]) bad |= 2;
        out[k] = (int32_t)((uint64_t)owner * chunk + local);
    }
    return bad;
}

void host_hub_order(const uint64_t *rp, uint64_t n, uint32_t *order) {
    uint64_t maxd = 0;
#pragma omp parallel for schedule(static) reduction(max : maxd)
    for (int64_t v = 0; v < (int64_t)n; v++) maxd = std::max<uint64_t>(maxd, rp[v + 1] - rp[v]);
    // stable counting sort by descending degree
    std::vector<uint64_t> start(maxd + 2, 0);
    for (uint64_t v = 0; v < n; v++) start[maxd - (rp[v + 1] - rp[v]) + 1]++;
    for (size_t k = 1; k < start.size(); k++) start[k] += start[k - 1];
    for (uint64_t v = 0; v < n; v++) order[start[maxd - (rp[v + 1] - rp[v])]++] = (uint32_t)v;
}

void host_pick_rows(const uint64_t *rp, const uint64_t *ci, const uint32_t *rows, uint64_t nrows, const int32_t *colmap,
                    int64_t *out_rp, int32_t *out_ci) {
    out_rp[0] = 0;
    for (uint64_t j = 0; j < nrows; j++) out_rp[j + 1] = out_rp[j] + (int64_t)(rp[rows[j] + 1] - rp[rows[j]]);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t j = 0; j < (int64_t)nrows; j++) {
        const uint64_t b = rp[rows[j]], e = rp[rows[j] + 1];
        int32_t *o = out_ci + out_rp[j];
        for (uint64_t k = b; k < e; k++) o[k - b] = colmap[ci[k]];
    }
}

void host_hub_order_par(const uint64_t *rp, uint64_t n, int32_t *order, int32_t *perm, int64_t *hdeg) {
    // stable counting sort by descending degree, in parallel: degrees below kD by a histogram per
    // thread (threads own contiguous vertex ranges, so equal degrees keep id order), the few
    // hubs at or above it sorted on their own and put first
    constexpr uint64_t kD = 1u << 16;
    const int T = std::max(1, omp_get_max_threads());
    std::vector<uint64_t> cnt((size_t)T * kD, 0);
    std::vector<std::vector<uint32_t>> big(T);
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        const uint64_t v0 = n * t / nt, v1 = n * (t + 1) / nt;
        uint64_t *c = cnt.data() + (size_t)t * kD;
        for (uint64_t v = v0; v < v1; v++) {
            const uint64_t d = rp[v + 1] - rp[v];
            if (d >= kD) big[t].push_back((uint32_t)v);
            else c[kD - 1 - d]++;   // bucket 0 = degree kD - 1 (descending order)
        }
    }
    std::vector<uint32_t> hubs;
    for (auto &b : big) hubs.insert(hubs.end(), b.begin(), b.end());
    std::stable_sort(hubs.begin(), hubs.end(),
                     [&](uint32_t a, uint32_t b) { return rp[a + 1] - rp[a] > rp[b + 1] - rp[b]; });
    // exclusive offsets, bucket-major then thread
    std::vector<uint64_t> off((size_t)T * kD);
    uint64_t acc = hubs.size();
    for (uint64_t b = 0; b < kD; b++)
        for (int t = 0; t < T; t++) {
            off[(size_t)t * kD + b] = acc;
            acc += cnt[(size_t)t * kD + b];
        }
    for (size_t h = 0; h < hubs.size(); h++) {
        order[h] = (int32_t)hubs[h];
        perm[hubs[h]] = (int32_t)h;
        hdeg[h] = (int64_t)(rp[hubs[h] + 1] - rp[hubs[h]]);
    }
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        const uint64_t v0 = n * t / nt, v1 = n * (t + 1) / nt;
        uint64_t *o = off.data() + (size_t)t * kD;
        for (uint64_t v = v0; v < v1; v++) {
            const uint64_t d = rp[v + 1] - rp[v];
            if (d >= kD) continue;
            const uint64_t pos = o[kD - 1 - d]++;
            order[pos] = (int32_t)v;
            perm[v] = (int32_t)pos;
            hdeg[pos] = (int64_t)d;
        }
    }
}

void host_compose(const int32_t *a, const int32_t *idx, uint64_t n, int32_t *out) {
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < (int64_t)n; v++) out[v] = a[idx[v]];
}

uint64_t host_count_live(const uint64_t *rp, uint64_t n) {
    uint64_t c = 0;
#pragma omp parallel for schedule(static) reduction(+ : c)
    for (int64_t v = 0; v < (int64_t)n; v++) c += rp[v + 1] != rp[v];
    return c;
}

bool host_pick_span(const uint64_t *rp, const uint64_t *ci, const int32_t *rows, const int64_t *lrp, uint64_t nrows,
                    uint64_t e0, uint64_t e1, uint64_t limit, int32_t *out) {
    if (e1 <= e0) return true;
    // the local rows overlapping [e0, e1): j0 = last row starting at or before e0
    const int64_t j0 = (int64_t)(std::upper_bound(lrp, lrp + nrows + 1, (int64_t)e0) - lrp) - 1;
    const int64_t j1 = (int64_t)(std::lower_bound(lrp, lrp + nrows + 1, (int64_t)e1) - lrp);
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(| : bad)
    for (int64_t j = std::max<int64_t>(j0, 0); j < std::min<int64_t>(j1, (int64_t)nrows); j++) {
        const int64_t lb = std::max<int64_t>(lrp[j], (int64_t)e0), le = std::min<int64_t>(lrp[j + 1], (int64_t)e1);
        if (lb >= le) continue;
        const uint64_t *src = ci + rp[rows[j]] + (uint64_t)(lb - lrp[j]);
        int32_t *o = out + (lb - (int64_t)e0);
        for (int64_t k = 0; k < le - lb; k++) {
            const uint64_t c = src[k];
            bad |= c >= limit;
            o[k] = (int32_t)(c < limit ? c : 0);
        }
    }
    return !bad;
}

void host_transpose(uint64_t n, const uint64_t *rp, const uint64_t *ci, uint64_t *trp, uint64_t *tci) {
    const uint64_t nnz = rp[n];
    std::fill(trp, trp + n + 1, 0);
    for (uint64_t k = 0; k < nnz; k++) trp[ci[k] + 1]++;
    for (uint64_t i = 0; i < n; i++) trp[i + 1] += trp[i];
    std::vector<uint64_t> cur(trp, trp + n);
    for (uint64_t i = 0; i < n; i++)
        for (uint64_t k = rp[i]; k < rp[i + 1]; k++) tci[cur[ci[k]]++] = i;
}

}  // namespace gx

// Host-only: the interleaved hub-first partition of gx_pagerank_multi (include/gx.h).
extern "C" int gx_pr_partition(uint64_t n, const uint64_t *rowptr, int nparts, uint32_t *order, uint64_t *rows,
                               uint64_t *live) {
    if (!rowptr || !order || !rows || !live) return fail(GX_NULL_POINTER, "gx_pr_partition: null argument");
    if (nparts < 1) return fail(GX_INVALID_VALUE, "gx_pr_partition: nparts < 1");
    if (n >= (1ull << 32)) return fail(GX_NOT_IMPLEMENTED, "gx_pr_partition: n >= 2^32");
    gx::host_hub_order(rowptr, n, order);
    for (int k = 0; k < nparts; k++) {
        rows[k] = n > (uint64_t)k ? (n - k + nparts - 1) / nparts : 0;
        live[k] = 0;
    }
    // hub-first: degrees descend, so each part's rows with out-edges come first
    for (uint64_t i = 0; i < n; i++)
        if (rowptr[order[i] + 1] > rowptr[order[i]]) live[i % nparts]++;
    return GX_SUCCESS;
}
