// common.cpp -- shared driver of the Graphalytics executables (see common.h).
#include "common.h"

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>

#include <omp.h>

namespace gxexe {

BenchmarkParameters ParseBenchmarkParameters(int argc, char **argv) {
    BenchmarkParameters p;
    for (int i = 0; i + 1 < argc; i++) {
        const char *key = argv[i];
        const char *value = argv[i + 1];
        if (std::strcmp(key, "--binary") == 0) p.binary = std::strcmp(value, "true") == 0;
        else if (std::strcmp(key, "--input-dir") == 0) p.input_dir = value;
        else if (std::strcmp(key, "--directed") == 0) p.directed = std::strcmp(value, "true") == 0;
        else if (std::strcmp(key, "--source-vertex") == 0) p.source_vertex = std::stoul(value);
        else if (std::strcmp(key, "--damping-factor") == 0) p.damping_factor = std::stod(value);
        else if (std::strcmp(key, "--max-iteration") == 0) p.max_iteration = std::stoi(value);
        else if (std::strcmp(key, "--output-file") == 0) p.output_file = value;
        else if (std::strcmp(key, "--threadnum") == 0) p.thread_num = std::stoul(value);
    }
    return p;
}

long long GetCurrentMilliseconds() {
    using namespace std::chrono;
    return duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count();
}

void OK(int info, const char *what) {
    if (info != GX_SUCCESS)
        throw std::runtime_error(std::string("GraphBLAS error [") + std::to_string(info) + "]  " + what +
                                 ": " + gx_last_error());
}

namespace {

struct CsrHolder {
    gx_csr csr{};
    ~CsrHolder() { gx_csr_release(&csr); }
};

struct IdsHolder {
    uint64_t *ids = nullptr;
    uint64_t n = 0;
    ~IdsHolder() { gx_host_free(ids); }
};

struct CtxHolder {
    gx_ctx *ctx = nullptr;
    gx_graph *g = nullptr;
    std::vector<gx_ctx *> more;   // GX_NGPUS > 1: the contexts of the other devices
    ~CtxHolder() {
        gx_graph_free(g);
        gx_free(ctx);
        for (gx_ctx *c : more) gx_free(c);
    }
};

// ReadMatrixMarket (graphio.cpp:4-32) without SuiteSparse
void ReadMatrix(const BenchmarkParameters &p, gx_csr *out) {
    if (p.binary) OK(gx_read_grb((p.input_dir + "/graph.grb").c_str(), out), "reading graph.grb");
    else OK(gx_read_mtx((p.input_dir + "/graph.mtx").c_str(), out), "reading graph.mtx");
}

// ReadMapping (graphio.cpp:34-60)
void ReadMapping(const BenchmarkParameters &p, IdsHolder *m) {
    if (p.binary) OK(gx_read_vtb((p.input_dir + "/graph.vtb").c_str(), &m->ids, &m->n), "reading graph.vtb");
    else OK(gx_read_vtx((p.input_dir + "/graph.vtx").c_str(), &m->ids, &m->n), "reading graph.vtx");
}

struct OutFile {
    FILE *f = nullptr;
    std::vector<char> buf;
    explicit OutFile(const std::string &path) : buf(1 << 22) {
        f = std::fopen(path.c_str(), "w");
        if (!f) {
            std::cerr << "Output file " << path << " does not exists" << std::endl;
            std::exit(-1);
        }
        std::setvbuf(f, buf.data(), _IOFBF, buf.size());
    }
    ~OutFile() {
        if (f) std::fclose(f);
    }
};

// "%.16e" == ostream precision(16) + std::scientific (pr.cpp:26-27)
void PutDouble(FILE *f, uint64_t id, double x) { std::fprintf(f, "%" PRIu64 " %.16e\n", id, x); }

// the names the reference's wrappers give their ComputationTimer (bfs.cpp:71, pr.cpp:48,
// sssp.cpp:64, wcc.cpp:40, cdlp.cpp:59, lcc.cpp:65)
const char *TimerName(Algorithm alg) {
    switch (alg) {
        case Algorithm::BFS: return "BFS";
        case Algorithm::PR: return "PageRank";
        case Algorithm::SSSP: return "SSSP";
        case Algorithm::WCC: return "WeaklyConnectedComponents";
        case Algorithm::CDLP: return "CDLP";
        case Algorithm::LCC: return "LCC";
    }
    return "?";
}

}  // namespace

int Main(int argc, char **argv, Algorithm alg) {
    try {
        BenchmarkParameters p = ParseBenchmarkParameters(argc, argv);
        if (p.thread_num > 0) omp_set_num_threads((int)p.thread_num);
        int device = 0;
        if (const char *d = std::getenv("GX_DEVICE")) device = std::atoi(d);
        // GX_NGPUS = N: every algorithm on devices [GX_DEVICE, GX_DEVICE + N) in this one process
        // (gx_pagerank_multi / gx_sssp_multi / gx_lcc_multi: PageRank, SSSP (BASELINE config 4)
        // and LCC (config 5) on 1-D partitions; gx_bfs_multi / gx_wcc_multi / gx_cdlp_multi on a
        // replicated graph with vertex ranges and change-sized exchanges; in-process RCCL
        // collectives); execute-job.sh cannot pass new flags (execute-job.sh:68-151), so the
        // backend comes from the environment.  GX_MULTI_SIM=1 puts the N contexts
        // on device GX_DEVICE alone (virtual devices, collectives as device copies): the N > 1
        // path on a one-GPU box.
        int ngpus = 0;
        if (const char *g = std::getenv("GX_NGPUS")) ngpus = std::max(1, std::atoi(g));
        const char *sim_env = std::getenv("GX_MULTI_SIM");
        const bool sim = sim_env && std::atoi(sim_env) != 0;
        const bool multi_alg = true;

        CsrHolder A;
        ReadMatrix(p, &A.csr);
        IdsHolder mapping;
        ReadMapping(p, &mapping);
        const uint64_t n = mapping.n;
        if (A.csr.n != n) throw std::runtime_error("graph and mapping sizes differ");

        uint64_t src = 0;
        if (alg == Algorithm::BFS || alg == Algorithm::SSSP) {
            // linear search of the original id, as bfs.cpp:94-103 / sssp.cpp:93-102
            const uint64_t *it = std::find(mapping.ids, mapping.ids + n, (uint64_t)p.source_vertex);
            if (it == mapping.ids + n) {
                std::cout << "Source vertex not found in mapping" << std::endl;
                return -1;
            }
            src = (uint64_t)(it - mapping.ids);
        }

        CtxHolder H;
        OK(gx_init(device, &H.ctx), "gx_init");
        const bool multi = ngpus > 0 && multi_alg;
        if (multi)
            for (int k = 1; k < ngpus; k++) {
                gx_ctx *c = nullptr;
                OK(gx_init(sim ? device : device + k, &c), "gx_init (GX_NGPUS)");
                H.more.push_back(c);
            }
        std::vector<gx_ctx *> ctxs{H.ctx};
        ctxs.insert(ctxs.end(), H.more.begin(), H.more.end());
        // the clique (ncclCommInitAll, ~0.5 s) is set-up like gx_init: made before the markers
        if (multi) OK(gx_multi_prepare(ctxs.data(), ngpus), "gx_multi_prepare");
        // result arrays are not value-initialised: zero-filling SYN-8_5's 67 MB on one thread cost
        // ~10 ms inside the markers; libgx touches their pages in parallel while the device works
        std::unique_ptr<int64_t[]> level;
        std::unique_ptr<double[]> vals;
        std::unique_ptr<uint64_t[]> labels;

        const auto t_start = GetCurrentMilliseconds();
        std::cout << "Processing starts at: " << t_start << std::endl;
        std::cout << TimerName(alg) << " starts" << std::endl;   // ComputationTimer's constructor line
        const auto wall0 = std::chrono::high_resolution_clock::now();
        // PageRank on one GPU: upload, plan and iterations in one call, the upload overlapped with
        // the plan (gx_pagerank_csr); the other algorithms upload first
        const bool pr_fused = alg == Algorithm::PR && !multi;
        if (!multi && !pr_fused) OK(gx_graph_create(H.ctx, &A.csr, p.directed ? 1 : 0, &H.g), "gx_graph_create");
        const auto t_uploaded = GetCurrentMilliseconds();
        switch (alg) {
            case Algorithm::BFS:
                level.reset(new int64_t[n]);
                if (multi)
                    OK(gx_bfs_multi(ctxs.data(), ngpus, &A.csr, p.directed ? 1 : 0, src, level.get()), "gx_bfs_multi");
                else
                    OK(gx_bfs(H.g, src, level.get()), "gx_bfs");
                break;
            case Algorithm::PR:
                vals.reset(new double[n]);
                if (multi) {
                    OK(gx_pagerank_multi(ctxs.data(), ngpus, &A.csr, p.directed ? 1 : 0, p.damping_factor,
                                         p.max_iteration, vals.get()),
                       "gx_pagerank_multi");
                } else {
                    OK(gx_pagerank_csr(H.ctx, &A.csr, p.directed ? 1 : 0, p.damping_factor, p.max_iteration,
                                       vals.get(), &H.g),   // freed after the end marker
                       "gx_pagerank_csr");
                }
                break;
            case Algorithm::SSSP:
                vals.reset(new double[n]);
                if (multi) {
                    OK(gx_sssp_multi(ctxs.data(), ngpus, &A.csr, p.directed ? 1 : 0, src, vals.get()),
                       "gx_sssp_multi");
                } else {
                    OK(gx_sssp(H.g, src, vals.get()), "gx_sssp");
                }
                break;
            case Algorithm::WCC:
                labels.reset(new uint64_t[n]);
                if (multi)
                    OK(gx_wcc_multi(ctxs.data(), ngpus, &A.csr, p.directed ? 1 : 0, labels.get()), "gx_wcc_multi");
                else
                    OK(gx_wcc(H.g, labels.get()), "gx_wcc");
                break;
            case Algorithm::CDLP:
                labels.reset(new uint64_t[n]);
                if (multi)
                    OK(gx_cdlp_multi(ctxs.data(), ngpus, &A.csr, p.directed ? 1 : 0, p.max_iteration, labels.get()),
                       "gx_cdlp_multi");
                else
                    OK(gx_cdlp(H.g, p.max_iteration, labels.get()), "gx_cdlp");
                break;
            case Algorithm::LCC:
                vals.reset(new double[n]);
                if (multi)
                    OK(gx_lcc_multi(ctxs.data(), ngpus, &A.csr, p.directed ? 1 : 0, vals.get()), "gx_lcc_multi");
                else
                    OK(gx_lcc(H.g, vals.get()), "gx_lcc");
                break;
        }
        const auto t_end = GetCurrentMilliseconds();
        {
            // ComputationTimer's line (computation_timer.hpp:38-49; "PageRank" at pr.cpp:48,
            // "SSSP" at sssp.cpp:64, ...): the scope's seconds rounded to milliseconds
            using namespace std::chrono;
            const duration<double> d = round<milliseconds>(high_resolution_clock::now() - wall0);
            std::cout << TimerName(alg) << " duration: " << d.count() << "s" << std::endl;
        }
        std::cout << "Processing ends at: " << t_end << std::endl;
        double dev_ms = 0;
        gx_last_device_ms(H.ctx, &dev_ms);
        std::cout << "Upload time: " << (t_uploaded - t_start) << " ms" << std::endl;
        std::cout << "Algorithm time: " << (t_end - t_uploaded) << " ms" << std::endl;
        std::cout << "Device time: " << dev_ms << " ms" << std::endl;

        OutFile out(p.output_file);
        const uint64_t *ids = mapping.ids;
        switch (alg) {
            case Algorithm::BFS:   // SerializeBFSResult (bfs.cpp:11-68)
                for (uint64_t v = 0; v < n; v++) std::fprintf(out.f, "%" PRIu64 " %" PRId64 "\n", ids[v], level[v]);
                break;
            case Algorithm::PR:    // SerializePageRankResult (pr.cpp:17-45)
            case Algorithm::LCC:   // SerializeLCCResult (lcc.cpp:17-59)
                for (uint64_t v = 0; v < n; v++) PutDouble(out.f, ids[v], vals[v]);
                break;
            case Algorithm::SSSP:  // SerializeSSSPResult (sssp.cpp:11-51)
                for (uint64_t v = 0; v < n; v++) {
                    if (std::isinf(vals[v])) std::fprintf(out.f, "%" PRIu64 " infinity\n", ids[v]);
                    else PutDouble(out.f, ids[v], vals[v]);
                }
                break;
            case Algorithm::WCC:   // SerializeWCCResult (wcc.cpp:11-37), label -> original id
            case Algorithm::CDLP:  // SerializeCDLPResult (cdlp.cpp:21-52): mapping[label]
                for (uint64_t v = 0; v < n; v++)
                    std::fprintf(out.f, "%" PRIu64 " %" PRIu64 "\n", ids[v], ids[labels[v]]);
                break;
        }
        return 0;
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
}

}  // namespace gxexe
