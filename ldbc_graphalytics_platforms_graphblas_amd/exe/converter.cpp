// bin/exe/converter -- drop-in for the reference's src/main/c/src/tools/converter.cpp:
// D/graph.vtx + D/graph.mtx  ->  D/graph.vtb + D/graph.grb  (called by load-graph.sh:63-67).
// SuiteSparse-free: the .mtx is parsed by gx_read_mtx and written by gx_write_grb in the
// sparse-CSR layout binread understands (graphio.h:49-285).
#include <cstring>
#include <iostream>
#include <string>

#include "common.h"

int main(int argc, char **argv) {
    std::string data_dir;
    // ParseConverterParameters (utils.cpp:55-68)
    for (int i = 0; i + 1 < argc; i++)
        if (std::strcmp(argv[i], "--data-dir") == 0) data_dir = argv[i + 1];
    try {
        uint64_t *ids = nullptr, n = 0;
        gxexe::OK(gx_read_vtx((data_dir + "/graph.vtx").c_str(), &ids, &n), "reading graph.vtx");
        gx_csr A{};
        gxexe::OK(gx_read_mtx((data_dir + "/graph.mtx").c_str(), &A), "reading graph.mtx");
        std::cout << "Serializing binary mapping file (vtb)" << std::endl;
        gxexe::OK(gx_write_vtb((data_dir + "/graph.vtb").c_str(), ids, n), "writing graph.vtb");
        std::cout << "Serializing binary matrix file (grb)" << std::endl;
        gxexe::OK(gx_write_grb((data_dir + "/graph.grb").c_str(), &A), "writing graph.grb");
        gx_csr_release(&A);
        gx_host_free(ids);
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
    return 0;
}
