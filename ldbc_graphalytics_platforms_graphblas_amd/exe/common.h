// common.h -- the per-algorithm Graphalytics executables (bin/exe/{bfs,pr,sssp,wcc,cdlp,lcc}).
//
// Same process contract as the reference wrapper executables
// (src/main/c/src/algorithms/<alg>.cpp, invoked by bin/sh/execute-job.sh:68-151):
//   CLI      --key value pairs in any order, unknown keys ignored (utils.cpp:19-53)
//   input    D/graph.grb + D/graph.vtb with --binary true, else D/graph.mtx + D/graph.vtx
//   stdout   "Processing starts at: <epoch ms>" / "Processing ends at: <epoch ms>"
//            around the algorithm only (bfs.cpp:105-107)
//   output   one "<original id> <value>" line per vertex in internal order
//   exit     0 on success, non-zero on failure
// The LAGraph call between the markers is replaced by the libgx C ABI (include/gx.h).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "gx.h"

namespace gxexe {

// BenchmarkParameters (utils.h:12-21)
struct BenchmarkParameters {
    bool binary = false;
    std::string input_dir;
    std::string output_file;
    bool directed = false;
    unsigned long source_vertex = 0;
    double damping_factor = 0.0;
    int max_iteration = 0;
    unsigned long thread_num = 1;
};

// ParseBenchmarkParameters (utils.cpp:19-53)
BenchmarkParameters ParseBenchmarkParameters(int argc, char **argv);

// GetCurrentMilliseconds (utils.cpp:8-13)
long long GetCurrentMilliseconds();

// OK(): throw on a non-success status (utils.h:45-55)
void OK(int info, const char *what);

enum class Algorithm { BFS, PR, SSSP, WCC, CDLP, LCC };

int Main(int argc, char **argv, Algorithm alg);

}  // namespace gxexe
