#!/bin/bash
# Round-end profiles (MI355X box, repo root): the CDLP PMC refresh, every algorithm's bench line, rocprofv3 --stats of the default bench command (in-run PMC off: --pmc-traffic committed, no nested profilers).
set -o pipefail
mkdir -p gpurun_out/fb
export TMPDIR=/tmp
bash tools/alg_pmc.sh gpurun_out/fb/pmc cdlp > gpurun_out/fb/pmc.log 2>&1 || { tail -5 gpurun_out/fb/pmc.log; exit 1; }
cp gpurun_out/fb/pmc/summary/pmc_algorithms.json profiles/r06_pmc_cdlp_end.json || exit 1
bash tools/bench_algorithms.sh gpurun_out/fb/algs bfs wcc cdlp lcc sssp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fb/trace -o bench -- python3 bench.py --pmc-traffic committed > gpurun_out/fb/trace_bench.json 2> gpurun_out/fb/trace.log || exit 1
f=$(find gpurun_out/fb/trace -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/fb/default_cmd_kernel_stats.csv; rm -rf gpurun_out/fb/trace
head -3 gpurun_out/fb/default_cmd_kernel_stats.csv | cut -c1-200
