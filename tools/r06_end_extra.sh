#!/bin/bash
# Round-end extras (MI355X box, repo root): BFS PMC of the final tree and its bench line, the
# SYN-cit CDLP line and its kernel trace (timeline).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ex
bash tools/alg_pmc.sh gpurun_out/ex/pmc bfs > gpurun_out/ex/pmc.log 2>&1 || { tail -5 gpurun_out/ex/pmc.log; exit 1; }
timeout -k 10 600 python bench.py --algorithm bfs --steps 5 --warmup 2 > gpurun_out/ex/bfs_line.json 2> gpurun_out/ex/bfs_line.err || exit 1
timeout -k 10 600 python bench.py --algorithm cdlp --graph SYN-cit > gpurun_out/ex/cdlp_cit_line.json 2> gpurun_out/ex/cdlp_cit_line.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ex/prof -o run -- python3 bench.py --algorithm cdlp --graph SYN-cit --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic committed > gpurun_out/ex/cdlp_cit_prof.json 2> gpurun_out/ex/cdlp_cit_prof.err || exit 1
python3 tools/cdlp_timeline.py gpurun_out/ex/prof/run_kernel_trace.csv > gpurun_out/ex/timeline_syncit.txt || exit 1
rm -f gpurun_out/ex/prof/run_kernel_trace.csv
tail -c 300 gpurun_out/ex/bfs_line.json; tail -c 300 gpurun_out/ex/cdlp_cit_line.json
