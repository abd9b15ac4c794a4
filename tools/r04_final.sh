#!/bin/bash
# Round-4 final evidence on one MI355X (repo root).  Part A: the default command's bench line
# and the rocprofv3 --kernel-trace --stats summary of that same command.  Part B: the PageRank
# PMC passes on SYN-8_5 / SYN-7_5 (tools/pr_profile.sh, summarised into pmc_pr_pull.json) and
# the per-algorithm bench lines (tools/bench_algorithms.sh).  Traces are deleted so gpurun_out
# stays under the copy-back limit.   Usage: bash tools/r04_final.sh OUT A|B
set -o pipefail
OUT=${1:-gpurun_out/r04_final}
PART=${2:-A}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PART" = "A" ]; then
    timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/defprof" -o run -- \
        python3 bench.py > "$OUT/defprof_bench.json" 2> "$OUT/defprof.err" || exit 1
    find "$OUT/defprof" -name '*kernel_stats.csv' -exec cp {} "$OUT/default_cmd_kernel_stats.csv" \;
    rm -rf "$OUT/defprof"
else
    DESC="k_pr_pull_units (column-sorted row blocks in interleaved units; narrow 2-byte lane-major codes, wide X4 entries for the rest; pipelined gathers; one workgroup per CU; fused dangling sum)"
    for G in SYN-8_5 SYN-7_5; do
        bash tools/pr_profile.sh "$OUT/prof" $G || exit 1
        find "$OUT/prof" -name "*.db" -delete
        find "$OUT/prof/${G}_trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/${G}_kernel_stats.csv" \;
        find "$OUT/prof" -name "*kernel_trace.csv" -delete
    done
    python3 tools/pmc_pr_json.py "$OUT/prof" "$DESC" SYN-8_5 SYN-7_5 > "$OUT/pmc_pr_pull.json" || exit 1
    bash tools/bench_algorithms.sh "$OUT/algs" || exit 1
fi
du -sh "$OUT"
echo "final-$PART-ok"
