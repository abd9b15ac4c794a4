#!/bin/bash
# CDLP x10 on SYN-7_5 (config 2's north-star CDLP workload): bench line and rocprofv3 kernel
# statistics (csv; traces removed, the stats are what profiles/ keeps).  Usage: bash
# tools/r04_cdlp_prof.sh OUT [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/r04_cdlp}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --algorithm cdlp --no-cpu-baseline --steps 10 --warmup 3 "$@" \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --algorithm cdlp --no-cpu-baseline --steps 10 --warmup 3 "$@" > "$OUT/prof.json" 2> "$OUT/prof.err" || exit 1
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/prof" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/prof"
