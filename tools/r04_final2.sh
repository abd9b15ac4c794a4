#!/bin/bash
# Round-4 closing run after the cost-weighted units: full-size + plan-variant PageRank parity,
# the default command's line and its rocprofv3 summary (tools/r04_final.sh A), the PMC passes.
set -o pipefail
OUT=${1:-gpurun_out/final2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_fullsize.py tests/test_gpu_parity.py -x -q -k "pagerank" --timeout 280 \
    --timeout-method thread > "$OUT/parity.log" 2>&1 || exit 1
timeout -k 10 600 bash tools/r04_final.sh "$OUT" A > "$OUT/final.log" 2>&1 || exit 1
timeout -k 10 250 bash tools/r04_pr_pmc.sh "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || exit 1
