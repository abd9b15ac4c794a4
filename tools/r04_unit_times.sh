#!/bin/bash
# Per-item timestamps of one k_pr_pull_units launch (GX_PR_UNIT_TIMES; the queued kernel on
# SYN-8_5, one workgroup per item on SYN-7_5), summarised by tools/unit_times.py.
# Usage (repo root, MI355X box): bash tools/r04_unit_times.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/unit_times}
mkdir -p "$OUT"
for G in SYN-8_5 SYN-7_5; do
  GX_PR_UNIT_TIMES="$OUT/ut_$G.txt" GX_PR_DRIVER=host GX_PR_GRAPH=0 timeout -k 10 300 python bench.py --graph $G \
      --no-secondary --no-cpu-baseline --steps 1 --warmup 1 > "$OUT/ut_$G.json" 2> "$OUT/ut_$G.err" || exit 1
  python3 tools/unit_times.py "$OUT/ut_$G.txt" > "$OUT/ut_${G}_summary.txt" || exit 1
done
