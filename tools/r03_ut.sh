#!/bin/bash
# Round 3: raw per-workgroup timestamps (GX_PR_UNIT_TIMES) of one PageRank launch.
set -o pipefail
OUT=${1:-gpurun_out/ut}
mkdir -p "$OUT"
for G in SYN-7_5 SYN-8_5; do
  GX_PR_UNIT_TIMES="$OUT/ut_$G.txt" GX_PR_DRIVER=host GX_PR_GRAPH=0 timeout -k 10 300 python bench.py --graph $G \
      --no-secondary --no-cpu-baseline --steps 1 --warmup 1 > "$OUT/ut_$G.json" 2> "$OUT/ut_$G.err" || exit 1
done
echo ut-ok
