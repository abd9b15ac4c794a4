#!/bin/bash
# Round 3: PageRank cache-policy A/B (GX_PR_CP=1: non-temporal index stream) on SYN-8_5 and
# SYN-7_5, alternated; then the plan's phase clock (GX_PLAN_TIMES=1) on both graphs.
set -o pipefail
OUT=${1:-gpurun_out/cp}
mkdir -p "$OUT"
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "cp0:GX_PR_CP=0" "cp1:GX_PR_CP=1" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "cp0:GX_PR_CP=0" "cp1:GX_PR_CP=1" || exit 1
for G in SYN-7_5 SYN-8_5; do
  GX_PLAN_TIMES=1 timeout -k 10 300 python bench.py --graph $G --no-secondary --no-cpu-baseline --steps 2 --warmup 1 \
      > "$OUT/plan_$G.json" 2> "$OUT/plan_$G.err" || exit 1
done
echo cp-ok
