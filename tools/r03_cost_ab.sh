#!/bin/bash
# Round 3: SYN-8_5 cache policy 1 vs 5 and the unit-order row cost (GX_PR_ROW_COST).
set -o pipefail
OUT=${1:-gpurun_out/cost}
mkdir -p "$OUT"
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "cp5:GX_PR_CP=5" "cp1:GX_PR_CP=1" "rc12:GX_PR_ROW_COST=12" "rc24:GX_PR_ROW_COST=24" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "rc4:GX_PR_ROW_COST=4" "rc12:GX_PR_ROW_COST=12" || exit 1
echo cost-ok
