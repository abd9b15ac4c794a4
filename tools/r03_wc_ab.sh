#!/bin/bash
# Round 3: default cache policy now reaches the bench's partition path; wide-entry cost in the
# unit order / launch simulation (GX_PR_WIDE_COST, quarters).
set -o pipefail
OUT=${1:-gpurun_out/wc}
mkdir -p "$OUT"
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "w4:GX_PR_WIDE_COST=4" "w8:GX_PR_WIDE_COST=8" "w12:GX_PR_WIDE_COST=12" "cp0:GX_PR_CP=0" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-7_5 1 "w4:GX_PR_WIDE_COST=4" "w8:GX_PR_WIDE_COST=8" || exit 1
echo wc-ok
