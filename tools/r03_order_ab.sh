#!/bin/bash
# Round 3: unit dispatch order (GX_PR_ORDER 0 largest first, 1 smallest first, 2 alternating).
set -o pipefail
OUT=${1:-gpurun_out/ord}
mkdir -p "$OUT"
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "o0:GX_PR_ORDER=0" "o1:GX_PR_ORDER=1" "o2:GX_PR_ORDER=2" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-8_5 1 "o0:GX_PR_ORDER=0" "o2:GX_PR_ORDER=2" || exit 1
echo ord-ok
