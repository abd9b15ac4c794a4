#!/bin/bash
# Round 3: non-temporal gather experiments on SYN-8_5 (GX_PR_CPX), then the PMC profile of
# the default kernel (tools/pr_profile.sh).
set -o pipefail
OUT=${1:-gpurun_out/ntx}
mkdir -p "$OUT"
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "def:GX_PR_CPX=0" "wnt:GX_PR_CPX=3" "n256k:GX_PR_CPX=5,GX_PR_NT_COL=262144" \
    "n64k:GX_PR_CPX=5,GX_PR_NT_COL=65536" "all256k:GX_PR_CPX=7,GX_PR_NT_COL=262144" || exit 1
bash tools/pr_profile.sh "$OUT/prof" SYN-8_5 || exit 1
echo ntx-ok
