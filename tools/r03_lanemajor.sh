#!/bin/bash
# Round 3: narrow codes stored lane-major (instruction k = 64 consecutive entries): PR parity,
# then SYN-8_5 / SYN-7_5 lines with and without the non-temporal sparse-column gathers.
set -o pipefail
OUT=${1:-gpurun_out/lm}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "pagerank or narrow or PR" > "$OUT/pytest_pr.log" 2>&1 || { tail -30 "$OUT/pytest_pr.log"; exit 1; }
tail -2 "$OUT/pytest_pr.log"
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "def:GX_PR_CPX=0" "n256k:GX_PR_CPX=5,GX_PR_NT_COL=262144" "n64k:GX_PR_CPX=5,GX_PR_NT_COL=65536" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "def:GX_PR_CPX=0" "n256k:GX_PR_CPX=5,GX_PR_NT_COL=262144" || exit 1
echo lm-ok
