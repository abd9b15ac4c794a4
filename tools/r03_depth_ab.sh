#!/bin/bash
# Round 3: narrow gathers three rounds deep (GX_PR_DEPTH=3) against two; PR parity first.
set -o pipefail
OUT=${1:-gpurun_out/depth}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "pagerank or narrow or PR" > "$OUT/pytest_pr.log" 2>&1 || { tail -30 "$OUT/pytest_pr.log"; exit 1; }
tail -1 "$OUT/pytest_pr.log"
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "d2:GX_PR_DEPTH=2" "d3:GX_PR_DEPTH=3" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "d2:GX_PR_DEPTH=2" "d3:GX_PR_DEPTH=3" || exit 1
echo depth-ok
