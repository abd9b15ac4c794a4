#!/bin/bash
# Round 3: PageRank narrow 2-byte codes.  GPU parity of the PR paths, then A/B of
# GX_PR_NARROW=1 (default) against 0 on SYN-8_5 and SYN-7_5, then the plan verbose line.
set -o pipefail
OUT=${1:-gpurun_out/narrow}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "pagerank or narrow or PR" > "$OUT/pytest_pr.log" 2>&1 || { tail -30 "$OUT/pytest_pr.log"; exit 1; }
tail -2 "$OUT/pytest_pr.log"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_distributed.py tests/test_ops.py > "$OUT/pytest_dist.log" 2>&1 || { tail -30 "$OUT/pytest_dist.log"; exit 1; }
tail -2 "$OUT/pytest_dist.log"
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "nar1:GX_PR_NARROW=1" "nar0:GX_PR_NARROW=0" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "nar1:GX_PR_NARROW=1" "nar0:GX_PR_NARROW=0" || exit 1
GX_PR_VERBOSE=1 timeout -k 10 300 python bench.py --graph SYN-8_5 --no-secondary --no-cpu-baseline --steps 2 --warmup 1 \
    > "$OUT/verbose.json" 2> "$OUT/verbose.err" || exit 1
grep "gx_pr" "$OUT/verbose.err" | head -5
echo narrow-ok
