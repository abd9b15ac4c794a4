#!/bin/bash
# Round 3: the plan's key sort in 32-bit groups: PR parity (plan variants + full-size SYN-8_5),
# then the plan phase times and processing time on SYN-8_5.
set -o pipefail
OUT=${1:-gpurun_out/sg}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_fullsize.py -k "pagerank or narrow or PR" > "$OUT/pytest_pr.log" 2>&1 || { tail -30 "$OUT/pytest_pr.log"; exit 1; }
tail -1 "$OUT/pytest_pr.log"
GX_PLAN_TIMES=1 timeout -k 10 300 python bench.py --graph SYN-8_5 --no-secondary --no-cpu-baseline --steps 2 --warmup 1 \
    > "$OUT/plan.json" 2> "$OUT/plan.err" || exit 1
grep "^\[plan" "$OUT/plan.err" | head -16
bash tools/pr_ab.sh "$OUT" SYN-8_5 2 "u32:GX_PR_WIDE_KEYS=0" "u64:GX_PR_WIDE_KEYS=1" || exit 1
echo sg-ok
