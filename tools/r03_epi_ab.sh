#!/bin/bash
# Round 3: batched epilogue loads + tail-row extension A/B, PR parity, plan phase times.
set -o pipefail
OUT=${1:-gpurun_out/epi}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "pagerank or narrow or PR" > "$OUT/pytest_pr.log" 2>&1 || { tail -30 "$OUT/pytest_pr.log"; exit 1; }
tail -1 "$OUT/pytest_pr.log"
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "def:GX_PR_TAIL_ROWS=4096" "t8k:GX_PR_TAIL_ROWS=8192" "t16k:GX_PR_TAIL_ROWS=16320" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-8_5 1 "def:GX_PR_TAIL_ROWS=16320" || exit 1
for G in SYN-7_5 SYN-8_5; do
  GX_PLAN_TIMES=1 timeout -k 10 300 python bench.py --graph $G --no-secondary --no-cpu-baseline --steps 2 --warmup 1 \
      > "$OUT/plan_$G.json" 2> "$OUT/plan_$G.err" || exit 1
  grep "^\[plan" "$OUT/plan_$G.err" | head -24
done
echo epi-ok
