#!/bin/bash
# Round-4 GPU batch 2 (repo root, MI355X box): PageRank parity after the plan changes, the
# executable path's processing time with the plan's phase times, SSSP step counts per setting.
set -o pipefail
OUT=${1:-gpurun_out/r4g}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py -x -q -k "pagerank" \
    --timeout 120 --timeout-method thread > "$OUT/parity.log" 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_fullsize.py -x -q -k "pagerank or multi" --timeout 300 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1 || exit 1
GX_PLAN_TIMES=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 \
    > "$OUT/plan_times.json" 2> "$OUT/plan_times.err" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 10 --warmup 2 > "$OUT/bench_pr.json" \
    2> "$OUT/bench_pr.err" || exit 1
for k in 1 8 16; do
  GX_SSSP_SUB=$k GX_SSSP_VERBOSE=1 timeout -k 10 300 python bench.py --algorithm sssp --no-cpu-baseline --steps 2 \
      --warmup 1 > "$OUT/sssp_v_$k.json" 2> "$OUT/sssp_v_$k.err" || exit 1
done
