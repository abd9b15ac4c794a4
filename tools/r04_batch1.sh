#!/bin/bash
# Round-4 GPU batch (repo root, MI355X box): parity of the new paths, then the A/Bs.
set -o pipefail
OUT=${1:-gpurun_out/r4f}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lcc or pagerank or sssp" --timeout 120 \
    --timeout-method thread > "$OUT/parity.log" 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_fullsize.py -x -q -k "sssp or lcc" --timeout 300 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1 || exit 1
bash tools/sssp_sub_ab.sh "$OUT" "1 4 8 16 1" > "$OUT/sssp_ab.log" 2>&1 || exit 1
bash tools/lcc_core_ab.sh "$OUT" "0 2048 4096 8192 0" > "$OUT/lcc_ab.log" 2>&1 || exit 1
GX_PLAN_TIMES=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 \
    > "$OUT/plan_times.json" 2> "$OUT/plan_times.err" || exit 1
