#!/bin/bash
# Round-4 GPU batch (repo root, MI355X box): parity of the round's last changes, the column
# pieces of config 4 (tools/pr_colpiece.py), then part A of the final evidence
# (tools/r04_final.sh).  Usage: bash tools/r04_combo.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r04_combo}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_ops.py tests/test_distributed.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
for a in "--pieces 1" "--pieces 8 --piece 0" "--pieces 8 --piece 5"; do
    timeout -k 10 300 python tools/pr_colpiece.py $a >> "$OUT/colpiece.jsonl" 2>> "$OUT/colpiece.err" || exit 1
done
bash tools/r04_final.sh "$OUT/final" A || exit 1
