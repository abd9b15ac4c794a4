#!/bin/bash
# Round 3: SSSP SYN-8_5 per-step log (GX_SSSP_VERBOSE=2) and totals (=1) of a warm call.
set -o pipefail
OUT=${1:-gpurun_out/sdiag}
mkdir -p "$OUT"
GX_SSSP_VERBOSE=2 timeout -k 10 300 python bench.py --algorithm sssp --steps 1 --warmup 2 --no-cpu-baseline \
    > "$OUT/v2.json" 2> "$OUT/v2.err" || exit 1
grep -c "^step" "$OUT/v2.err"
timeout -k 10 300 python bench.py --algorithm sssp --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/plain.json" 2> "$OUT/plain.err" || exit 1
echo sdiag-ok
