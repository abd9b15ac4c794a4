#!/bin/bash
# Unit size with 32 Mi blocks under the queue (SYN-8_5).  Usage: bash tools/r04_unit_sweep32.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/unit_sweep32}
mkdir -p "$OUT"
for t in 1048576 1310720 1572864 1835008 2097152 2637824; do
  GX_PR_UNIT_NNZ=$t timeout -k 10 200 python3 bench.py --steps 30 --no-cpu-baseline --no-secondary > "$OUT/t$t.json" 2> "$OUT/t$t.err" || exit 1
done
