#!/bin/bash
# Block size under the work queue (SYN-8_5; default 8 Mi entries, unit size simulated per block
# size).  Usage (repo root, MI355X box): bash tools/r04_block_sweep.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/block_sweep}
mkdir -p "$OUT"
for b in ${BLOCKS:-8388608 4194304 16777216 33554432}; do
  GX_PR_VERBOSE=1 GX_PR_BLOCK_NNZ=$b timeout -k 10 200 python3 bench.py --steps 30 --no-cpu-baseline --no-secondary \
      > "$OUT/b$b.json" 2> "$OUT/b$b.err" || exit 1
done
