#!/bin/bash
# Cache policy under the work queue and 32 Mi blocks (SYN-8_5): GX_PR_CP 5 (default: index stream
# and the narrow gathers past GX_PR_NT_COL non-temporal) at several NT_COL, and CP 1 / 0.
# Usage (repo root, MI355X box): bash tools/r04_cp_sweep.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/cp_sweep}
mkdir -p "$OUT"
for cfg in "5 65536" "5 32768" "5 131072" "5 262144" "1 0" "0 0"; do
  set -- $cfg
  GX_PR_CP=$1 GX_PR_NT_COL=$2 timeout -k 10 200 python3 bench.py --steps 30 --no-cpu-baseline --no-secondary \
      > "$OUT/cp$1_nt$2.json" 2> "$OUT/cp$1_nt$2.err" || exit 1
done
