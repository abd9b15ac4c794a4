#!/bin/bash
# CDLP x10 on SYN-7_5: the own-label check's chunk size (GX_CDLP_KEEP_U) and the check off
# (GX_CDLP_KEEP=0), bench lines with per-kernel event times.  Usage: bash tools/r04_cdlp_keep_ab.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r04_cdlp_keep}
mkdir -p "$OUT"
for cfg in ${CFGS:-"GX_CDLP_KEEP=0" "GX_CDLP_KEEP_U=8" "GX_CDLP_KEEP_U=16" "GX_CDLP_KEEP_U=32"}; do
    env $cfg timeout -k 10 300 python bench.py --algorithm cdlp --no-cpu-baseline --steps 10 --warmup 3 \
        > "$OUT/${cfg}.json" 2> "$OUT/${cfg}.err" || exit 1
done
