#!/bin/bash
# Units cut by weighted entries (GX_PR_UNIT_BY_COST=1, default on huge graphs) against by
# entries (0), SYN-8_5, alternated; then the full-size PageRank parity.  Usage: bash tools/r04_bycost_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/bycost}
mkdir -p "$OUT"
for r in 1 2; do
  for c in 1 0; do
    GX_PR_VERBOSE=1 GX_PR_UNIT_BY_COST=$c timeout -k 10 200 python3 bench.py --steps 30 --no-cpu-baseline --no-secondary \
        > "$OUT/c${c}_r$r.json" 2> "$OUT/c${c}_r$r.err" || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_fullsize.py -x -q -k pagerank --timeout 280 --timeout-method thread > "$OUT/full.log" 2>&1 || exit 1
