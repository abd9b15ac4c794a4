#!/bin/bash
# Round-4 GPU batch 3 (repo root, MI355X box): rocprofv3 kernel summaries of LCC (SYN-cit) with
# and without the dense core (GX_LCC_CORE), only the stats files kept.
set -o pipefail
OUT=${1:-gpurun_out/r4i}
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 0 2048 4096; do
  GX_LCC_CORE=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_lcc_$k -o lcc -- \
      python3 bench.py --algorithm lcc --no-cpu-baseline --steps 10 --warmup 2 > "$OUT/lcc_$k.json" 2> "$OUT/lcc_$k.err" || exit 1
  f=$(find /tmp/prof_lcc_$k -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/lcc_core_${k}_kernel_stats.csv"
  rm -rf /tmp/prof_lcc_$k
done
