#!/bin/bash
# Round-4 GPU batch 3 (repo root, MI355X box): SSSP sub-phases in the source's bucket only, and
# rocprofv3 kernel summaries of LCC with and without the dense core.
set -o pipefail
OUT=${1:-gpurun_out/r4h}
mkdir -p "$OUT"
for cfg in "1:1" "4:4000000000" "8:4000000000" "16:4000000000" "1:1"; do
  k=${cfg%%:*}; m=${cfg#*:}
  GX_SSSP_SUB=$k GX_SSSP_SUB_MIN=$m timeout -k 10 300 python bench.py --algorithm sssp --no-cpu-baseline --steps 10 \
      --warmup 3 > "$OUT/sssp_b0_${k}.json" 2> "$OUT/sssp_b0_${k}.err" || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/sssp_b0_${k}.json').read().strip().splitlines()[-1])
print('GX_SSSP_SUB=$k (source bucket only)', 'device %.3f ms' % d['ms_per_step'])" | tee -a "$OUT/summary.txt"
done
export TMPDIR=/tmp
for k in 0 2048; do
  GX_LCC_CORE=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_lcc_$k" -o lcc -- \
      python3 bench.py --algorithm lcc --no-cpu-baseline --steps 10 --warmup 2 > "$OUT/lcc_$k.json" 2> "$OUT/lcc_$k.err" || exit 1
done
