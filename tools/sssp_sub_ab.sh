#!/bin/bash
# SSSP light sub-phase A/B on SYN-8_5 (config 4): GX_SSSP_SUB = S (1: none), bit-exact parity
# against the oracle in every line.  Usage (repo root, MI355X box):
#   bash tools/sssp_sub_ab.sh OUT "1 4 8 16" [GRAPH]
set -o pipefail
OUT=${1:-gpurun_out/sssp_sub}
G=${3:-SYN-8_5}
mkdir -p "$OUT"
first=1
for k in ${2:-1 4 8 16}; do
  extra="--no-cpu-baseline"
  [ $first = 1 ] && extra=""   # one line with the oracle check (bit-exact) per graph
  GX_SSSP_SUB=$k timeout -k 10 300 python bench.py --algorithm sssp --graph "$G" --steps 10 --warmup 3 $extra \
      > "$OUT/sssp_sub_${G}_$k.json" 2> "$OUT/sssp_sub_${G}_$k.err" || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/sssp_sub_${G}_$k.json').read().strip().splitlines()[-1])
print('$G GX_SSSP_SUB=$k', 'device %.3f ms' % d['ms_per_step'], 'parity', d['parity_vs_oracle'],
      'split', None if not d.get('split_n1') else round(d['split_n1']['ms'], 3))" | tee -a "$OUT/summary.txt"
  first=0
done
