#!/bin/bash
# A/B of PageRank plan / kernel switches on one box, alternated so clock drift shows:
# bash tools/pr_ab.sh OUT GRAPH ROUNDS "name:ENV=V,ENV=V" ...   (each config one bench run
# per round; prints launch us, frac, G edges/s and the parity error of each run)
set -o pipefail
OUT=$1; G=$2; N=$3; shift 3
mkdir -p "$OUT"
for k in $(seq 1 "$N"); do
  for cfg in "$@"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python bench.py --graph "$G" --no-secondary --cpu-seconds 0.1 \
        --steps 10 --warmup 2 > "$OUT/${G}_${name}_$k.json" 2> "$OUT/${G}_${name}_$k.err" || exit 1
    python3 -c "
import json; d=json.loads(open('$OUT/${G}_${name}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$G $name', 'launch %.1f us' % r['mean_launch_us'], 'frac %.3f' % r['frac'], '%.1f G edges/s' % (d['value']/1e9),
      'err %.2e' % d['parity_max_rel_err_vs_oracle'], 'proc %.0f ms' % d['processing_ms'])" | tee -a "$OUT/summary.txt"
  done
done
