#!/bin/bash
# A/B of the split-block PageRank kernel's index loads: GX_PR_INDEX_X4=1 (default,
# four entries per 16-B load) against 0 (one 4-B load per entry), alternated so clock drift
# shows; the bench line's parity field checks each against the oracle.
# Usage (repo root, MI355X box): bash tools/pr_x4_ab.sh OUTDIR [ROUNDS]
set -o pipefail
OUT=${1:-gpurun_out/x4_ab}
mkdir -p "$OUT"
for k in $(seq 1 "${2:-2}"); do
  for x in 1 0; do
    GX_PR_INDEX_X4=$x timeout -k 10 240 python bench.py --cpu-seconds 1 --steps 10 --warmup 2 \
        > "$OUT/x4_${x}_$k.json" 2> "$OUT/x4_${x}_$k.err" || exit 1
    python3 -c "
import json; d=json.loads(open('$OUT/x4_${x}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']
print('x4=$x', 'launch %.1f us' % r['mean_launch_us'], 'frac %.3f' % r['frac'], '%.1f G edges/s' % (d['value']/1e9),
      'err', d.get('parity_max_rel_err_vs_oracle'))"
  done
done
