#!/bin/bash
# A/B of one PageRank environment knob on the default bench line (SYN-8_5 headline + SYN-7_5
# secondary), alternated: bash tools/pr_env_ab.sh OUT VAR "v1 v2 ..." [ROUNDS]
set -o pipefail
OUT=$1; VAR=$2; VALS=$3; ROUNDS=${4:-2}
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > "$OUT/${VAR}_${v}_$r.json" 2> "$OUT/${VAR}_${v}_$r.err" || exit 1
    python3 -c "
import json; d=json.loads(open('$OUT/${VAR}_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; s=d.get('secondary') or {}
print('$VAR=$v round $r: SYN-8_5 %.1f us frac %.3f | SYN-7_5 %s us' % (r['mean_launch_us'], r['frac'], s.get('mean_launch_us')))" | tee -a "$OUT/summary.txt"
  done
done
