#!/bin/bash
# A/B of one environment knob on a bench.py --algorithm line, alternated:
# bash tools/alg_env_ab.sh OUT ALG VAR "v1 v2 ..." [ROUNDS]
set -o pipefail
OUT=$1; ALG=$2; VAR=$3; VALS=$4; ROUNDS=${5:-2}
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --algorithm "$ALG" --no-cpu-baseline --steps 20 --warmup 3 > "$OUT/${ALG}_${VAR}_${v}_$r.json" 2> "$OUT/${ALG}_${VAR}_${v}_$r.err" || exit 1
    python3 -c "
import json; d=json.loads(open('$OUT/${ALG}_${VAR}_${v}_$r.json').read().strip().splitlines()[-1])
print('$ALG $VAR=$v round $r: %.3f ms frac %.3f' % (d['ms_per_step'], d['roofline']['frac']))" | tee -a "$OUT/summary.txt"
  done
done
