#!/bin/bash
# PageRank SYN-7_5 (config 2) launch time under a list of plan settings, alternated with the
# default: bash tools/pr_env_sweep7.sh OUT "ENV1=a,ENV2=b" "ENV3=c" ...   (empty = default)
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
i=0
for spec in "" "$@" ""; do
  i=$((i+1))
  envs=$(echo "$spec" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --graph SYN-7_5 --no-cpu-baseline --no-secondary --pmc-traffic committed \
      --steps 300 --warmup 5 > "$OUT/s$i.json" 2> "$OUT/s$i.err" || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/s$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('[%s] SYN-7_5 %.1f us frac %.3f' % ('$spec' or 'default', r['mean_launch_us'], r['frac']))" | tee -a "$OUT/summary.txt"
done
