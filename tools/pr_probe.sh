#!/bin/bash
# PageRank timing probes: the k_pr_pull_units launch with parts of its work
# removed or redirected, from the diagnostic build tools/probe/libgx.so (make probe;
# GX_PR_PROBE=k, wrong results by design).  One bench line per probe on OUT; prints
# "probe k: launch us".  Usage (repo root, MI355X box): bash tools/pr_probe.sh OUT [GRAPH] [PROBES]
set -o pipefail
OUT=${1:-gpurun_out/pr_probe}
G=${2:-SYN-7_5}
mkdir -p "$OUT"
for k in ${3:-0 1 2 3 4 5 6 7 0}; do
  GX_LIB=${PROBE_LIB:-tools/probe/libgx.so} GX_PR_PROBE=$k timeout -k 10 300 python bench.py --graph "$G" --no-cpu-baseline \
      --no-secondary --steps 10 --warmup 2 > "$OUT/probe_${G}_$k.json" 2> "$OUT/probe_${G}_$k.err" || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/probe_${G}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']
print('probe $k $G', 'launch %.1f us' % r['mean_launch_us'], 'frac %.3f' % r['frac'])" | tee -a "$OUT/summary.txt"
done
