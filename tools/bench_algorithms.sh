#!/bin/bash
# Per-algorithm bench lines (BASELINE configs 3-5 + CDLP) on one MI355X.
# Usage (repo root, GPU box): bash tools/bench_algorithms.sh OUTDIR [alg ...]
set -o pipefail
OUT=${1:-gpurun_out/algs}
shift
ALGS=${@:-bfs wcc cdlp lcc sssp}
mkdir -p "$OUT"
for a in $ALGS; do
    extra=""
    [ "$a" = "sssp" ] && extra="--steps 3 --warmup 1"
    timeout -k 10 600 python bench.py --algorithm $a --steps 5 --warmup 2 $extra > "$OUT/$a.json" 2> "$OUT/$a.err"
    rc=$?
    echo "$a rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$OUT/$a.err"; exit $rc; }
    python3 -c "
import json,sys
d=json.loads(open('$OUT/$a.json').read().strip().splitlines()[-1])
c=d['cpu_baseline'] or {}
print(f\"{d['config']['workload']:22s} n={d['config']['n']} nnz={d['config']['nnz']}  {d['value']/1e9:8.2f} G{d['unit']}  dev {d['ms_per_step']:.2f} ms  first {d['first_call_ms']:.1f} ms  frac {d['roofline']['frac']:.3f}  cpu {c.get('value',0)/1e9:.3f} G  parity {d['parity_vs_oracle']}\")
"
done
