#!/bin/bash
# Round 3: per-rank PageRank pieces at N = 1 (GX_PR_PIECES = 8: the eight rank shares of an
# 8-GPU run, back to back on one GPU) on SYN-8_5 and SYN-7_5, and an SSSP bucket-width sweep.
set -o pipefail
OUT=${1:-gpurun_out/pieces}
mkdir -p "$OUT"
for G in SYN-8_5 SYN-7_5; do
  for P in 1 8; do
    GX_PR_PIECES=$P timeout -k 10 300 python bench.py --graph $G --steps 10 --warmup 2 --no-cpu-baseline --no-secondary \
        > "$OUT/${G}_p$P.json" 2> "$OUT/${G}_p$P.err" || exit 1
    tail -1 "$OUT/${G}_p$P.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$G P=$P', round(d['roofline']['mean_launch_us'],1), 'us per piece launch', round(d['ms_per_step'],3), 'ms per PR', d['config'].get('exchanged_doubles_per_n'), flush=True)" | tee -a "$OUT/summary.txt"
  done
done
for S in 2 3 4 6; do
  GX_SSSP_DSCALE=$S timeout -k 10 300 python bench.py --algorithm sssp --steps 4 --warmup 2 --no-cpu-baseline \
      > "$OUT/sssp_s$S.json" 2> "$OUT/sssp_s$S.err" || exit 1
  tail -1 "$OUT/sssp_s$S.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SSSP SYN-8_5 dscale $S', round(d['ms_per_step'],3), 'ms', flush=True)" | tee -a "$OUT/summary.txt"
done
echo pieces-ok
