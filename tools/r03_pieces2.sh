#!/bin/bash
# Round 3: SYN-8_5 per-rank pieces with 16 Ki-row blocks; SSSP bucket width 3 vs 4 on the
# undirected stand-ins.
set -o pipefail
OUT=${1:-gpurun_out/pieces2}
mkdir -p "$OUT"
for R in 4096 16320; do
  GX_PR_SORTED_ROWS=$R GX_PR_PIECES=8 timeout -k 10 300 python bench.py --graph SYN-8_5 --steps 10 --warmup 2 --no-cpu-baseline --no-secondary \
      > "$OUT/p8_r$R.json" 2> "$OUT/p8_r$R.err" || exit 1
  tail -1 "$OUT/p8_r$R.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SYN-8_5 P=8 rows $R', round(d['roofline']['mean_launch_us'],1), 'us per piece launch', flush=True)" | tee -a "$OUT/summary.txt"
done
for G in SYN-8_5 SYN-g500-22; do
  for S in 3 4 3 4; do
    GX_SSSP_DSCALE=$S timeout -k 10 300 python bench.py --algorithm sssp --graph $G --steps 4 --warmup 2 --no-cpu-baseline \
        > "$OUT/sssp_${G}_s$S.json" 2> "$OUT/sssp_${G}_s$S.err" || exit 1
    tail -1 "$OUT/sssp_${G}_s$S.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SSSP $G dscale $S', round(d['ms_per_step'],3), 'ms', flush=True)" | tee -a "$OUT/summary.txt"
  done
done
echo pieces2-ok
