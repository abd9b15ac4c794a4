#!/bin/bash
# Round 3: SYN-8_5 1/8 pieces with larger sorted blocks (GX_PR_BLOCK_NNZ, 16 Ki rows).
set -o pipefail
OUT=${1:-gpurun_out/pieces3}
mkdir -p "$OUT"
for cfg in "b1m:GX_PR_BLOCK_NNZ=1048576" "b4m:GX_PR_BLOCK_NNZ=4194304,GX_PR_SORTED_ROWS=16320" \
           "b8m:GX_PR_BLOCK_NNZ=8388608,GX_PR_SORTED_ROWS=16320" "b4mu:GX_PR_BLOCK_NNZ=4194304,GX_PR_SORTED_ROWS=16320,GX_PR_UNIT_NNZ=524288"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env GX_PR_PIECES=8 $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python bench.py --graph SYN-8_5 --steps 10 --warmup 2 \
      --no-cpu-baseline --no-secondary > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
  tail -1 "$OUT/$name.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SYN-8_5 P=8 $name', round(d['roofline']['mean_launch_us'],1), 'us per piece launch', round(d['ms_per_step'],3), 'ms per PR', flush=True)" | tee -a "$OUT/summary.txt"
done
echo pieces3-ok
