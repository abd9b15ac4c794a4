#!/bin/bash
# Round 3: SYN-7_5 unit size sweep; SSSP pull threshold and fusion sweeps on SYN-8_5.
set -o pipefail
OUT=${1:-gpurun_out/sw3}
mkdir -p "$OUT"
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "t256k:GX_PR_UNIT_NNZ=262144" "t128k:GX_PR_UNIT_NNZ=131072" "t192k:GX_PR_UNIT_NNZ=196608" || exit 1
for cfg in "f8:GX_SSSP_PULL_FRAC=8" "f4:GX_SSSP_PULL_FRAC=4" "f16:GX_SSSP_PULL_FRAC=16" "fm8:GX_SSSP_FUSE_MAX=8" "f8b:GX_SSSP_PULL_FRAC=8"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 python bench.py --algorithm sssp --steps 4 --warmup 2 --no-cpu-baseline \
      > "$OUT/sssp_$name.json" 2> "$OUT/sssp_$name.err" || exit 1
  tail -1 "$OUT/sssp_$name.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SSSP SYN-8_5 $name', round(d['ms_per_step'],3), 'ms', flush=True)" | tee -a "$OUT/summary.txt"
done
echo sw3-ok
