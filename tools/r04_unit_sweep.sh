#!/bin/bash
# Unit size under the work queue (SYN-8_5): the plan's simulated pick (GX_PR_VERBOSE prints it),
# then fixed sizes around it.  Usage (repo root, MI355X box): bash tools/r04_unit_sweep.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/unit_sweep}
mkdir -p "$OUT"
GX_PR_VERBOSE=1 timeout -k 10 200 python3 bench.py --steps 30 --no-cpu-baseline --no-secondary > "$OUT/auto.json" 2> "$OUT/auto.err" || exit 1
T=$(grep -o "unit size [0-9]*" "$OUT/auto.err" | head -1 | awk '{print $3}')
echo "auto T=$T"
for f in 50 75 125 150 200; do
  t=$(( (T * f / 100 + 8191) / 8192 * 8192 ))
  GX_PR_UNIT_NNZ=$t timeout -k 10 200 python3 bench.py --steps 30 --no-cpu-baseline --no-secondary > "$OUT/t$t.json" 2> "$OUT/t$t.err" || exit 1
done
