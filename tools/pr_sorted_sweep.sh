#!/bin/bash
# PR kernel variants on the headline graph (run on the MI355X box from the repo root):
#   bash tools/pr_sorted_sweep.sh OUTDIR [tests]
set -o pipefail
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
if [ "$2" = tests ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
fi
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
}
for rep in a b; do
run v0$rep
run v1$rep GX_PR_SORTED_VARIANT=1
run v2$rep GX_PR_SORTED_VARIANT=2
run v3$rep GX_PR_SORTED_VARIANT=3
done
run v1_hot256k GX_PR_SORTED_VARIANT=1 GX_PR_HOT_COLS=262144
run v1_r2k GX_PR_SORTED_VARIANT=1 GX_PR_SORTED_ROWS=2048
run v1_b128k GX_PR_SORTED_VARIANT=1 GX_PR_SORTED_NNZ=131072
echo sweep-ok
