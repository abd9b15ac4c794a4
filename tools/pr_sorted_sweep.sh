#!/bin/bash
# PR kernel variants on the headline graph (run on the MI355X box from the repo root):
#   bash tools/pr_sorted_sweep.sh OUTDIR [tests]
set -o pipefail
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
if [ "$2" = tests ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
fi
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
}
run packed
run unpacked GX_PR_SORTED_VARIANT=5
run packed_v1 GX_PR_SORTED_VARIANT=1
run packed_v2 GX_PR_SORTED_VARIANT=2
run packed_b32k GX_PR_SORTED_NNZ=32768 GX_PR_LONG_NNZ=32768
run packed_r2k GX_PR_SORTED_ROWS=2048
run packed_v9 GX_PR_SORTED_VARIANT=9
echo sweep-ok
