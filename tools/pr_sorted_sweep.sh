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
for B in 40960 49152 57344 65536 73728 81920 98304; do
run b$B GX_PR_SORTED_NNZ=$B GX_PR_LONG_NNZ=$B
done
run r2048 GX_PR_SORTED_ROWS=2048
run r1024 GX_PR_SORTED_ROWS=1024
echo sweep-ok
