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
dist() {  # name, pieces, env...
    local name=$1 P=$2; shift 2
    env GX_PR_PIECES=$P "$@" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
}
run s1 GX_PR_SLICES=1
run s2 GX_PR_SLICES=2
run s4 GX_PR_SLICES=4
run s8 GX_PR_SLICES=8
run s4_b128k GX_PR_SLICES=4 GX_PR_SORTED_NNZ=131072
run s8_b128k GX_PR_SLICES=8 GX_PR_SORTED_NNZ=131072
dist p8_s1 8 GX_PR_SLICES=1
dist p8_s4 8 GX_PR_SLICES=4
dist p8_s8 8 GX_PR_SLICES=8
echo sweep-ok
