#!/bin/bash
# Device-driven partitioned PageRank under torch.distributed.run at N = 1 (the only size a
# one-GPU box runs): P pieces = P virtual ranks, so a piece has the rows one rank holds at
# N = P (P = 8: the per-rank SpMV of an 8-GPU run; 16: 8 GPUs x 2 pipelined pieces).
#   bash tools/pr_dist_n1.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/dist}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/n1.json" 2> "$OUT/n1.err" || exit 1
for P in 1 2 8 16; do
GX_PR_PIECES=$P timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/d$P.json" 2> "$OUT/d$P.err" || exit 1
done
GX_PR_PIECES=16 GX_PR_GRAPH=0 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/ng16.json" 2> "$OUT/ng16.err" || exit 1
GX_PR_PIECES=16 GX_PR_DRIVER=host timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/host16.json" 2> "$OUT/host16.err" || exit 1
echo dist-ok
