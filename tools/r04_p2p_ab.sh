#!/bin/bash
# The one-shot peer-to-peer exchange against the device copies and RCCL at N = 1 (one GPU: the
# exchange protocol's cost per iteration, not xGMI bandwidth): bench.py --partitioned on
# SYN-8_5 cut into GX_PR_PIECES pieces.  Usage (repo root, MI355X box): bash tools/r04_p2p_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/p2p_ab}
mkdir -p "$OUT"
for pc in 1 8; do
  GX_PR_PIECES=$pc timeout -k 10 200 python3 bench.py --partitioned --steps 30 --no-cpu-baseline --no-secondary \
      > "$OUT/copies_p$pc.json" 2> "$OUT/copies_p$pc.err" || exit 1
  GX_PR_PIECES=$pc GX_PR_EXCHANGE=p2p timeout -k 10 200 python3 bench.py --partitioned --steps 30 --no-cpu-baseline \
      --no-secondary > "$OUT/p2p_p$pc.json" 2> "$OUT/p2p_p$pc.err" || exit 1
  GX_PR_PIECES=$pc timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --partitioned --steps 30 --no-cpu-baseline --no-secondary \
      > "$OUT/rccl_p$pc.json" 2> "$OUT/rccl_p$pc.err" || exit 1
done
