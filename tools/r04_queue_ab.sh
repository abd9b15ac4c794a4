#!/bin/bash
# k_pr_pull_units from a work queue (GX_PR_QUEUE=1: one resident workgroup per CU) against one
# workgroup per item: parity of the PageRank tests under the queue, then bench lines of both on
# SYN-8_5 / SYN-7_5, alternated.  Usage (repo root, MI355X box): bash tools/r04_queue_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/queue_ab}
mkdir -p "$OUT"
GX_PR_QUEUE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py -m gpu -x -q \
    -k "pagerank or pr_ or partition or device_driven or p2p" --timeout 150 --timeout-method thread > "$OUT/parity.log" 2>&1 || exit 1
for r in 1 2; do
  for q in 0 1; do
    GX_PR_QUEUE=$q timeout -k 10 200 python3 bench.py --steps 50 --no-cpu-baseline > "$OUT/q${q}_r$r.json" 2> "$OUT/q${q}_r$r.err" || exit 1
  done
done
