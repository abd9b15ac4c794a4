#!/bin/bash
# PMC of the queued PageRank kernel, then SYN-7_5 unit sizes with and without the queue.
set -o pipefail
mkdir -p gpurun_out/r5o
timeout -k 10 700 bash tools/r04_pr_pmc.sh gpurun_out/r5o > gpurun_out/r5o/pmc.log 2>&1 || exit 1
for cfg in "0 -" "1 -" "1 131072" "1 65536" "0 131072"; do
  set -- $cfg
  if [ "$2" = "-" ]; then
    GX_PR_QUEUE=$1 timeout -k 10 120 python3 bench.py --graph SYN-7_5 --steps 100 --no-cpu-baseline > gpurun_out/r5o/s75_q$1_auto.json 2>/dev/null || exit 1
  else
    GX_PR_QUEUE=$1 GX_PR_UNIT_NNZ=$2 timeout -k 10 120 python3 bench.py --graph SYN-7_5 --steps 100 --no-cpu-baseline > gpurun_out/r5o/s75_q$1_t$2.json 2>/dev/null || exit 1
  fi
done
