#!/bin/bash
# rocprofv3 evidence for the PageRank pull kernel on one graph: a kernel-trace --stats pass of
# the bench line and three PMC passes (FETCH_SIZE; WRITE_SIZE; L2 requests / hits / misses /
# fabric reads), each its own run.  Summarise with tools/pmc_pr_json.py.
# Usage (repo root, MI355X box): bash tools/pr_profile.sh OUTDIR GRAPH [ENV=V ...]
set -o pipefail
OUT=$1; G=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${G}_trace" -o trace -- \
    python3 bench.py --graph "$G" --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > "$OUT/${G}_trace.json" 2> "$OUT/${G}_trace.err" || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  env "$@" timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex k_pr_pull --output-format csv -d "$OUT/${G}_pmc$i" -o pmc -- \
      python3 bench.py --graph "$G" --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > "$OUT/${G}_pmc$i.log" 2>&1 || exit 1
done
