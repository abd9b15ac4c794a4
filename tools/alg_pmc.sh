#!/bin/bash
# rocprofv3 evidence for the non-PR algorithms: a kernel-trace --stats pass and
# three PMC passes (FETCH_SIZE; WRITE_SIZE; TCC_EA0_RDREQ + its 32-B part), each its own run of
# `bench.py --algorithm ALG --steps 4 --warmup 1 --no-cpu-baseline` (8 calls: first, 4 timed,
# 3 instrumented).  Summarise with tools/alg_pmc_json.py.
# Usage (repo root, MI355X box): bash tools/alg_pmc.sh OUTDIR [alg ...]
# The raw traces are summarised on the box (OUTDIR/summary/: pmc_algorithms.json and each
# algorithm's kernel_stats.csv) and then deleted: gpurun copies back at most 64 MiB.
set -o pipefail
OUT=${1:-gpurun_out/alg_pmc}
shift
ALGS=("$@")
[ ${#ALGS[@]} -eq 0 ] && ALGS=(bfs wcc sssp cdlp lcc)
mkdir -p "$OUT"
export TMPDIR=/tmp
for alg in "${ALGS[@]}"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${alg}_trace" -o trace -- \
      python3 bench.py --algorithm "$alg" --steps 4 --warmup 1 --no-cpu-baseline > "$OUT/${alg}_trace.json" 2> "$OUT/${alg}_trace.err" || exit 1
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex '::k_' --output-format csv -d "$OUT/${alg}_pmc$i" -o pmc -- \
        python3 bench.py --algorithm "$alg" --steps 4 --warmup 1 --no-cpu-baseline > "$OUT/${alg}_pmc$i.log" 2>&1 || exit 1
  done
  echo "$alg done"
done
mkdir -p "$OUT/summary"
python3 tools/alg_pmc_json.py "$OUT" "$OUT/summary/pmc_algorithms.json" || exit 1
for alg in "${ALGS[@]}"; do
  f=$(find "$OUT/${alg}_trace" -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/summary/${alg}_kernel_stats.csv"
  cp "$OUT/${alg}_trace.json" "$OUT/summary/${alg}_bench.json"
  rm -rf "$OUT/${alg}_trace" "$OUT/${alg}_pmc1" "$OUT/${alg}_pmc2" "$OUT/${alg}_pmc3"
done
