#!/bin/bash
# Round profile of the headline bench (run on the MI355X box from the repo root):
#   bash tools/profile_round.sh OUTDIR
# 1. rocprofv3 --kernel-trace --stats of `python3 bench.py` (default workload)
# 2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) on k_pr_pull, as the microarch guide
#    prescribes (TCC FETCH_SIZE and WRITE_SIZE do not fit one pass)
set -o pipefail
OUT=${1:-gpurun_out/profile}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.log" || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_pr_pull --output-format csv -d "$OUT/fetch" -o pmc \
    -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > "$OUT/fetch.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_pr_pull --output-format csv -d "$OUT/write" -o pmc \
    -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > "$OUT/write.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_pr_pull \
    --output-format csv -d "$OUT/l2" -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > "$OUT/l2.log" 2>&1 || exit 1
echo profile-ok
