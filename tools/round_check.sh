#!/bin/bash
# End-of-round evidence on the MI355X box (repo root): rocprofv3 kernel trace + PMC passes of
# the headline bench, the PR counter sets, the bench line with the CPU baseline, and smoke().
#   bash tools/round_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
bash tools/profile_round.sh "$OUT/prof" > "$OUT/prof.log" 2>&1 || exit 1
bash tools/pr_counters.sh "$OUT/cnt" "sorted:GX_PR_KERNEL=sorted" > "$OUT/cnt.txt" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
echo final-ok
