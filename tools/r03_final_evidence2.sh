#!/bin/bash
# Round 3 evidence after the cache-policy threshold fix: SYN-8_5 rocprofv3 trace + PMC of the
# default kernel, unit times, then the full GPU suite, smoke() and the default bench line.
set -o pipefail
OUT=gpurun_out/ev2
mkdir -p "$OUT"
GX_PR_UNIT_TIMES="$OUT/ut_SYN-8_5.txt" GX_PR_DRIVER=host GX_PR_GRAPH=0 timeout -k 10 300 python bench.py --graph SYN-8_5 \
    --no-secondary --no-cpu-baseline --steps 1 --warmup 1 > "$OUT/ut_SYN-8_5.json" 2> "$OUT/ut_SYN-8_5.err" || exit 1
python3 tools/unit_times.py "$OUT/ut_SYN-8_5.txt" > "$OUT/ut_SYN-8_5_summary.txt" || exit 1
bash tools/pr_profile.sh "$OUT/prof" SYN-8_5 || exit 1
find "$OUT/prof" -name "*.db" -delete
find "$OUT/prof" -name "*kernel_trace.csv" -delete
python3 tools/pmc_pr_json.py "$OUT/prof" "k_pr_pull_units (column-sorted row blocks in interleaved units; narrow 2-byte lane-major codes for each block's dense prefix, wide X4 entries for the rest; pipelined gathers; one workgroup per CU; slab combine; fused dangling sum)" SYN-8_5 > "$OUT/pmc_pr_pull_syn8_5.json" || exit 1
bash tools/round_end_check.sh || exit 1
tail -1 gpurun_out/full_t.log
cat gpurun_out/smoke.log
echo final-evidence2-ok
