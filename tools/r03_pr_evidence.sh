#!/bin/bash
# Round 3: per-workgroup timestamps of one launch (GX_PR_UNIT_TIMES) and the rocprofv3 kernel
# trace + PMC passes (tools/pr_profile.sh) of the PageRank kernel on SYN-8_5 and SYN-7_5,
# summarised on the box (profiles/pmc_pr_pull.json format); the bulky trace databases are
# deleted so that gpurun_out stays under the copy-back limit.
set -o pipefail
OUT=${1:-gpurun_out/ev}
DESC=${2:-"k_pr_pull_units (column-sorted row blocks in interleaved units; narrow 2-byte lane-major codes for each block's dense prefix, wide X4 entries for the rest; pipelined gathers; one workgroup per CU; slab combine; fused dangling sum)"}
mkdir -p "$OUT"
for G in SYN-7_5 SYN-8_5; do
  GX_PR_UNIT_TIMES="$OUT/ut_$G.txt" GX_PR_DRIVER=host GX_PR_GRAPH=0 timeout -k 10 300 python bench.py --graph $G \
      --no-secondary --no-cpu-baseline --steps 1 --warmup 1 > "$OUT/ut_$G.json" 2> "$OUT/ut_$G.err" || exit 1
  python3 tools/unit_times.py "$OUT/ut_$G.txt" > "$OUT/ut_${G}_summary.txt" || exit 1
  rm -f "$OUT/ut_$G.txt"
done
for G in SYN-8_5 SYN-7_5; do
  bash tools/pr_profile.sh "$OUT/prof" $G || exit 1
  find "$OUT/prof" -name "*.db" -delete
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/${G}_kernel_stats.csv" \;
  find "$OUT/prof" -name "*kernel_trace.csv" -delete
done
python3 tools/pmc_pr_json.py "$OUT/prof" "$DESC" SYN-8_5 SYN-7_5 > "$OUT/pmc_pr_pull.json" || exit 1
du -sh "$OUT"
echo ev-ok
