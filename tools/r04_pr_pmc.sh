#!/bin/bash
# PageRank PMC passes on SYN-8_5 / SYN-7_5 (tools/pr_profile.sh) summarised into pmc_pr_pull.json;
# part B of tools/r04_final.sh without the per-algorithm lines.  Usage: bash tools/r04_pr_pmc.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/pr_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
DESC="k_pr_pull_units (column-sorted row blocks in interleaved units; narrow 2-byte lane-major codes, wide X4 entries for the rest; pipelined gathers; one resident workgroup per CU taking the units from a device work queue on SYN-8_5; fused dangling sum)"
for G in SYN-8_5 SYN-7_5; do
    bash tools/pr_profile.sh "$OUT/prof" $G || exit 1
    find "$OUT/prof" -name "*.db" -delete
    find "$OUT/prof/${G}_trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/${G}_kernel_stats.csv" \;
    find "$OUT/prof" -name "*kernel_trace.csv" -delete
done
python3 tools/pmc_pr_json.py "$OUT/prof" "$DESC" SYN-8_5 SYN-7_5 > "$OUT/pmc_pr_pull.json" || exit 1
du -sh "$OUT"
