#!/bin/bash
# Round-4 diagnostics on one MI355X box (repo root): PageRank tail-locality probes on SYN-8_5
# (tools/pr_probe.sh; probe 2 no gathers, 8 sparse-tail gathers folded into the hub lines,
# 9 every gather folded into 512 KiB, 4 every gather an L1 hit), the plan's phase times of the
# executable path (GX_PLAN_TIMES) and SSSP's per-step log.  Usage: bash tools/r04_diag.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r04_diag}
mkdir -p "$OUT"
bash tools/pr_probe.sh "$OUT" SYN-8_5 "${PROBES:-0 2 8 9 4}" || exit 1
GX_PLAN_TIMES=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 \
    > "$OUT/plan_times.json" 2> "$OUT/plan_times.err" || exit 1
GX_SSSP_VERBOSE=2 timeout -k 10 300 python bench.py --algorithm sssp --no-cpu-baseline --steps 3 --warmup 2 \
    > "$OUT/sssp.json" 2> "$OUT/sssp_verbose.err" || exit 1
