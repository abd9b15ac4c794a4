#!/bin/bash
# PMC passes on k_pr_pull for both pull kernels (hub = default, adaptive).
# Usage (repo root, MI355X box): bash tools/pr_counters.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/counters}
mkdir -p "$OUT"
export TMPDIR=/tmp
SETS=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum"
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_PENDING_STALL_CYCLES_sum"
  "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
  "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
  "TD_TD_BUSY_sum TD_TC_STALL_sum"
  "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
)
for kern in hub adaptive; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    GX_PR_KERNEL=$kern timeout -k 10 240 rocprofv3 --pmc $set --kernel-include-regex k_pr_pull --output-format csv \
        -d "$OUT/${kern}_$i" -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/${kern}_$i.log" 2>&1
    echo "$kern set $i rc=$?"
  done
done
python3 - "$OUT" <<'EOF'
import csv, collections, glob, os, sys
out = sys.argv[1]
for kern in ("hub", "adaptive"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out, f"{kern}_*", "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {kern}")
    for k in sorted(acc):
        v = acc[k]
        print(f"  {k:40s} {sum(v)/len(v):18.1f}")
EOF
