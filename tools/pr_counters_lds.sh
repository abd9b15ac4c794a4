#!/bin/bash
# LDS / texture-path PMC passes on the PageRank pull kernel of one graph (one rocprofv3 run per
# set): what bounds a launch besides bytes.  Usage (repo root, MI355X box):
#   bash tools/pr_counters_lds.sh OUTDIR GRAPH [ENV=VAL ...]
set -o pipefail
OUT=${1:-gpurun_out/counters_lds}; G=${2:-SYN-8_5}; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
SETS=(
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_COUNT"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
)
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  env "$@" timeout -k 10 240 rocprofv3 --pmc $set --kernel-include-regex k_pr_pull --output-format csv \
      -d "$OUT/set_$i" -o pmc -- python3 bench.py --graph "$G" --steps 1 --warmup 0 --no-cpu-baseline --no-secondary \
      > "$OUT/set_$i.log" 2>&1 || { echo "set $i failed"; tail -5 "$OUT/set_$i.log"; exit 1; }
  echo "set $i ok"
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, os, sys
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "set_*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"  {k:40s} {sum(v)/len(v):20.1f}  (n={len(v)})")
PY
