#!/bin/bash
# PMC passes on the PageRank pull kernel, one rocprofv3 run per counter set (the microarch
# guide's rule: FETCH_SIZE and WRITE_SIZE in passes of their own).
# Usage (repo root, MI355X box): bash tools/pr_counters.sh OUTDIR [config ...]
#   config = name:ENV=VAL,ENV=VAL   e.g. sorted:GX_PR_KERNEL=sorted adaptive:GX_PR_KERNEL=adaptive
set -o pipefail
OUT=${1:-gpurun_out/counters}
shift
CONFIGS=("$@")
[ ${#CONFIGS[@]} -eq 0 ] && CONFIGS=("sorted:GX_PR_KERNEL=sorted" "adaptive:GX_PR_KERNEL=adaptive")
mkdir -p "$OUT"
export TMPDIR=/tmp
SETS=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
  "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
)
for cfg in "${CONFIGS[@]}"; do
  name=${cfg%%:*}
  envs=${cfg#*:}
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    env ${envs//,/ } timeout -k 10 240 rocprofv3 --pmc $set --kernel-include-regex k_pr_pull --output-format csv \
        -d "$OUT/${name}_$i" -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/${name}_$i.log" 2>&1
    echo "$name set $i rc=$?"
  done
done
python3 - "$OUT" "${CONFIGS[@]}" <<'PY'
import csv, collections, glob, os, sys
out = sys.argv[1]
for cfg in sys.argv[2:]:
    name = cfg.split(":")[0]
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out, f"{name}_*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {name}")
    for k in sorted(acc):
        v = acc[k]
        print(f"  {k:40s} {sum(v)/len(v):18.1f}  (n={len(v)})")
PY
