#!/bin/bash
# PMC passes on the dispatches of one kernel (regex) under a bench.py command line; prints
# per-counter values of the longest dispatch and the sum over all dispatches.
# Usage (repo root, MI355X box): bash tools/kernel_counters.sh OUTDIR REGEX bench-args...
set -o pipefail
OUT=$1
REGEX=$2
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
SETS=(
  "TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"
  "TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_WRITE_REQ_sum"
  "TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS"
)
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$REGEX" --output-format csv \
      -d "$OUT/p$i" -o pmc -- python3 bench.py "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "set $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 - "$OUT" <<'EOF'
import csv, collections, glob, os, sys
out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "p*", "pmc_counter_collection.csv"))):
    rows = list(csv.DictReader(open(f)))
    disp = collections.defaultdict(dict)
    for r in rows:
        disp[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    # the longest dispatch is the one with the largest GRBM / wave cycles; fall back to the max of the first counter
    names = sorted({k for d in disp.values() for k in d})
    key = names[0]
    big = max(disp.values(), key=lambda d: max(d.values()))
    print(f"== {os.path.basename(os.path.dirname(f))}  dispatches={len(disp)}")
    for k in names:
        tot = sum(d.get(k, 0.0) for d in disp.values())
        print(f"  {k:40s} largest {big.get(k, 0):18.1f}   total {tot:18.1f}")
EOF
