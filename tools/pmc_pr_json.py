#!/usr/bin/env python3
"""Per-iteration HBM traffic of the PageRank pull step from the rocprofv3 PMC passes of
tools/pr_counters.sh -> profiles/pmc_pr_pull.json (bench.py reads it for roofline.traffic).

    python tools/pmc_pr_json.py COUNTER_DIR CONFIG_NAME KERNEL_DESC > profiles/pmc_pr_pull.json

FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: on gfx950 FETCH_SIZE reports half the bytes
of a streaming read; FETCH_SIZE = TCC_EA0_RDREQ x 64 B for 128-B requests), WRITE_SIZE taken
as is; both are KB per dispatch.  Every dispatch matched by the pass is one iteration's SpMV.
"""
import collections
import csv
import glob
import json
import os
import sys

d, name, desc = sys.argv[1], sys.argv[2], sys.argv[3]
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, f"{name}_*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
fetch_kb, write_kb = mean["FETCH_SIZE"], mean["WRITE_SIZE"]
out = {
    "workload": "PageRank SYN-7_5 (R-MAT scale 20, ef 32, seed 75, undirected)",
    "kernel": desc,
    "launches_profiled": {"FETCH_SIZE": len(vals["FETCH_SIZE"]), "WRITE_SIZE": len(vals["WRITE_SIZE"])},
    "fetch_size_kb_per_launch": fetch_kb,
    "write_size_kb_per_launch": write_kb,
    "fetch_correction": "x2 (MI355X_MICROARCH.md HBM: FETCH_SIZE = TCC_EA0_RDREQ x 64 B; checked: "
                        "TCC_EA0_RDREQ x 128 B equals 2 x FETCH_SIZE here)",
    "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024,
    "algorithmic_bytes_per_launch": 4 * 60677656 + 8 * (1048576 + 1) + 16 * 1048576,
    "l2": {k: mean[k] for k in ("TCP_TCC_READ_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum") if k in mean},
    "stalls": {k: mean[k] for k in ("TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum",
                                    "TCP_TCC_READ_REQ_LATENCY_sum", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY",
                                    "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE") if k in mean},
}
print(json.dumps(out, indent=1))
