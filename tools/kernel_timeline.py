#!/usr/bin/env python3
"""Per-iteration kernel timeline of one call from a rocprofv3 --kernel-trace CSV.
    python tools/kernel_timeline.py TRACE.csv [marker-regex] [call-index]
A call starts at each launch whose name matches the marker (default k_cdlp_iota)."""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_cdlp_iota"
call = int(sys.argv[3]) if len(sys.argv) > 3 else 1
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))


def nm(k):
    m = re.search(r"(k_\w+(<[^>]*>)?)", k)
    return m.group(1) if m else k[:40]


names = [nm(r["Kernel_Name"]) for r in rows]
starts = [i for i, n in enumerate(names) if re.search(marker, n)]
s = starts[call]
e = starts[call + 1] if call + 1 < len(starts) else len(rows)
t0 = int(rows[s]["Start_Timestamp"])
tot = defaultdict(float)
for i in range(s, e):
    r = rows[i]
    st = (int(r["Start_Timestamp"]) - t0) / 1e3
    du = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[names[i]] += du
    print(f"{st:9.1f} {du:8.1f} {names[i][:70]}")
print("-- total us per kernel:")
for k, v in sorted(tot.items(), key=lambda t: -t[1]):
    print(f"{v:9.1f} {k}")
