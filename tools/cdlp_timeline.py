"""Per-iteration timeline of the last gx_cdlp call in a rocprofv3 kernel_trace.csv:
python tools/cdlp_timeline.py kernel_trace.csv.  A call starts at k_cdlp_first_sorted or
k_cdlp_first_dir (or the first tier kernel after a gather); iterations end at k_cdlp_flag_out."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"gx::\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*$", "", name)


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2].startswith(("k_cdlp_first_sorted", "k_cdlp_first_dir"))]
if not starts:
    # rows not sorted, or the shortcut off: a call (relabelled) ends with the gather
    # back to the caller's order, so the last call starts after the second-to-last gather
    ends = [i for i, r in enumerate(rows) if r[2].startswith("k_cdlp_gather_i32")]
    if len(ends) < 2:
        sys.exit("no call boundary in the trace")
    starts = [ends[-2] + 1]
i0 = starts[-1]
t0 = rows[i0][0]
last_end = t0
it = 0
for s, e, k in rows[i0:]:
    if not (k.startswith("k_cdlp") or k.startswith("k_keep")):
        continue
    print("%9.1f %7.1f %s" % ((s - t0) / 1e3, (e - s) / 1e3, k))
    if k.startswith("k_cdlp_flag_out"):
        print("# -- iteration %d ends at %.1f us (span %.1f)" % (it, (e - t0) / 1e3, (e - last_end) / 1e3))
        last_end = e
        it += 1
    if k.startswith("k_cdlp_gather_i32") and it > 0:
        print("# call ends at %.1f us" % ((e - t0) / 1e3))
        break
