#!/usr/bin/env python3
"""Summarise tools/alg_pmc.sh output into profiles/<tag>_pmc_algorithms.json.

Per algorithm: the kernels launched by (nearly) every one of the 8 calls bench.py --steps 4
--warmup 1 makes (at least 4 dispatches; totals divided by 8) with their rocprofv3 mean
duration and per-run fabric bytes, and the one-off plan kernels (built by the first call,
cached) listed apart.  Bytes:
2 x FETCH_SIZE (gfx950 tallies a 128-B read request at 64 B, MI355X_MICROARCH.md HBM) +
WRITE_SIZE; the 32-B share of the read requests is reported so the x2 can be checked.

    python tools/alg_pmc_json.py OUTDIR OUTFILE
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def kname(full):
    """k_* symbol of a rocprof kernel name ("void gx::(anonymous namespace)::k_x<...>(...)")."""
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", full)
    return m.group(1) if m else None

CALLS = 8


def pmc(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k is None:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if (r["Dispatch_Id"], r["Counter_Name"]) not in seen:
                seen.add((r["Dispatch_Id"], r["Counter_Name"]))
    return acc


def stats(path):
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Name"])
            if k:
                d = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
                d["calls"] += int(r["Calls"])
                d["total_ns"] += float(r["TotalDurationNs"])
    return out


def main():
    outdir, outfile = sys.argv[1], sys.argv[2]
    res = {"how": __doc__.strip().splitlines()[2:8], "algorithms": {}}
    for alg in ("bfs", "wcc", "sssp", "cdlp", "lcc"):
        tr = os.path.join(outdir, f"{alg}_trace")
        if not os.path.isdir(tr):
            continue
        st = stats(tr)
        f1, f2, f3 = (pmc(os.path.join(outdir, f"{alg}_pmc{i}")) for i in (1, 2, 3))
        try:
            line = json.loads(open(os.path.join(outdir, f"{alg}_trace.json")).read().strip().splitlines()[-1])
            workload, bytes_model = line["config"]["workload"], line["roofline"]["bytes_per_run"]
        except Exception:
            workload, bytes_model = alg, None
        per_run, plan, other = {}, {}, {}
        for k, d in sorted(st.items(), key=lambda kv: -kv[1]["total_ns"]):
            e = {"dispatches": d["calls"], "mean_us": d["total_ns"] / d["calls"] / 1e3,
                 "fetch_bytes": 2.0 * f1.get(k, {}).get("FETCH_SIZE", 0.0) * 1024,
                 "write_bytes": f2.get(k, {}).get("WRITE_SIZE", 0.0) * 1024,
                 "ea_rdreq": f3.get(k, {}).get("TCC_EA0_RDREQ_sum", 0.0),
                 "ea_rdreq_32b": f3.get(k, {}).get("TCC_EA0_RDREQ_32B_sum", 0.0)}
            if alg == "sssp" and k.startswith("k_split_"):   # the bench's split-path leg, not gx_sssp
                other[k] = e
            elif d["calls"] >= CALLS // 2:   # launched by (nearly) every call; plan kernels run once or twice
                for x in ("fetch_bytes", "write_bytes", "ea_rdreq", "ea_rdreq_32b"):
                    e[x] /= CALLS
                e["dispatches_per_run"] = d["calls"] / CALLS
                e["us_per_run"] = d["total_ns"] / CALLS / 1e3
                per_run[k] = e
            else:
                plan[k] = e
        hbm = sum(e["fetch_bytes"] + e["write_bytes"] for e in per_run.values())
        res["algorithms"][alg] = {
            "workload": workload, "calls_profiled": CALLS, "per_run_kernels": per_run, "plan_kernels": plan,
            "other_path_kernels": other,
            "hbm_bytes_per_run": hbm, "algorithmic_bytes_per_run": bytes_model,
            "traffic_over_algorithmic": hbm / bytes_model if bytes_model else None,
            "device_us_per_run": sum(e["us_per_run"] for e in per_run.values())}
    with open(outfile, "w") as f:
        json.dump(res, f, indent=1)
    for alg, a in res["algorithms"].items():
        print(alg, a["workload"], "hbm %.1f MB/run" % (a["hbm_bytes_per_run"] / 1e6),
              "ratio", a["traffic_over_algorithmic"], "device %.0f us/run" % a["device_us_per_run"])
        for k, e in list(a["per_run_kernels"].items())[:4]:
            print("   ", k, "%.1f us/run" % e["us_per_run"], "%.1f MB" % ((e["fetch_bytes"] + e["write_bytes"]) / 1e6),
                  "32B share %.2f" % (e["ea_rdreq_32b"] / e["ea_rdreq"] if e["ea_rdreq"] else 0))


if __name__ == "__main__":
    main()
