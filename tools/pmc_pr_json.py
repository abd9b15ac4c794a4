#!/usr/bin/env python3
"""Per-iteration HBM traffic of the PageRank pull step from the rocprofv3 passes of
tools/pr_profile.sh -> profiles/pmc_pr_pull.json (bench.py reads it for roofline.traffic).

    python tools/pmc_pr_json.py OUTDIR KERNEL_DESC GRAPH [GRAPH ...] > profiles/pmc_pr_pull.json

FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: on gfx950 FETCH_SIZE reports half the bytes
of a streaming read; FETCH_SIZE = TCC_EA0_RDREQ x 64 B for 128-B requests), WRITE_SIZE taken
as is; both are KB per dispatch.  Every dispatch matched by the pass is one iteration's SpMV.
The kernel-trace pass gives the mean launch duration the bench line's HIP events must match.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def counters(path):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def trace_mean_us(path):
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Name"].startswith("void gx::(anonymous namespace)::k_pr_pull_units") or "k_pr_pull_units" in r["Name"]:
                return float(r["AverageNs"]) / 1e3, int(r["Calls"])
    return None, 0


def entry(outdir, g, desc):
    from bench import pr_workload
    line = json.loads(open(os.path.join(outdir, f"{g}_trace.json")).read().strip().splitlines()[-1])
    vals = collections.defaultdict(list)
    for i in (1, 2, 3):
        for k, v in counters(os.path.join(outdir, f"{g}_pmc{i}")).items():
            vals[k] += v
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    fetch_kb, write_kb = mean["FETCH_SIZE"], mean["WRITE_SIZE"]
    algo = line["roofline"]["bytes_per_launch"]
    hbm = (2 * fetch_kb + write_kb) * 1024
    t_us, calls = trace_mean_us(os.path.join(outdir, f"{g}_trace"))
    return {
        "workload": pr_workload(g),
        "kernel": desc,
        "launches_profiled": {"FETCH_SIZE": len(vals["FETCH_SIZE"]), "WRITE_SIZE": len(vals["WRITE_SIZE"])},
        "fetch_size_kb_per_launch": fetch_kb,
        "write_size_kb_per_launch": write_kb,
        "fetch_correction": "x2 (MI355X_MICROARCH.md HBM: FETCH_SIZE = TCC_EA0_RDREQ x 64 B for 128-B requests)",
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": hbm / algo,
        "l2": {k: mean[k] for k in ("TCP_TCC_READ_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum")
               if k in mean},
        "rocprof_mean_launch_us": t_us, "rocprof_launches": calls,
        "bench_mean_launch_us": line["roofline"]["mean_launch_us"],
    }


def main():
    outdir, desc, graphs = sys.argv[1], sys.argv[2], sys.argv[3:]
    print(json.dumps({"entries": [entry(outdir, g, desc) for g in graphs]}, indent=1))


if __name__ == "__main__":
    main()
