"""Graphalytics processing time through the drop-in executables.

For each algorithm: write its BASELINE stand-in graph as graph.grb + graph.vtb, run
bin/exe/<alg> with the argument vector execute-job.sh builds, and read the processing time
from the `Processing starts/ends at: <epoch-ms>` markers (the collector's measure: graph
upload, derived structures and the algorithm; not file load or serialisation).  Prints one
JSON line per algorithm with processing_ms and EVPS = (|V| + |E|) / T_proc.

Usage (repo root, GPU box): python tools/exe_proc_time.py OUTDIR [alg ...]
"""
import json
import os
import re
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from bench import DEFAULT_GRAPH, PRESETS  # noqa: E402
from ldbc_graphalytics_platforms_graphblas_amd import graphio  # noqa: E402

EXE = ROOT / "bin" / "exe"


def main():
    out = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/exe")
    algs = sys.argv[2:] or ["bfs", "wcc", "pr", "cdlp", "lcc", "sssp"]
    out.mkdir(parents=True, exist_ok=True)
    work = Path(os.environ.get("TMPDIR", "/tmp")) / "gx_exe_graphs"
    written = {}
    for alg in algs:
        gname = DEFAULT_GRAPH[alg]
        P = PRESETS[gname]
        weighted = alg == "sssp"
        key = (gname, weighted)
        d = work / f"{gname}{'_w' if weighted else ''}"
        if key not in written:
            t0 = time.time()
            csr = graphio.rmat(P["scale"], P["ef"], P["seed"], undirected=P["undirected"], weighted=weighted)
            d.mkdir(parents=True, exist_ok=True)
            graphio.write_grb(d / "graph.grb", csr)
            graphio.write_vtb(d / "graph.vtb", np.arange(1, csr.n + 1, dtype=np.uint64))   # original ids 1..n
            deg = np.diff(csr.rowptr.astype(np.int64))
            written[key] = (csr.n, csr.nnz, int(np.argmax(deg)) + 1)
            print(f"# wrote {d} in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
            del csr
        n, nnz, src = written[key]
        directed = "false" if P["undirected"] else "true"
        res = out / f"{alg}.out"
        argv = [str(EXE / alg), "--binary", "true", "--jobid", "job-1", "--input-dir", str(d), "--output-file",
                str(res), "--directed", directed]
        if alg in ("bfs", "sssp"):
            argv += ["--source-vertex", str(src)]
        elif alg == "pr":
            argv += ["--damping-factor", "0.85", "--max-iteration", "10"]
        elif alg == "cdlp":
            argv += ["--max-iteration", "10"]
        argv += ["--log-path", str(out), "--threadnum", "16"]
        t0 = time.time()
        p = subprocess.run(argv, capture_output=True, text=True, timeout=900)
        wall = time.time() - t0
        if p.returncode != 0:
            print(p.stdout[-2000:], p.stderr[-2000:], file=sys.stderr)
            raise SystemExit(f"{alg}: exit code {p.returncode}")
        s = int(re.findall(r"Processing starts at:\s*(\d+)", p.stdout)[-1])
        e = int(re.findall(r"Processing ends at:\s*(\d+)", p.stdout)[-1])
        lines = sum(1 for _ in open(res))
        extra = {k: float(m[-1]) for k, m in
                 (("upload_ms", re.findall(r"Upload time:\s*([\d.]+)", p.stdout)),
                  ("algorithm_ms", re.findall(r"Algorithm time:\s*([\d.]+)", p.stdout)),
                  ("device_ms", re.findall(r"Device time:\s*([\d.]+)", p.stdout))) if m}
        edges = nnz if directed == "true" else nnz // 2
        proc_ms = float(e - s)
        print(json.dumps({"algorithm": alg, "graph": gname, "n": n, "nnz": nnz, "directed": directed == "true",
                          "processing_ms": proc_ms, "evps": (n + edges) / max(proc_ms, 1e-3) * 1e3,
                          "process_wall_s": wall, "output_lines": lines, "output_complete": lines == n,
                          **extra}),
              flush=True)
        res.unlink()


if __name__ == "__main__":
    main()
