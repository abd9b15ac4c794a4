#!/usr/bin/env python3
"""Drop-in for the reference's bin/py/relabel.py (called by load-graph.sh:50-60), without DuckDB.

Same command line (relabel.py:82-95): --graph-name --input-vertex-path --input-edge-path
--output-path --weighted --directed [--use-disk].  Writes graph.vtx (original ids in .v order)
and graph.mtx (1-based dense ids, `general` for directed and `symmetric` for undirected graphs,
`%%GraphBLAS GrB_BOOL|GrB_FP64` type line), exactly the layout of relabel.py:52-79.
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from ldbc_graphalytics_platforms_graphblas_amd.graphio import relabel, write_vtx_mtx  # noqa: E402


def _bool(x):
    return str(x).lower() in ["true", "1", "yes"]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph-name", type=str, required=True)
    ap.add_argument("--input-vertex-path", type=str, required=True)
    ap.add_argument("--input-edge-path", type=str, required=True)
    ap.add_argument("--output-path", type=str, required=True)
    ap.add_argument("--weighted", type=_bool, required=True)
    ap.add_argument("--directed", type=_bool, required=True)
    ap.add_argument("--use-disk", action="store_true", required=False)   # accepted, unused
    args = ap.parse_args(argv)
    print("Loading...")
    mapping, src, dst, w = relabel(args.input_vertex_path, args.input_edge_path, args.directed, args.weighted)
    print("Relabelling...")
    print("Serializing textual mapping file (vtx)")
    print("Serializing textual matrix file (mtx)")
    write_vtx_mtx(args.output_path, mapping, src, dst, w, args.directed)


if __name__ == "__main__":
    main()
