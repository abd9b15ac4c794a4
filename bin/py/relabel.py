#!/usr/bin/env python3
"""Drop-in for the reference's bin/py/relabel.py (called by load-graph.sh:50-60), without DuckDB.

Self-contained (numpy only), so it runs from a reference checkout where only this file is
copied.  Same command line (relabel.py:82-95): --graph-name
--input-vertex-path --input-edge-path --output-path --weighted --directed [--use-disk];
load-graph.sh:51-58 passes the abbreviated --input-vertex / --input-edge, which are accepted
as aliases.  Writes graph.vtx (original ids in .v order) and graph.mtx (1-based dense ids,
`general` for directed and `symmetric` for undirected graphs, `%%GraphBLAS GrB_BOOL|GrB_FP64`
type line), the layout of relabel.py:52-79.
"""
import argparse
from pathlib import Path

import numpy as np


def _bool(x):
    return str(x).lower() in ["true", "1", "yes"]


def relabel(v_path, e_path, weighted: bool):
    """relabel.py:37-79 restated: dense 0-based ids in .v file order (relabel.py:41);
    returns (mapping uint64, src int64, dst int64, weights float64 or None)."""
    ids = np.array(Path(v_path).read_text().split(), dtype=np.uint64)
    cols = 3 if weighted else 2
    tok = Path(e_path).read_text().split()
    if len(tok) % cols:
        raise SystemExit(f"relabel: {e_path}: expected {cols} fields per edge line")
    tok = np.array(tok, dtype=object).reshape(-1, cols) if tok else np.zeros((0, cols), dtype=object)
    es = tok[:, 0].astype(np.uint64)
    ed = tok[:, 1].astype(np.uint64)
    order = np.argsort(ids, kind="stable")
    sids = ids[order]

    def index(e):
        pos = np.searchsorted(sids, e)
        pos_c = np.minimum(pos, max(len(sids) - 1, 0))
        if len(e) and (len(sids) == 0 or not np.array_equal(sids[pos_c], e)):
            bad = e[(pos >= len(sids)) | (sids[pos_c] != e)][0] if len(sids) else e[0]
            raise SystemExit(f"relabel: edge endpoint {int(bad)} is not in {v_path}")
        return order[pos_c].astype(np.int64)

    w = tok[:, 2].astype(np.float64) if weighted else None
    return ids, index(es), index(ed), w


def write_vtx_mtx(out_dir, mapping, src, dst, w, directed: bool) -> None:
    """graph.vtx + graph.mtx as relabel.py:52-79 lays them out."""
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    with open(out / "graph.vtx", "w") as f:
        f.write("".join(f"{int(x)}\n" for x in mapping))
    element = "real" if w is not None else "integer"
    sym = "general" if directed else "symmetric"
    grb = "GrB_FP64" if w is not None else "GrB_BOOL"
    n = len(mapping)
    with open(out / "graph.mtx", "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate {element} {sym}\n%%GraphBLAS {grb}\n{n} {n} {len(src)}\n")
        step = 1 << 20
        for k0 in range(0, len(src), step):
            s1, d1 = src[k0:k0 + step] + 1, dst[k0:k0 + step] + 1
            if w is None:
                f.write("".join(f"{a} {b} 1\n" for a, b in zip(s1.tolist(), d1.tolist())))
            else:
                f.write("".join(f"{a} {b} {c!r}\n" for a, b, c in
                                zip(s1.tolist(), d1.tolist(), w[k0:k0 + step].tolist())))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph-name", type=str, required=True)
    ap.add_argument("--input-vertex-path", "--input-vertex", dest="input_vertex_path", type=str, required=True)
    ap.add_argument("--input-edge-path", "--input-edge", dest="input_edge_path", type=str, required=True)
    ap.add_argument("--output-path", type=str, required=True)
    ap.add_argument("--weighted", type=_bool, required=True)
    ap.add_argument("--directed", type=_bool, required=True)
    ap.add_argument("--use-disk", action="store_true", required=False)   # accepted, unused
    args = ap.parse_args(argv)
    print("Loading...")
    mapping, src, dst, w = relabel(args.input_vertex_path, args.input_edge_path, args.weighted)
    print("Relabelling...")
    print("Serializing textual mapping file (vtx)")
    print("Serializing textual matrix file (mtx)")
    write_vtx_mtx(args.output_path, mapping, src, dst, w, args.directed)


if __name__ == "__main__":
    main()
