"""MI355X-native GraphBLAS execution layer for the LDBC Graphalytics algorithm hot path.

Drop-in for the LAGraph / SuiteSparse:GraphBLAS calls of the reference platform driver
(tomzzy1/ldbc_graphalytics_platforms_graphblas): BFS, PageRank, SSSP, WCC, CDLP and LCC as
hand-written HIP kernels for gfx950 behind the C ABI in include/gx.h (libgx.so).
"""
from ._native import GxError, device_count, lib  # noqa: F401
from .graphio import CSR, load_graphalytics, read_grb, read_vtb, rmat  # noqa: F401

__all__ = ["GxError", "device_count", "lib", "CSR", "load_graphalytics", "read_grb", "read_vtb", "rmat"]
