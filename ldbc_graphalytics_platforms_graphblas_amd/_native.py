"""ctypes binding of libgx.so (the C ABI declared in include/gx.h).

The HIP library is the product path: importing this module never falls back to a CPU
implementation.  If libgx.so is missing, `lib()` raises; if no gfx950 device is visible,
`Context()` raises (gx_init fails) -- both loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("GX_LIB", _HERE / "libgx.so"))


class GxError(RuntimeError):
    """Raised on a non-success gx_* status (mirrors OK() throwing, utils.h:45-55)."""

    def __init__(self, code: int, what: str, msg: str):
        super().__init__(f"GraphBLAS error [{code}]  {what}: {msg}")
        self.code = code


class gx_csr(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("nnz", C.c_uint64),
        ("rowptr", C.POINTER(C.c_uint64)),
        ("colidx", C.POINTER(C.c_uint64)),
        ("vals", C.POINTER(C.c_double)),
    ]


_P = C.c_void_p
_U64P = C.POINTER(C.c_uint64)
_I64P = C.POINTER(C.c_int64)
_DP = C.POINTER(C.c_double)

# (name, restype, argtypes) for every entry point of include/gx.h
SIGNATURES = [
    ("gx_init", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("gx_free", C.c_int, [_P]),
    ("gx_last_error", C.c_char_p, []),
    ("gx_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("gx_device_info", C.c_int, [_P, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]),
    ("gx_read_grb", C.c_int, [C.c_char_p, C.POINTER(gx_csr)]),
    ("gx_write_grb", C.c_int, [C.c_char_p, C.POINTER(gx_csr)]),
    ("gx_read_vtb", C.c_int, [C.c_char_p, C.POINTER(_U64P), _U64P]),
    ("gx_write_vtb", C.c_int, [C.c_char_p, _U64P, C.c_uint64]),
    ("gx_read_mtx", C.c_int, [C.c_char_p, C.POINTER(gx_csr)]),
    ("gx_read_vtx", C.c_int, [C.c_char_p, C.POINTER(_U64P), _U64P]),
    ("gx_csr_release", None, [C.POINTER(gx_csr)]),
    ("gx_host_free", None, [_P]),
    ("gx_rmat_csr", C.c_int, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_uint64,
                              C.c_int, C.c_int, C.POINTER(gx_csr)]),
    ("gx_graph_create", C.c_int, [_P, C.POINTER(gx_csr), C.c_int, C.POINTER(_P)]),
    ("gx_graph_free", C.c_int, [_P]),
    ("gx_graph_info", C.c_int, [_P, _U64P, _U64P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("gx_bfs", C.c_int, [_P, C.c_uint64, _I64P]),
    ("gx_pagerank", C.c_int, [_P, C.c_double, C.c_int, _DP]),
    ("gx_sssp", C.c_int, [_P, C.c_uint64, _DP]),
    ("gx_wcc", C.c_int, [_P, _U64P]),
    ("gx_cdlp", C.c_int, [_P, C.c_int, _U64P]),
    ("gx_lcc", C.c_int, [_P, _DP]),
    ("gx_mxv", C.c_int, [_P, C.c_int, C.c_int, _P, _P, _P, _P, _P]),
    ("gx_vxm", C.c_int, [_P, C.c_int, C.c_int, _P, _P, _P, _P, _P]),
    ("gx_mxm_masked", C.c_int, [_P, C.c_int, C.c_int, _I64P]),
    ("gx_set_kernel_timing", C.c_int, [_P, C.c_int]),
    ("gx_kernel_stats", C.c_int, [_P, C.c_char_p, _U64P, _DP]),
    ("gx_reset_kernel_stats", C.c_int, [_P]),
    ("gx_last_device_ms", C.c_int, [_P, _DP]),
    ("gx_pr_part_create", C.c_int, [_P, C.c_uint64, C.c_int, C.c_int, _U64P, _U64P, _U64P, _U64P,
                                    C.c_double, C.POINTER(_P)]),
    ("gx_pr_part_create_live", C.c_int, [_P, C.c_uint64, C.c_int, C.c_int, _U64P, _U64P, _U64P, _U64P, _U64P,
                                         C.c_double, C.POINTER(_P)]),
    ("gx_pr_part_chunk", C.c_int, [_P, _U64P]),
    ("gx_pr_part_init", C.c_int, [_P, _P, _P]),
    ("gx_pr_part_step", C.c_int, [_P, _P, _P, _P, _P]),
    ("gx_pr_part_free", C.c_int, [_P]),
    ("gx_comm_unique_id", C.c_int, [C.c_char_p]),
    ("gx_comm_create", C.c_int, [_P, C.c_int, C.c_int, C.c_char_p, C.POINTER(_P)]),
    ("gx_comm_free", C.c_int, [_P]),
    ("gx_pr_dist_create", C.c_int, [_P, C.POINTER(_P), C.c_int, C.POINTER(_P)]),
    ("gx_pr_dist_run", C.c_int, [_P, C.c_int, C.c_int, _P]),
    ("gx_pr_dist_scores", C.c_int, [_P, C.c_int, _DP]),
    ("gx_pr_dist_free", C.c_int, [_P]),
    ("gx_pr_dist_create_p2p", C.c_int, [C.c_int, C.c_int, C.POINTER(_P), C.c_int, C.c_char_p, C.POINTER(_P)]),
    ("gx_pr_dist_p2p_attach", C.c_int, [_P, C.c_char_p]),
    ("gx_pagerank_multi", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(gx_csr), C.c_int, C.c_double, C.c_int, _DP]),
    ("gx_sssp_multi", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(gx_csr), C.c_int, C.c_uint64, _DP]),
    ("gx_lcc_multi", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(gx_csr), C.c_int, _DP]),
    ("gx_bfs_multi", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(gx_csr), C.c_int, C.c_uint64,
                               C.POINTER(C.c_int64)]),
    ("gx_wcc_multi", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(gx_csr), C.c_int, C.POINTER(C.c_uint64)]),
    ("gx_cdlp_multi", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(gx_csr), C.c_int, C.c_int,
                                C.POINTER(C.c_uint64)]),
    ("gx_multi_prepare", C.c_int, [C.POINTER(_P), C.c_int]),
    ("gx_pagerank_csr", C.c_int, [_P, C.POINTER(gx_csr), C.c_int, C.c_double, C.c_int, _DP, C.POINTER(_P)]),
    ("gx_pr_partition", C.c_int, [C.c_uint64, _U64P, C.c_int, C.POINTER(C.c_uint32), _U64P, _U64P]),
    # multi-GPU steps (device pointers as c_void_p)
    ("gx_bfs_part_init", C.c_int, [_P, C.c_uint64, _P, _P]),
    ("gx_bfs_part_expand", C.c_int, [_P, C.c_uint64, C.c_uint64, _P, C.c_int64, _P, _P]),
    ("gx_bfs_part_commit", C.c_int, [_P, _P, _P, C.c_int64, _P, _P]),
    ("gx_wcc_part_init", C.c_int, [_P, _P, _P]),
    ("gx_wcc_part_hook", C.c_int, [_P, C.c_uint64, C.c_uint64, _P, _P, _P]),
    ("gx_wcc_part_compress", C.c_int, [_P, _P, _P]),
    ("gx_part_changes", C.c_int, [_P, _P, C.c_uint64, C.c_uint64, C.c_int, _P, _P, _P]),
    ("gx_part_apply", C.c_int, [_P, _P, C.c_int, C.c_uint64, _P, C.c_int, C.c_int, _P]),
    ("gx_part_pack_bits", C.c_int, [_P, C.c_uint64, _P, _P]),
    ("gx_part_or_bits", C.c_int, [_P, C.c_int, C.c_uint64, _P, _P]),
    ("gx_sssp_split_create", C.c_int, [_P, C.c_uint64, C.c_uint64, C.POINTER(_P)]),
    ("gx_sssp_split_delta", C.c_int, [_P, _DP]),
    ("gx_sssp_split_start", C.c_int, [_P, C.c_uint64, _P]),
    ("gx_sssp_split_relax", C.c_int, [_P, _P, _P, _P]),
    ("gx_sssp_split_apply", C.c_int, [_P, _P, _P, C.c_int, C.c_uint64, _P]),
    ("gx_sssp_split_distances", C.c_int, [_P, _P, _P]),
    ("gx_sssp_split_run", C.c_int, [_P, C.c_uint64, _DP]),
    ("gx_sssp_split_free", C.c_int, [_P]),
    ("gx_cdlp_part_create", C.c_int, [_P, C.c_uint64, C.c_uint64, C.POINTER(_P)]),
    ("gx_cdlp_part_init", C.c_int, [_P, _P, _P]),
    ("gx_cdlp_part_step", C.c_int, [_P, _P, _P, _P, _P]),
    ("gx_cdlp_part_free", C.c_int, [_P]),
    ("gx_lcc_part_create", C.c_int, [_P, C.POINTER(_P)]),
    ("gx_lcc_part_ranges", C.c_int, [_P, C.c_int, _U64P]),
    ("gx_lcc_part_counts", C.c_int, [_P, C.c_uint64, C.c_uint64, _P, _P]),
    ("gx_lcc_part_finish", C.c_int, [_P, _P, _P, _P]),
    ("gx_lcc_part_free", C.c_int, [_P]),
]

_lib = None


def lib() -> C.CDLL:
    """Load libgx.so (built in-tree by `make` / __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise FileNotFoundError(
                f"{LIB_PATH} is missing: build the HIP extension first (make, or "
                "python -c 'import __graft_entry__; __graft_entry__.build()'); there is no CPU fallback")
        L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code: int, what: str) -> None:
    if code != 0:
        raise GxError(code, what, lib().gx_last_error().decode(errors="replace"))


def as_u64p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    return a.ctypes.data_as(_U64P)


def as_dp(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_DP)


def as_i64p(a: np.ndarray):
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(_I64P)


def device_count() -> int:
    c = C.c_int(0)
    check(lib().gx_device_count(C.byref(c)), "gx_device_count")
    return c.value
