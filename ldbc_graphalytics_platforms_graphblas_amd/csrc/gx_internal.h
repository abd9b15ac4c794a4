// gx_internal.h -- shared declarations of libgx (host runtime + HIP kernels).
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>

#include "gx.h"

namespace gx {

// Thread-local last-error message (gx_last_error).
void set_error(const std::string &msg);

// Return `code` after recording `msg`; used as `return fail(GX_INVALID_VALUE, "...")`.
int fail(int code, const std::string &msg);

// ---- multi-threaded host helpers (gx_host.cpp, OpenMP): the host side of uploads and
// result hand-back, which sit inside the Graphalytics processing time ----
// out[i] = (int32) in[i]; false if any in[i] >= limit.
bool host_narrow(const uint64_t *in, uint64_t count, uint64_t limit, int32_t *out, bool nt = false);
bool host_pack24(const uint64_t *in, uint64_t count, uint64_t limit, uint32_t *out);
// parallel memcpy
void host_copy(void *dst, const void *src, size_t bytes);
// rp[i] <= rp[i+1] for all i < n
bool host_monotone(const uint64_t *rp, uint64_t n);
// BFS levels: negative (unreached) -> INT64_MAX
void host_levels(const int32_t *in, uint64_t n, int64_t *out);
// labels: out[i] = (uint64) in[i]
void host_widen(const int32_t *in, uint64_t n, uint64_t *out);
// PageRank exchange layout: global column c of rank `owner` (ranges[owner] <= c < ranges[owner+1])
// -> owner * chunk + (c - ranges[owner]); returns 0, or bit 0 = a column >= n, bit 1 = a column
// past its owner's live rows
int host_chunk_columns(const uint64_t *ci, uint64_t nnz, const uint64_t *ranges, int nranks, const uint64_t *live,
                       uint64_t chunk, uint64_t n, int32_t *out);
// hub-first order: order[i] = the vertex at position i, out-degree descending, ties by id
void host_hub_order(const uint64_t *rp, uint64_t n, uint32_t *order);
// the rows `rows[j]` of (rp, ci) as a local CSR (out_rp from 0) with columns renamed by colmap
void host_pick_rows(const uint64_t *rp, const uint64_t *ci, const uint32_t *rows, uint64_t nrows, const int32_t *colmap,
                    int64_t *out_rp, int32_t *out_ci);
// hub-first order in parallel (the same order as host_hub_order): order[h] = vertex, perm[v] =
// position, hdeg[h] = degree of the vertex at position h
void host_hub_order_par(const uint64_t *rp, uint64_t n, int32_t *order, int32_t *perm, int64_t *hdeg);
// out[v] = a[idx[v]] (parallel)
void host_compose(const int32_t *a, const int32_t *idx, uint64_t n, int32_t *out);
// rows with at least one entry
uint64_t host_count_live(const uint64_t *rp, uint64_t n);
// entries [e0, e1) of the local CSR made of the rows `rows[j]` of (rp, ci) (local row
// pointers lrp, from 0), narrowed to int32 into out[0, e1 - e0); false: a column >= limit
bool host_pick_span(const uint64_t *rp, const uint64_t *ci, const int32_t *rows, const int64_t *lrp, uint64_t nrows,
                    uint64_t e0, uint64_t e1, uint64_t limit, int32_t *out);
// Write one byte per 4 KiB page of a caller's output buffer (parallel) while the device
// computes: its first-touch page faults are then off the result copy's critical path.
void host_prefault(void *p, size_t bytes);
// OpenMP threads of the calling host thread (gx_*_multi gives each device's thread a share)
int host_threads();
void host_set_threads(int n);
// CSR of A' (rows sorted)
void host_transpose(uint64_t n, const uint64_t *rp, const uint64_t *ci, uint64_t *trp, uint64_t *tci);

}  // namespace gx
