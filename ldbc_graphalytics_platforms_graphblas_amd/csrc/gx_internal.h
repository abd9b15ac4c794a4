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
bool host_narrow(const uint64_t *in, uint64_t count, uint64_t limit, int32_t *out);
// parallel memcpy
void host_copy(void *dst, const void *src, size_t bytes);
// rp[i] <= rp[i+1] for all i < n
bool host_monotone(const uint64_t *rp, uint64_t n);
// BFS levels: negative (unreached) -> INT64_MAX
void host_levels(const int32_t *in, uint64_t n, int64_t *out);
// labels: out[i] = (uint64) in[i]
void host_widen(const int32_t *in, uint64_t n, uint64_t *out);

}  // namespace gx
