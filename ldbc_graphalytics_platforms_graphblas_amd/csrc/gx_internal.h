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

}  // namespace gx
