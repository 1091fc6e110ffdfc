// ipt_internal.h — what the library's translation units share about a context
// (defined in ipt_kernels.hip); not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ipt_capi.h"

namespace ipt_internal {
int ctx_fail(ipt_ctx* ctx, int code, const std::string& msg);  // records ipt_last_error, returns code
hipStream_t ctx_stream(ipt_ctx* ctx);
int ctx_device(ipt_ctx* ctx);
int ctx_cus(ipt_ctx* ctx);
}  // namespace ipt_internal
