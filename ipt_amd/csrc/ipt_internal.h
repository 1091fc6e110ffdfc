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

// Owning device allocation: a call's temporaries are freed on every return
// path, early error returns included; release() hands the pointer over.
template <class T>
struct DevBuf {
    T* p = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    T* release() {
        T* q = p;
        p = nullptr;
        return q;
    }
};
}  // namespace ipt_internal
