// rt_internal.h — helpers shared by the C-ABI translation units of librt_hip.so
// (rt_abi.cpp, rt_comm.cpp).  Internal; not part of the public boundary.
#pragma once

#include <hip/hip_runtime_api.h>

#include <string>

#include "rt_abi.h"

namespace rti {

// Records `msg` as this thread's rt_last_error() text and returns `s`.
rt_status fail(rt_status s, const std::string& msg);
rt_status hip_fail(hipError_t e, const char* what);
// RT_ERR_INVALID_SIZE unless 1 <= w, h <= 65536.
rt_status check_image(uint32_t w, uint32_t h);
// The HIP device of a context (rt_create's argument).
int ctx_device(const rt_ctx* ctx);

// Switches to a device for the duration of a call.
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace rti
