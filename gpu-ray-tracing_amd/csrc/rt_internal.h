// rt_internal.h — helpers shared by the C-ABI translation units of librt_hip.so
// (rt_abi.cpp, rt_comm.cpp, rt_chain.cpp).  Internal; not part of the public boundary.
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
// Whether nranks band sets cover every band of a height-row image exactly once, each within
// rows_per_rank rows (rt_deinterleave_bands' precondition).
bool band_sets_cover(uint32_t height, uint32_t nranks, const rt_band_set* sets,
                     uint32_t rows_per_rank);

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

namespace rtk {
struct TraceParams;
}

// One-frame updates as AQL packets on context-owned HSA queues (rt_chain.cpp).  A segment
// is begin, up to kMaxSegmentPackets frame packets (one per frame and part, part k on queue
// k), end; it is ordered after the work issued on `stream` before begin, and `stream`'s
// later work after it.  chain_create never fails softly: chain_ok tells whether the
// machine offers what the chain needs (why: the reason if not), a hard error is returned.
// Every wait is bounded: a segment whose go wait gives up drops its frames (the chain
// kernels check the abort word before storing), a queue error or a segment that does not
// complete within the bound marks the chain failed (chain_failed), and the context then
// runs HIP launches.
namespace rtc {
struct Chain;
constexpr uint32_t kMaxSegmentPackets = 1024;
Chain* chain_create(int device, rt_status* status);
// RT_ERR_HIP (and the resources left in place) if a segment did not complete in time
rt_status chain_destroy(Chain* c);
bool chain_ok(const Chain* c, const char** why);
// whether a go wait gave up or a queue reported an error (no synchronisation)
bool chain_failed(Chain* c);
// the queues of `parts` parts exist (created now if not); false if one cannot be created
bool chain_queues(Chain* c, uint32_t parts);
rt_status chain_begin(Chain* c, hipStream_t stream, uint32_t parts);
rt_status chain_frame(Chain* c, const rtk::TraceParams& p, int kernel, uint32_t part);
rt_status chain_end(Chain* c, hipStream_t stream);
// drops an open segment (nothing of it has been submitted yet)
void chain_abort(Chain* c);
// 1 if a go wait gave up (its segment's frames were dropped), else 0; waits (bounded) for
// every segment in flight
rt_status chain_errors(Chain* c, uint32_t* out);
uint64_t chain_packets(const Chain* c);
}  // namespace rtc
