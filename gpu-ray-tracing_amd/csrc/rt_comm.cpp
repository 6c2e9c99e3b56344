// rt_comm.cpp — the multi-GPU collective of librt_hip.so behind the C ABI (rt_abi.h,
// rt_comm_* / rt_gather_stripes).
//
// pixels are independent and every seed is a function of the global pixel, so
// the image shards over GPUs with no per-frame exchange; 8-row bands are dealt round-robin
// and each rank renders its bands into a compact buffer.  The one exchange is at the end
// of a job: ONE ncclGather (RCCL over xGMI, rccl.h:745) of the finished bands to the root,
// whose de-interleave kernel scatters them into the image.  The reference has no
// counterpart (one device, ComputeShaderNode::run, lib.rs:379-421); this is the call a host
// that drives one context per GPU makes after its last rt_update_frames.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_internal.h"
#include "rt_kernels.h"

struct rt_comm {
    ncclComm_t nccl = nullptr;
    int device = 0;
    uint32_t rank = 0, nranks = 0;
    // the root's gather buffer when the caller passes none (grown on demand)
    float* scratch = nullptr;
    size_t scratch_bytes = 0;
};

static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RT_COMM_ID_BYTES is RCCL's id size");

namespace {

using rti::DeviceGuard;
using rti::fail;
using rti::hip_fail;

// The root's gather buffer when the caller passes none: at least `bytes`, grown on demand.
rt_status scratch_buffer(rt_comm* comm, size_t bytes, hipStream_t stream) {
    if (bytes <= comm->scratch_bytes) return RT_OK;
    if (comm->scratch) {
        hipError_t e = hipStreamSynchronize(stream);   // the old one may be in use
        if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        (void)hipFree(comm->scratch);
        comm->scratch = nullptr;
        comm->scratch_bytes = 0;
    }
    hipError_t e = hipMalloc(&comm->scratch, bytes);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(gather buffer)");
    comm->scratch_bytes = bytes;
    return RT_OK;
}

rt_status nccl_fail(ncclResult_t r, const char* what) {
    return fail(RT_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

// Fills an rt_comm from an initialised RCCL communicator.
rt_status describe(rt_comm* c, ncclComm_t nc, int device) {
    int rank = 0, n = 0;
    ncclResult_t r = ncclCommUserRank(nc, &rank);
    if (r == ncclSuccess) r = ncclCommCount(nc, &n);
    if (r != ncclSuccess) return nccl_fail(r, "ncclCommUserRank/ncclCommCount");
    c->nccl = nc;
    c->device = device;
    c->rank = (uint32_t)rank;
    c->nranks = (uint32_t)n;
    return RT_OK;
}

}  // namespace

extern "C" {

rt_status rt_comm_unique_id(uint8_t out_id[RT_COMM_ID_BYTES]) {
    if (!out_id) return fail(RT_ERR_INVALID_ARGUMENT, "out_id is NULL");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    std::memcpy(out_id, &id, RT_COMM_ID_BYTES);
    return RT_OK;
}

rt_status rt_comm_create(rt_ctx* ctx, const uint8_t id[RT_COMM_ID_BYTES], uint32_t nranks,
                         uint32_t rank, rt_comm** out_comm) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!id || !out_comm) return fail(RT_ERR_INVALID_ARGUMENT, "NULL id or out_comm");
    *out_comm = nullptr;
    if (nranks == 0 || rank >= nranks) return fail(RT_ERR_INVALID_ARGUMENT, "bad rank/nranks");
    const int dev = rti::ctx_device(ctx);
    DeviceGuard guard(dev);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    rt_comm* c = new (std::nothrow) rt_comm();
    if (!c) return fail(RT_ERR_NO_MEMORY, "out of host memory");
    ncclUniqueId uid;
    std::memcpy(&uid, id, RT_COMM_ID_BYTES);
    ncclComm_t nc = nullptr;
    // (RCCL binds the communicator to the current device: the guard's)
    ncclResult_t r = ncclCommInitRank(&nc, (int)nranks, uid, (int)rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(r, "ncclCommInitRank");
    }
    if (rt_status s = describe(c, nc, dev)) {
        (void)ncclCommDestroy(nc);
        delete c;
        return s;
    }
    *out_comm = c;
    return RT_OK;
}

rt_status rt_comm_create_all(uint32_t ndev, const int* devices, rt_comm** out_comms) {
    if (ndev == 0 || !devices || !out_comms)
        return fail(RT_ERR_INVALID_ARGUMENT, "ndev is 0 or NULL devices / out_comms");
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    for (uint32_t i = 0; i < ndev; ++i) {
        out_comms[i] = nullptr;
        if (devices[i] < 0 || devices[i] >= count)
            return fail(RT_ERR_INVALID_DEVICE, "no such HIP device");
    }
    std::vector<ncclComm_t> nc(ndev, nullptr);
    {
        int prev = 0;
        (void)hipGetDevice(&prev);
        const ncclResult_t r = ncclCommInitAll(nc.data(), (int)ndev, devices);
        (void)hipSetDevice(prev);
        if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitAll");
    }
    for (uint32_t i = 0; i < ndev; ++i) {
        rt_comm* c = new (std::nothrow) rt_comm();
        rt_status s = c ? describe(c, nc[i], devices[i]) : fail(RT_ERR_NO_MEMORY, "out of host memory");
        if (s != RT_OK) {
            delete c;
            for (uint32_t j = 0; j < i; ++j) {
                delete out_comms[j];
                out_comms[j] = nullptr;
            }
            for (uint32_t j = 0; j < ndev; ++j) (void)ncclCommDestroy(nc[j]);
            return s;
        }
        out_comms[i] = c;
    }
    return RT_OK;
}

rt_status rt_comm_destroy(rt_comm* comm) {
    if (!comm) return fail(RT_ERR_INVALID_ARGUMENT, "comm is NULL");
    rt_status s = RT_OK;
    {
        DeviceGuard guard(comm->device);
        if (comm->scratch) {
            (void)hipDeviceSynchronize();   // a queued gather may still write it
            (void)hipFree(comm->scratch);
        }
        const ncclResult_t r = ncclCommDestroy(comm->nccl);
        if (r != ncclSuccess) s = nccl_fail(r, "ncclCommDestroy");
    }
    delete comm;
    return s;
}

rt_status rt_comm_info(const rt_comm* comm, uint32_t* out_rank, uint32_t* out_nranks,
                       int* out_device) {
    if (!comm) return fail(RT_ERR_INVALID_ARGUMENT, "comm is NULL");
    if (out_rank) *out_rank = comm->rank;
    if (out_nranks) *out_nranks = comm->nranks;
    if (out_device) *out_device = comm->device;
    return RT_OK;
}

rt_status rt_comm_group_start(void) {
    const ncclResult_t r = ncclGroupStart();
    return r == ncclSuccess ? RT_OK : nccl_fail(r, "ncclGroupStart");
}

rt_status rt_comm_group_end(void) {
    const ncclResult_t r = ncclGroupEnd();
    return r == ncclSuccess ? RT_OK : nccl_fail(r, "ncclGroupEnd");
}

rt_status rt_gather_stripes(rt_ctx* ctx, rt_comm* comm, const float* local, float* gathered,
                            float* out_rgba, uint32_t width, uint32_t height, uint32_t root,
                            void* stream_v) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!comm) return fail(RT_ERR_INVALID_ARGUMENT, "comm is NULL");
    if (!local) return fail(RT_ERR_INVALID_ARGUMENT, "local is NULL");
    if (rt_status s = rti::check_image(width, height)) return s;
    if (root >= comm->nranks) return fail(RT_ERR_INVALID_ARGUMENT, "root >= nranks");
    if (rti::ctx_device(ctx) != comm->device)
        return fail(RT_ERR_INVALID_ARGUMENT, "ctx and comm are on different devices");
    const bool is_root = comm->rank == root;
    if (is_root && !out_rgba) return fail(RT_ERR_INVALID_ARGUMENT, "out_rgba is NULL on the root");
    DeviceGuard guard(comm->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipStream_t stream = static_cast<hipStream_t>(stream_v);
    // every rank's send buffer has the root's row count (rank 0 holds the most bands)
    const uint32_t rows0 = rt_stripe_local_rows(height, 0, comm->nranks);
    const size_t count = (size_t)rows0 * width * 4u;   // floats per rank
    float* recv = nullptr;
    if (is_root) {
        recv = gathered;
        if (!recv) {
            if (rt_status s = scratch_buffer(comm, count * comm->nranks * sizeof(float), stream))
                return s;
            recv = comm->scratch;
        }
    }
    const ncclResult_t r =
        ncclGather(local, recv, count, ncclFloat32, (int)root, comm->nccl, stream);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGather");
    if (!is_root) return RT_OK;
    hipError_t e = rtk::launch_deinterleave(reinterpret_cast<const float4*>(recv),
                                            reinterpret_cast<float4*>(out_rgba), width, height,
                                            comm->nranks, rows0, stream);
    return e == hipSuccess ? RT_OK : hip_fail(e, "rt_deinterleave_kernel launch");
}

rt_status rt_gather_bands(rt_ctx* ctx, rt_comm* comm, const float* local, float* gathered,
                          float* out_rgba, uint32_t width, uint32_t height,
                          const rt_band_set* sets, uint32_t root, void* stream_v) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!comm) return fail(RT_ERR_INVALID_ARGUMENT, "comm is NULL");
    if (!local || !sets) return fail(RT_ERR_INVALID_ARGUMENT, "local or sets is NULL");
    if (rt_status s = rti::check_image(width, height)) return s;
    if (root >= comm->nranks) return fail(RT_ERR_INVALID_ARGUMENT, "root >= nranks");
    if (rti::ctx_device(ctx) != comm->device)
        return fail(RT_ERR_INVALID_ARGUMENT, "ctx and comm are on different devices");
    const bool is_root = comm->rank == root;
    if (is_root && !out_rgba) return fail(RT_ERR_INVALID_ARGUMENT, "out_rgba is NULL on the root");
    // every rank's send buffer has the largest share's row count
    uint32_t rows = 0;
    for (uint32_t r = 0; r < comm->nranks; ++r)
        rows = std::max(rows, sets[r].count * (uint32_t)RT_STRIPE_ROWS);
    if (rows == 0) return fail(RT_ERR_INVALID_ARGUMENT, "the band sets hold no band");
    // (checked before the collective, on every rank: the root would refuse them after it)
    if (!rti::band_sets_cover(height, comm->nranks, sets, rows))
        return fail(RT_ERR_INVALID_ARGUMENT, "band sets must cover every band once");
    DeviceGuard guard(comm->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipStream_t stream = static_cast<hipStream_t>(stream_v);
    const size_t count = (size_t)rows * width * 4u;   // floats per rank
    float* recv = nullptr;
    if (is_root) {
        recv = gathered;
        if (!recv) {
            if (rt_status s = scratch_buffer(comm, count * comm->nranks * sizeof(float), stream))
                return s;
            recv = comm->scratch;
        }
    }
    const ncclResult_t r =
        ncclGather(local, recv, count, ncclFloat32, (int)root, comm->nccl, stream);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGather");
    if (!is_root) return RT_OK;
    return rt_deinterleave_bands(ctx, recv, out_rgba, width, height, comm->nranks, sets, rows,
                                 stream);
}

}  // extern "C"
