// rt_kernels.h — launch interface between the C-ABI layer (rt_abi.cpp) and the HIP
// kernels (rt_kernels.hip).  Internal; not part of the public boundary.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "rt_abi.h"

namespace rtk {

// Seeds travel in the kernarg segment (no H2D copy, graph-capturable).  rt_render with
// more frames is split into several launches that continue the accumulation.
constexpr uint32_t kMaxFramesPerLaunch = 128;
// Culled scan: lists up to this many spheres are staged in LDS (64 KiB per workgroup).
constexpr uint32_t kLdsMaxRecords = 4096;
// Per-tile candidate lists of camera rays (culled scan): capacity and the "no list" mark.
constexpr uint32_t kCandMax = 32;
constexpr uint32_t kNoHint = 0xFFFFFFFFu;
constexpr uint32_t kCandNone = 0xFFFFFFFFu;

// Everything the `update` kernel needs, passed by value (kernarg -> SGPRs).
struct TraceParams {
    const float4* in;    // local image (compact stripes), row pitch = width
    float4* out;
    const float4* geom;  // per sphere: (cx, cy, cz, r*r) — the scan's 16-B record
    const float4* sph;   // per sphere: the 32-B GpuSphere as two float4 (pos+r, color)
    uint32_t width, height, count;
    uint32_t band_first, band_step, local_bands;  // stripe map (RT_STRIPE_ROWS rows/band)
    uint32_t frames;       // accumulation frames in this launch (1 = one `update`)
    uint32_t reset_first;  // camera_has_moved > 0.5 applies to frame 0 only
    uint32_t lds_records;  // culled scan: records staged in LDS (0 = read from HBM/L2)
    uint32_t cand_k;       // per-tile candidate list capacity (0 = no lists)
    uint32_t n_hint;       // expected sample count of `in` (kNoHint = unknown), see trace_pixel
    const uint32_t* cand_cnt;  // [tile] listed spheres, kCandNone = no list
    const uint32_t* cand_idx;  // [tile][cand_k] sphere indices, ascending
    const float4* cand_rec;    // [tile][cand_k] their scan records
    float center[3], vul[3], pdu[3], pdv[3], ddu[3], ddv[3];
    float defocus_angle, max_depth, spp;
    float seeds[kMaxFramesPerLaunch];
};

hipError_t launch_trace(const TraceParams& p, int scan_mode, hipStream_t stream);
hipError_t launch_init(float4* out, uint64_t texels, hipStream_t stream);
// Builds the per-tile candidate lists for p's camera/scene/stripes (p.cand_k slots each).
hipError_t launch_candidates(const TraceParams& p, uint32_t* cnt, uint32_t* ids, float4* rec,
                             hipStream_t stream);
hipError_t launch_deinterleave(const float4* gathered, float4* out, uint32_t width,
                               uint32_t height, uint32_t nranks, uint32_t max_local_rows,
                               hipStream_t stream);
// 8-bit presentation of a float image (rt_present_rgba8); srgb_t = device T[256] or null
// for the linear encoding.
hipError_t launch_present(const float4* in, uchar4* out, uint64_t texels,
                          const float* srgb_t, hipStream_t stream);
const char* trace_kernel_name();

}  // namespace rtk
