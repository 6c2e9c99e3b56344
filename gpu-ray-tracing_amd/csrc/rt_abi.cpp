// rt_abi.cpp — C-ABI entry points of librt_hip.so (declared in include/rt_abi.h).
//
// Replaces the render-world half of the reference's plugin (src/lib.rs):
//   ComputeShaderPipeline::from_world (240-324)  -> rt_create (code objects are linked in)
//   prepare_sphere_buffer (177-207)              -> sphere upload, only when bytes change
//   prepare_camera_bind_group (151-175)          -> camera passed by value as kernarg
//   ComputeShaderNode::run (379-421)             -> rt_init_image / rt_update launches
// Errors are status codes instead of panics/unwraps (lib.rs:216-217, 356-358, 399-411).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_device.h"
#ifdef RT_CALL_STAMPS
// (diagnostic builds: host time stamps of rt_update_frames' phases, one stderr line per call)
#include <chrono>
static thread_local unsigned long long g_call_stamp[8];
static void call_stamp(int i) {
    g_call_stamp[i] = (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now().time_since_epoch())
                          .count();
}
#define CALL_STAMP(i) call_stamp(i)
#else
#define CALL_STAMP(i) ((void)0)
#endif
#include "rt_internal.h"
#include "rt_kernels.h"

struct rt_ctx {
    int device = 0;
    int scan_mode = RT_SCAN_CULLED;
    float4* d_geom = nullptr;  // count x (cx, cy, cz, r*r)
    float4* d_sph = nullptr;   // count x 2 float4 (the 32-B GpuSphere records)
    uint32_t capacity = 0;
    uint32_t count = 0;
    bool valid = false;
    std::vector<rt_sphere> cached;  // bytes currently on the device
    uint64_t scene_gen = 0;         // bumped on every sphere upload
    // max over spheres of |C| + |R| (inf if any value is not finite) and whether every
    // |R| lies in [2^-20, 2^20]: the scene half of camera_rays_bounded
    double scene_bound = 0.0;
    bool radii_ok = true;
    // one Markstein step from rcp_refined(R) is the IEEE division by every distinct radius
    // (rt_rcp_check_kernel, exhaustive over the numerators; TraceParams::normal_rn)
    bool normal_rn = false;
    uint32_t* d_flag = nullptr;     // the check's result word, then up to kRcpRadii radii
    float4* d_hint_rs = nullptr;    // TraceParams::hint_rs_dev (plan_hint_rs)
    // XZ grid of the small spheres for bounce rays (build_grid; TraceParams
    // grid_*): device arrays and the parameters copied into every launch.
    void* d_grid = nullptr;  // cell ranges (uint2), item records (float4), item indices, big list
    struct Grid {
        uint32_t nx = 0, nz = 0, nbig = 0, items = 0;
        float x0, z0, s, inv_s, ylo, yhi, cx, cy, cz, reach, m, e;
    } grid;
    // Per-tile candidate lists of camera rays (culled scan), valid for cand_key.
    float4* cand = nullptr;   // [tile][rtk::kCandStride] candidate blocks
    // workgroup order of one-frame launches (rtk::launch_wg_order), for candidate generation
    // band_gen; built when a generation is used a second time (a camera that moves every
    // frame never pays for it)
    uint32_t* wg_buf = nullptr;      // cost + order words
    uint64_t wg_cap = 0;
    uint32_t wg_pix = 0;
    uint32_t wg_parts = 0;           // sub-lists the order was dealt into
    uint64_t wg_builds = 0;          // order launches so far (a new order needs a new fork)
    uint64_t band_gen = ~0ull, band_seen_gen = ~0ull;
    uint64_t cand_tiles = 0;        // allocated tiles
    uint64_t cand_live = 0;         // tiles of the current lists
    std::vector<unsigned char> cand_key;
    uint64_t cand_gen = 0;          // bumped whenever the lists are rebuilt
    // Cost-ordered tiles (TraceParams::tile_order): per-tile durations recorded by the
    // first camera-ray-only launch of a list generation, and the order derived from them.
    uint32_t* tile_cost = nullptr;
    uint32_t* tile_order = nullptr;
    uint64_t order_tiles = 0;       // allocated tiles
    uint64_t cost_gen = ~0ull;      // cand_gen tile_cost was measured for
    uint32_t cost_frames = 0;       // frames of the launch that measured it
    uint64_t order_gen = ~0ull;     // cand_gen tile_order was derived for
    uint32_t order_frames = 0;      // frames of the measurement it came from
    uint32_t cost_group = 1;        // tiles per tile_cost/tile_order unit (bounce workgroups, pairs)
    // the share the last cost-recording launch ran (rt_band_costs): width, height, band
    // first, step, count, unit group; valid when cost_key_ok
    uint32_t cost_key[6] = {};
    bool cost_key_ok = false;
    // rt_deinterleave_bands' per-band source table on the device, and its host copy
    uint32_t* d_band_src = nullptr;
    std::vector<uint32_t> band_src;
    int tile_order_mode = RT_TILE_ORDER_AUTO;
    float* d_srgb = nullptr;  // rt_srgb_thresholds table on the device (256 floats)
    // hash(x*73) for x < hx_len (= rtk::hy_offset(width)), then hash(y*51) for y < hy_len
    // (wgsl:309-310), one buffer
    uint32_t* d_hx = nullptr;
    uint32_t hx_len = 0, hy_len = 0;
    // Sample counts of images this context wrote, when every pixel holds the same count:
    // the source of TraceParams::hint_n (a hint only: the kernel verifies it per pixel).
    struct CountRecord {
        const void* image;
        uint32_t w, h, first, step, bands, n;   // the image's size and band set, its count
    };
    std::vector<CountRecord> counts;
    uint32_t frames_per_launch = 0;  // rt_update_frames fusion cap (0 = automatic)
    rt_launch_info last = {0, 0, 0, -1, 0, 0, 0};  // the last call's launches (rt_last_launch_info)
    int path_compaction = RT_PATHS_AUTO;
    int frame_pairs = RT_FRAME_PAIRS_AUTO;
    int single_kernel = RT_SINGLE_AUTO;
    // Concurrent parts of one-frame updates (rt_set_update_queues): part 0 on the caller's
    // stream, part k on aux[k - 1], forked and joined through events.
    uint32_t update_queues = 0;      // 0 = automatic
    hipStream_t aux[RT_MAX_UPDATE_QUEUES - 1] = {};
    hipEvent_t fork_ev = nullptr;
    hipEvent_t join_ev[RT_MAX_UPDATE_QUEUES - 1] = {};
    // One-frame updates as AQL packets on the context's own HSA queues (rt_chain.cpp,
    // rt_set_update_submit), created on first use.
    int update_submit = RT_SUBMIT_AUTO;
    rtc::Chain* chain = nullptr;
    bool chain_tried = false;
    bool chain_reported = false;     // a chain failure has been returned to the caller once
    // Images of fused multi-frame launches (rt_set_frame_images): the last two frames' only,
    // or every frame's (TraceParams::store_each 1 / 2)
    int frame_images = RT_FRAME_IMAGES_LAST_TWO;
    // split bounce launches (TraceParams::split_col / split_cnt, plan_split)
    float4* split_col = nullptr;
    uint32_t* split_cnt = nullptr;
    uint64_t split_col_bytes = 0, split_cnt_tiles = 0;
    // their unit order (launch_unit_order) and its count, rebuilt when unit_key changes
    uint32_t* unit_order = nullptr;     // unit_cap entries, then the count
    uint64_t unit_cap = 0;
    uint64_t unit_key[5] = {~0ull, 0, 0, 0, 0};
    int cus = 0;                        // compute units of `device` (0: not queried yet)
    // rt_set_launch_timing: events the fused launches of each call carry, and how many
    // launches the last call timed
    hipEvent_t time_ev[2] = {};
    bool timing = false;
    uint32_t timed_launches = 0;
};

namespace {
thread_local std::string g_last_error = "";
}  // namespace

namespace rti {

rt_status fail(rt_status s, const std::string& msg) {
    g_last_error = msg;
    return s;
}

rt_status hip_fail(hipError_t e, const char* what) {
    return fail(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr uint32_t kMaxDim = 1u << 16;         // 65536 x 65536 texels

rt_status check_image(uint32_t w, uint32_t h) {
    if (w == 0 || h == 0 || w > kMaxDim || h > kMaxDim)
        return fail(RT_ERR_INVALID_SIZE, "image size out of range (1..65536 per side)");
    return RT_OK;
}

int ctx_device(const rt_ctx* ctx) { return ctx->device; }

}  // namespace rti

namespace {

using rti::check_image;
using rti::DeviceGuard;
using rti::fail;
using rti::hip_fail;

constexpr uint32_t kMaxSpheres = 1u << 20;
constexpr uint32_t kScanPad = 68;  // >= chunk round-up + one chunk + a 64-lane block

// WGSL u32(f32) on the host (truncate, saturate, NaN -> 0), as rtd::f2u.
uint32_t host_f2u(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

double norm3(const float* v) {
    return std::sqrt((double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2]);
}
double norm3d(const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// Whether every camera ray of p's camera, image and stripes, against the context's scene,
// stays inside the domain where the camera-ray-only instances use the exact fast division
// and sqrt cores (rt_kernels.hip consider_fast / fast_core): a = |d|^2 in [2^-11, 2^20],
// |O| + max(|C| + |R|) <= 2^40 (so |h|, sqrt(D) <= 2^53 and the hit-point numerators of
// the normal <= 2^43), and every |R| in [2^-20, 2^20].  d = pc - O (get_ray,
// wgsl:305-325) with pc = vul + sx pdu + sy pdv, sx in [0, W + 8], sy in [0, H + 8] (lanes
// past a ragged edge included), and O = center, or center + (cos, sin) (ddu, ddv) with a
// unit (cos, sin) when defocus_angle > 0.  |d| is bounded above by the sum of the parts and
// below by the distance along the normal of the pixel-delta plane, each widened by
// 1e-5 x the magnitudes entering the f32 evaluation (its rounding is < 1e-6 of them).
// Cameras or scenes outside the domain (degenerate, huge, non-finite, zero radii) run the
// IEEE operations in the culled instance instead.  Evaluated in double; NaN fails.
bool camera_rays_bounded(const rt_ctx* ctx, const rtk::TraceParams& p) {
    if (!ctx->radii_ok) return false;
    const bool defocus = p.defocus_angle > 0.0f;
    const double W = (double)p.width + 8.0, H = (double)p.height + 8.0;
    double e[3], nrm[3];
    for (int i = 0; i < 3; ++i) e[i] = (double)p.vul[i] - p.center[i];
    nrm[0] = (double)p.pdu[1] * p.pdv[2] - (double)p.pdu[2] * p.pdv[1];
    nrm[1] = (double)p.pdu[2] * p.pdv[0] - (double)p.pdu[0] * p.pdv[2];
    nrm[2] = (double)p.pdu[0] * p.pdv[1] - (double)p.pdu[1] * p.pdv[0];
    const double nn = std::sqrt(nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2]);
    if (!(nn > 0.0) || !std::isfinite(nn)) return false;
    auto along = [&](const double* v) {
        return std::fabs(v[0] * nrm[0] + v[1] * nrm[1] + v[2] * nrm[2]) / nn;
    };
    double du[3], dv[3];
    for (int i = 0; i < 3; ++i) {
        du[i] = defocus ? p.ddu[i] : 0.0;
        dv[i] = defocus ? p.ddv[i] : 0.0;
    }
    const double lens = std::sqrt(du[0] * du[0] + du[1] * du[1] + du[2] * du[2]) +
                        std::sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
    const double span = W * norm3(p.pdu) + H * norm3(p.pdv);
    const double mag = norm3(p.vul) + norm3(p.center) + span + lens;
    const double dmax = std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]) + span + lens +
                        1e-5 * mag;
    const double dmin = along(e) - along(du) - along(dv) - 1e-5 * mag;
    if (!(dmin > 0.0 && dmin * dmin >= 0x1p-11 && dmax * dmax <= 0x1p20)) return false;
    const double origin = norm3(p.center) + lens * (1.0 + 1e-5);
    return origin + ctx->scene_bound <= 0x1p40;
}

// Kernel instance for a launch (rtk::kTrace*): without bounce rays (max_depth <= 1) the
// culled mode needs only the candidate lists; the camera-ray-only instance also requires
// camera_rays_bounded (its fast cores).  Bounce rays (max_depth >= 2) run the bounce
// instance, whose path schedule (per wave by default, compacted or frame pairs) is
// rt_set_path_compaction's.
int trace_kernel_for(const rt_ctx* ctx, const rtk::TraceParams& p) {
    if (ctx->scan_mode == RT_SCAN_EXHAUSTIVE) return rtk::kTraceExhaustive;
#ifndef RT_FORCE_CULLED_KERNEL
    if (p.depth <= 1u && camera_rays_bounded(ctx, p)) return rtk::kTraceList;
#endif
#ifndef RT_NO_BOUNCE_KERNEL
    // bounce rays: the bounce instance (path schedule: TraceParams::compact)
    if (p.depth >= 2u) return rtk::kTraceBounce;
#endif
    return rtk::kTraceCulled;
}

// One-frame launches of the camera-ray-only instance run rt_single_kernel (rt_kernels.hip)
// unless rt_set_single_kernel(OFF).
int single_or(const rt_ctx* ctx, const rtk::TraceParams& p, int kernel) {
    if (kernel != rtk::kTraceList || p.frames != 1u || !p.cand ||
        ctx->single_kernel == RT_SINGLE_OFF)
        return kernel;
    if (ctx->single_kernel == RT_SINGLE_PAIR) return rtk::kTraceSingle;
    if (ctx->single_kernel == RT_SINGLE_ONE) return rtk::kTraceSingleOne;
    const uint64_t tiles = (uint64_t)((p.width + 7u) >> 3) * p.local_bands;
    return tiles <= rtk::kSingleOneMaxTiles ? rtk::kTraceSingleOne : rtk::kTraceSingle;
}

// Frames per rt_update_frames launch (see rt_update_frames): the camera-ray-only and the
// bounce instances fuse frames (both keep the accumulator in registers and store the last
// two frames' images); the others run one frame per launch.
uint32_t frames_per_launch_for(const rt_ctx* ctx, const rtk::TraceParams& p) {
    const int k = trace_kernel_for(ctx, p);
    const bool fusable = k == rtk::kTraceList || k == rtk::kTraceBounce;
    if (!fusable) return 1u;
    if (ctx->frames_per_launch)
        return std::min<uint32_t>(ctx->frames_per_launch, rtk::kMaxFramesPerLaunch);
    return rtk::kHintFrames;
}

// Uniform XZ grid of the small spheres (rt_kernels.hip scan_grid), built on every scene
// upload of at least kGridMinSpheres spheres whose |C| + |R| stay within 2^40 (so no f32
// intermediate of the root test overflows for the rays that may use the grid).  Small:
// |R| <= 4x the median radius; the others (the ground, the few large spheres) go to the
// big list that every ray tests.  Cells are about one small sphere's worth of the centres'
// bounding area, at most kGridMaxDim per axis.  A ray may walk the grid when
// 2.5e-3 (|o - c| + reach) <= m (c, reach: centre and radius of the small spheres' extent),
// which bounds the f32 discriminant margin of every small sphere by m; each sphere is then
// registered in every cell within sqrt(R^2 + m^2) + e of its centre, e bounding the f32 error of
// the walk's cell positions: (steps + 16) x 8 eps x the largest coordinate magnitude it
// handles, plus 1e-3 of a cell.  Rays further out, with |d|^2 outside [2^-20, 2^20] or
// non-finite, keep the exhaustive scan.
constexpr uint32_t kGridMinSpheres = 64;
// small spheres' centres per cell (round 5, with the sqrt(R^2 + m^2) registration: 1.0 —
// K5 436 against 445 us per fused frame at 2.0, profiles/r05/r05ab/, r05ac/)
#ifndef RT_GRID_PER_CELL
#define RT_GRID_PER_CELL 1.0
#endif
// (A/B) round 4's registration pad, R + m
#ifndef RT_GRID_PAD_ROUND4
#define RT_GRID_PAD_ROUND4 0
#endif
// (K5 per 64-spp step with far rays sharing the walk, tools/k5_ab.py, profiles/r06/r06x/,
// r06y/: 2 / 2.5 / 3 / 3.5 / 4 reaches 18.75 / 17.82 / 17.83-17.90 / 17.97 / 18.14 ms — a wider
// reach pads every registration, a narrower one leaves more far lanes that fail the miss test)
#ifndef RT_GRID_REACHES
#define RT_GRID_REACHES 3.0
#endif
#ifndef RT_GRID_E_STEPS
#define RT_GRID_E_STEPS 1
#endif
#ifndef RT_GRID_DISK
#define RT_GRID_DISK 1
#endif
constexpr uint32_t kGridMaxDim = 256;

rt_status build_grid(rt_ctx* ctx, const rt_sphere* sp, uint32_t count, hipStream_t stream) {
    ctx->grid.nx = 0;
    if (count < kGridMinSpheres || !(ctx->scene_bound <= 0x1p40)) return RT_OK;
    std::vector<double> radii(count);
    for (uint32_t i = 0; i < count; ++i) radii[i] = std::fabs((double)sp[i].radius);
    std::vector<double> sorted = radii;
    std::nth_element(sorted.begin(), sorted.begin() + count / 2, sorted.end());
    const double r_small = 4.0 * sorted[count / 2];
    std::vector<uint32_t> small, big;
    for (uint32_t i = 0; i < count; ++i) (radii[i] <= r_small ? small : big).push_back(i);
    if (small.size() < kGridMinSpheres / 2) return RT_OK;
    // extent of the small spheres: centre c (mid-point of the bounding box) and reach
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double rmax = 0.0;
    for (uint32_t i : small) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], (double)sp[i].position[k]);
            hi[k] = std::max(hi[k], (double)sp[i].position[k]);
        }
        rmax = std::max(rmax, radii[i]);
    }
    double c[3], g_r = 0.0;
    for (int k = 0; k < 3; ++k) c[k] = (double)(float)(0.5 * (lo[k] + hi[k]));
    for (uint32_t i : small) {
        double v[3];
        for (int k = 0; k < 3; ++k) v[k] = (double)sp[i].position[k] - c[k];
        g_r = std::max(g_r, norm3d(v));
    }
    const double reach = (g_r + rmax) * 1.001;
    // rays up to RT_GRID_REACHES - 1 reaches from the centre may use the grid
    const double m = 2.5e-3 * RT_GRID_REACHES * reach * 1.001 + 1e-30;
    const double area = std::max(hi[0] - lo[0], 1e-30) * std::max(hi[2] - lo[2], 1e-30);
    double s = std::sqrt(area * RT_GRID_PER_CELL / (double)small.size());
    s = std::max({s, (hi[0] - lo[0]) / (kGridMaxDim - 8), (hi[2] - lo[2]) / (kGridMaxDim - 8),
                  2.0 * rmax / 8.0, 1e-6});
    const double L = norm3d(c) + m / 2.5e-3 + 2.0 * reach + 4.0 * s;
    // e for walks of up to 2 kGridMaxDim steps; re-derived below from the grid's own step
    // bound nx + nz + 2 (RT_GRID_E_STEPS)
    double e = (2.0 * kGridMaxDim + 16.0) * 8.0 * 0x1p-24 * L + 1e-3 * s;
    // A ray that may use the grid accepts sphere (C, R) only at a point within
    // sqrt(R^2 + m^2) of C, plus the root's own rounding (< 1e-5 L): the computed
    // discriminant is negative beyond (the bound E <= m^2 of the culled scan).
    // Round 4 padded by R + m, up to m more (2.40 -> 1.98 registrations per small sphere of
    // the K5 scene).
    auto reg_w = [&](double r) {
        const double rr = r * 1.0001;
#if RT_GRID_PAD_ROUND4
        return rr + m + e;
#else
        return std::sqrt(rr * rr + m * m) + e + 1e-5 * L;
#endif
    };
    double x0, x1, z0, z1, ylo, yhi;
    uint32_t nx = 0, nz = 0;
    s = (double)(float)s;
    auto box = [&]() {
        x0 = INFINITY, x1 = -INFINITY, z0 = INFINITY, z1 = -INFINITY;
        ylo = INFINITY, yhi = -INFINITY;
        for (uint32_t i : small) {
            const double w = reg_w(radii[i]);
            x0 = std::min(x0, sp[i].position[0] - w);
            x1 = std::max(x1, sp[i].position[0] + w);
            z0 = std::min(z0, sp[i].position[2] - w);
            z1 = std::max(z1, sp[i].position[2] + w);
            ylo = std::min(ylo, sp[i].position[1] - w);
            yhi = std::max(yhi, sp[i].position[1] + w);
        }
        x0 = (double)(float)x0 - e;
        z0 = (double)(float)z0 - e;
        const double fx = std::ceil((x1 + e - x0) / s), fz = std::ceil((z1 + e - z0) / s);
        nx = fx >= 1.0 && fx <= kGridMaxDim ? (uint32_t)fx : 0u;
        nz = fz >= 1.0 && fz <= kGridMaxDim ? (uint32_t)fz : 0u;
    };
    box();
    if (nx < 1 || nz < 1) return RT_OK;
#if RT_GRID_E_STEPS
    // A walk takes at most nx + nz + 2 steps of this grid; e for that many is smaller, and
    // the box it gives lies inside this one (nx, nz do not grow), so it still bounds the
    // walks of the final grid (K5: 0.019 -> 0.003, 12 % fewer registrations).
    e = ((double)nx + (double)nz + 2.0 + 16.0) * 8.0 * 0x1p-24 * L + 1e-3 * s;
    box();
    if (nx < 1 || nz < 1) return RT_OK;
#endif
    // CSR: count, prefix, fill (small spheres in index order within every cell)
    const uint32_t cells = nx * nz;
    std::vector<uint32_t> start(cells + 1, 0u);
    auto span = [&](uint32_t i, uint32_t& ax, uint32_t& bx, uint32_t& az, uint32_t& bz) {
        const double w = reg_w(radii[i]);
        auto cell = [&](double v, double o, uint32_t n) {
            const double f = std::floor((v - o) / s);
            return (uint32_t)std::min(std::max(f, 0.0), (double)(n - 1));
        };
        ax = cell(sp[i].position[0] - w, x0, nx);
        bx = cell(sp[i].position[0] + w, x0, nx);
        az = cell(sp[i].position[2] - w, z0, nz);
        bz = cell(sp[i].position[2] + w, z0, nz);
    };
    // Of the square of cells, only those that meet the disk of radius w around the centre
    // (in XZ) can hold a point where the sphere is accepted, so only they list it (a walk
    // that passes such a point passes through the cell that contains it).  Widened by 1e-6
    // of a cell for the float rounding of the cell origin the kernel uses (RT_GRID_DISK).
    auto touches = [&](uint32_t i, uint32_t x, uint32_t z) {
#if RT_GRID_DISK
        const double w = reg_w(radii[i]) + 1e-6 * s;
        const double cx = sp[i].position[0], cz = sp[i].position[2];
        const double lx = x0 + s * x, hx = lx + s, lz = z0 + s * z, hz = lz + s;
        const double dx = std::max({lx - cx, cx - hx, 0.0});
        const double dz = std::max({lz - cz, cz - hz, 0.0});
        return dx * dx + dz * dz <= w * w;
#else
        (void)i, (void)x, (void)z;
        return true;
#endif
    };
    for (uint32_t i : small) {
        uint32_t ax, bx, az, bz;
        span(i, ax, bx, az, bz);
        for (uint32_t z = az; z <= bz; ++z)
            for (uint32_t x = ax; x <= bx; ++x)
                if (touches(i, x, z)) start[z * nx + x + 1]++;
    }
    for (uint32_t k = 0; k < cells; ++k) start[k + 1] += start[k];
    const uint32_t items = start[cells];
    // one buffer: cells x uint2, items x float4, items x u32, big x u32
    const size_t geom_off = ((size_t)cells * 8 + 15) & ~(size_t)15;   // float4-aligned
    const size_t idx_off = geom_off + (size_t)items * 16;
    const size_t big_off = idx_off + (size_t)items * 4;
    std::vector<unsigned char> buf(big_off + big.size() * 4 + 16);
    uint2* rng = reinterpret_cast<uint2*>(buf.data());
    float4* gg = reinterpret_cast<float4*>(buf.data() + geom_off);
    uint32_t* gi = reinterpret_cast<uint32_t*>(buf.data() + idx_off);
    for (uint32_t k = 0; k < cells; ++k) rng[k] = make_uint2(start[k], start[k + 1]);
    std::vector<uint32_t> fill(start.begin(), start.end() - 1);
    for (uint32_t i : small) {
        uint32_t ax, bx, az, bz;
        span(i, ax, bx, az, bz);
        const float4 rec = make_float4(sp[i].position[0], sp[i].position[1], sp[i].position[2],
                                       sp[i].radius * sp[i].radius);   // as upload_spheres
        for (uint32_t z = az; z <= bz; ++z)
            for (uint32_t x = ax; x <= bx; ++x) {
                if (!touches(i, x, z)) continue;
                const uint32_t k = fill[z * nx + x]++;
                gg[k] = rec;
                gi[k] = i;
            }
    }
    std::memcpy(buf.data() + big_off, big.data(), big.size() * 4);
    // The previous grid may still be read by queued launches: order on the stream.
    hipError_t err = hipStreamSynchronize(stream);
    if (err != hipSuccess) return hip_fail(err, "hipStreamSynchronize");
    (void)hipFree(ctx->d_grid);
    ctx->d_grid = nullptr;
    err = hipMalloc(&ctx->d_grid, buf.size());
    if (err != hipSuccess) return hip_fail(err, "hipMalloc(sphere grid)");
    err = hipMemcpyAsync(ctx->d_grid, buf.data(), buf.size(), hipMemcpyHostToDevice, stream);
    if (err == hipSuccess) err = hipStreamSynchronize(stream);
    if (err != hipSuccess) return hip_fail(err, "hipMemcpyAsync(sphere grid)");
    rt_ctx::Grid& g = ctx->grid;
    g.nx = nx;
    g.nz = nz;
    g.nbig = (uint32_t)big.size();
    g.items = items;
    g.x0 = (float)x0;
    g.z0 = (float)z0;
    g.s = (float)s;
    g.inv_s = (float)(1.0 / s);
    g.ylo = (float)(ylo - e);
    g.yhi = (float)(yhi + e);
    g.cx = (float)c[0];
    g.cy = (float)c[1];
    g.cz = (float)c[2];
    g.reach = (float)reach;
    g.m = (float)m;
    g.e = (float)e;
    return RT_OK;
}

rt_status upload_spheres(rt_ctx* ctx, const rt_sphere* spheres, uint32_t count,
                         hipStream_t stream) {
    if (count > kMaxSpheres) return fail(RT_ERR_INVALID_SIZE, "sphere_count too large");
    if (count > 0 && spheres == nullptr)
        return fail(RT_ERR_INVALID_ARGUMENT, "spheres is NULL with sphere_count > 0");
    if (ctx->valid && count == ctx->count &&
        (count == 0 || std::memcmp(ctx->cached.data(), spheres, count * sizeof(rt_sphere)) == 0))
        return RT_OK;  // unchanged since the last upload
    // From here the device copy no longer matches `cached`: a failure below leaves the
    // context invalid (the next call uploads again) and retires every scene-derived cache
    // (candidate lists, tile costs) by bumping the generation.
    ctx->valid = false;
    ctx->normal_rn = false;
    ctx->scene_gen++;
    if (count > ctx->capacity || ctx->d_geom == nullptr) {
        uint32_t cap = ctx->capacity ? ctx->capacity : 64u;
        while (cap < count) cap *= 2u;
        float4 *g = nullptr, *s = nullptr;
        // kScanPad zero records after the list: the scan prefetches one chunk ahead.
        const size_t geom_bytes = ((size_t)cap + kScanPad) * sizeof(float4);
        hipError_t e = hipMalloc(&g, geom_bytes);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(sphere geometry)");
        e = hipMemsetAsync(g, 0, geom_bytes, stream);
        if (e != hipSuccess) {
            (void)hipFree(g);
            return hip_fail(e, "hipMemsetAsync(sphere geometry)");
        }
        e = hipMalloc(&s, (size_t)cap * 2 * sizeof(float4));
        if (e != hipSuccess) {
            (void)hipFree(g);
            return hip_fail(e, "hipMalloc(sphere records)");
        }
        // The previous buffers may still be read by queued launches on `stream`.
        if (ctx->d_geom || ctx->d_sph) {
            e = hipStreamSynchronize(stream);
            if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
            (void)hipFree(ctx->d_geom);
            (void)hipFree(ctx->d_sph);
        }
        ctx->d_geom = g;
        ctx->d_sph = s;
        ctx->capacity = cap;
    }
    if (count > 0) {
        // Scan record: center + radius^2.  r*r is one IEEE f32 multiply, bit-identical to
        // the shader's `sphere.radius * sphere.radius` (wgsl:186).
        std::vector<float4> geom(count);
        for (uint32_t i = 0; i < count; ++i) {
            const rt_sphere& s = spheres[i];
            geom[i] = make_float4(s.position[0], s.position[1], s.position[2],
                                  s.radius * s.radius);
        }
        // Queued launches may still read the old scene: order the copies on the stream,
        // and wait for them so the host staging vectors can be released.
        hipError_t e = hipMemcpyAsync(ctx->d_geom, geom.data(), geom.size() * sizeof(float4),
                                      hipMemcpyHostToDevice, stream);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(sphere geometry)");
        // the sphere records as the reference uploads them (bytemuck, lib.rs:186)
        e = hipMemcpyAsync(ctx->d_sph, spheres, count * sizeof(rt_sphere),
                           hipMemcpyHostToDevice, stream);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(sphere records)");
        // the hit normal's one-step division by each distinct radius, checked on the device
        // against the IEEE division for every numerator significand (2^24 divisions per
        // radius); scenes with more than kRcpRadii distinct radii keep the two-step form.
        // (RT_NORMAL_RN=0 in the environment turns the Markstein normal off: a test switch)
        constexpr size_t kRcpRadii = 16;
        std::vector<float> radii(count);
        for (uint32_t i = 0; i < count; ++i) radii[i] = spheres[i].radius;
        std::sort(radii.begin(), radii.end(), [](float a, float b) {
            uint32_t x, y;
            std::memcpy(&x, &a, 4);
            std::memcpy(&y, &b, 4);
            return x < y;
        });
        radii.erase(std::unique(radii.begin(), radii.end(), [](float a, float b) {
                        return std::memcmp(&a, &b, 4) == 0;
                    }), radii.end());
        uint32_t bad = 1u;
        if (radii.size() <= kRcpRadii) {
            if (!ctx->d_flag) {
                e = hipMalloc(&ctx->d_flag, sizeof(uint32_t) * (1 + kRcpRadii));
                if (e != hipSuccess) return hip_fail(e, "hipMalloc(check flag)");
            }
            float* d_radii = reinterpret_cast<float*>(ctx->d_flag + 1);
            e = hipMemsetAsync(ctx->d_flag, 0, sizeof(uint32_t), stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(d_radii, radii.data(), radii.size() * sizeof(float),
                                   hipMemcpyHostToDevice, stream);
            if (e == hipSuccess)
                e = rtk::launch_rcp_check(d_radii, (uint32_t)radii.size(), ctx->d_flag, stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(&bad, ctx->d_flag, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   stream);
            if (e != hipSuccess) return hip_fail(e, "radius reciprocal check");
        }
        e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        const char* env = std::getenv("RT_NORMAL_RN");
        ctx->normal_rn = bad == 0u && !(env && env[0] == '0');
    }
    double bound = 0.0;
    bool radii_ok = true;
    for (uint32_t i = 0; i < count; ++i) {
        const double r = std::fabs((double)spheres[i].radius);
        const double b = norm3(spheres[i].position) + r;
        bound = std::isfinite(b) ? std::max(bound, b) : INFINITY;
        radii_ok = radii_ok && r >= 0x1p-20 && r <= 0x1p20;
    }
    ctx->scene_bound = bound;
    ctx->radii_ok = radii_ok;
    if (rt_status s = build_grid(ctx, spheres, count, stream)) return s;
    ctx->cached.assign(spheres, spheres + count);
    ctx->count = count;
    ctx->valid = true;
    return RT_OK;
}

void free_candidates(rt_ctx* ctx) {
    (void)hipFree(ctx->cand);
    ctx->cand = nullptr;
    ctx->cand_tiles = 0;
    ctx->cand_live = 0;
    ctx->cand_key.clear();
}

// Makes the per-tile candidate lists current for p's camera geometry, image, stripes and
// scene; rebuilds them (one small kernel) only when one of those changed.  The per-frame
// fields (random_seed, camera_has_moved, samples_per_pixel, max_depth) are not part of
// the key: the lists hold for every frame of a camera.
rt_status ensure_candidates(rt_ctx* ctx, rtk::TraceParams& p, hipStream_t stream) {
    struct Key {
        float center[3], vul[3], pdu[3], pdv[3], ddu[3], ddv[3], defocus;
        uint32_t w, h, first, step, bands;
        uint64_t scene;
    } key;
    std::memset(&key, 0, sizeof(key));
    std::memcpy(key.center, p.center, sizeof(key.center));
    std::memcpy(key.vul, p.vul, sizeof(key.vul));
    std::memcpy(key.pdu, p.pdu, sizeof(key.pdu));
    std::memcpy(key.pdv, p.pdv, sizeof(key.pdv));
    std::memcpy(key.ddu, p.ddu, sizeof(key.ddu));
    std::memcpy(key.ddv, p.ddv, sizeof(key.ddv));
    key.defocus = p.defocus_angle;
    key.w = p.width;
    key.h = p.height;
    key.first = p.band_first;
    key.step = p.band_step;
    key.bands = p.local_bands;
    key.scene = ctx->scene_gen;
    const unsigned char* kb = reinterpret_cast<const unsigned char*>(&key);
    const uint64_t tiles = (uint64_t)((p.width + 7u) >> 3) * p.local_bands;
    p.cand_k = rtk::kCandMax;
    if (ctx->cand_key.size() != sizeof(key) ||
        std::memcmp(ctx->cand_key.data(), kb, sizeof(key)) != 0) {
        if (tiles > ctx->cand_tiles) {
            if (ctx->cand_tiles) {
                hipError_t e = hipStreamSynchronize(stream);  // old lists may be in use
                if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
            }
            free_candidates(ctx);
            hipError_t e = hipMalloc(&ctx->cand, tiles * rtk::kCandStride * sizeof(float4));
            if (e != hipSuccess) {
                free_candidates(ctx);
                return hip_fail(e, "hipMalloc(candidate lists)");
            }
            ctx->cand_tiles = tiles;
        }
        hipError_t e = rtk::launch_candidates(p, ctx->cand, stream);
        if (e != hipSuccess) return hip_fail(e, "rt_candidates_kernel launch");
        ctx->cand_key.assign(kb, kb + sizeof(key));
        ctx->cand_gen++;
        ctx->cand_live = tiles;
    }
    p.cand = ctx->cand;
    return RT_OK;
}

// Cost-ordered tiles for the camera-ray-only instances: a fused launch of a candidate-list
// generation (same camera geometry, image, stripes and scene) records each tile's
// duration; the next launch of the generation first sorts the tiles by it
// (rtk::launch_tile_order, on the stream) and then starts the costliest tiles first so
// that the cheap ones fill the tail.  The sort runs only when a generation is reused, so a
// camera that moves every call never pays for it.  Only the workgroup -> tile assignment
// changes, never a pixel's result.
rt_status plan_tile_order(rt_ctx* ctx, rtk::TraceParams& p, int kernel, hipStream_t stream) {
    p.tile_order = nullptr;
    p.tile_cost = nullptr;
    // (single-frame launches keep raster order: their accumulator traffic is a large part
    // of the frame, and scattered tiles cost more in HBM than the tail they save)
    const bool bounce = kernel == rtk::kTraceBounce;
    if (!(rtk::trace_ordered(kernel) || bounce) || ctx->tile_order_mode == RT_TILE_ORDER_OFF ||
        p.cand_k == 0 || p.frames < 2)
        return RT_OK;
    // scheduling units: 8x8 tiles, the compacting bounce instance's workgroups of
    // kBounceWaves tiles or rt_tpair_kernel's tile pairs (costs measured in another unit are
    // discarded)
    const uint32_t group = (bounce && p.compact == 1u)         ? rtk::kBounceWaves
                           : (kernel == rtk::kTraceListQuad2 ||
                              kernel == rtk::kTraceListPair2) ? 2u
                                                            : 1u;
    if (ctx->cost_group != group) {
        ctx->cost_gen = ctx->order_gen = ~0ull;
        ctx->cost_group = group;
    }
    const uint64_t gen = ctx->cand_gen;
    const uint32_t tiles_x0 = (p.width + 7u) >> 3;
    const uint32_t tiles_x = (tiles_x0 + group - 1u) / group;
    const uint64_t tiles = (uint64_t)tiles_x * p.local_bands;
    if (tiles > ctx->order_tiles) {
        if (ctx->order_tiles) {
            hipError_t e = hipStreamSynchronize(stream);   // old order may be in use
            if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        }
        (void)hipFree(ctx->tile_cost);
        (void)hipFree(ctx->tile_order);
        ctx->tile_cost = ctx->tile_order = nullptr;
        ctx->order_tiles = 0;
        ctx->cost_gen = ctx->order_gen = ~0ull;
        hipError_t e = hipMalloc(&ctx->tile_cost, tiles * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc(&ctx->tile_order, tiles * sizeof(uint32_t));
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(tile order)");
        ctx->order_tiles = tiles;
    }
    // the order from the newest measurement of this generation
    if (ctx->cost_gen == gen && (ctx->order_gen != gen || ctx->order_frames < ctx->cost_frames)) {
        hipError_t e = rtk::launch_tile_order(ctx->tile_cost, ctx->tile_order,
                                              (uint32_t)tiles, tiles_x, stream);
        if (e != hipSuccess) return hip_fail(e, "rt_tile_order_kernel launch");
        ctx->order_gen = gen;
        ctx->order_frames = ctx->cost_frames;
    }
    const bool have = ctx->order_gen == gen;
    if (have) p.tile_order = ctx->tile_order;
    // A launch of a few frames measures mostly start-up and placement noise: launches keep
    // re-measuring (in the current order) until one of kOrderFrames frames or more has.
    constexpr uint32_t kOrderFrames = 16;
    if (have && ctx->order_frames >= std::min(kOrderFrames, p.frames)) return RT_OK;
    p.tile_cost = ctx->tile_cost;
    return RT_OK;
}

// Dispatch order of one-frame launches (rt_single_kernel): the workgroups of the current
// candidate generation by decreasing candidate-list load, costliest first (scheduling only;
// rtk::launch_wg_order).  Built on the second launch of a generation (a camera that moves
// every frame never pays for it); rt_set_tile_order(OFF) keeps raster order.
rt_status plan_wg_order(rt_ctx* ctx, rtk::TraceParams& p, int kernel, hipStream_t stream) {
    const uint32_t parts = p.parts > 1u ? p.parts : 1u;
    p.wg_order = nullptr;
    if ((kernel != rtk::kTraceSingle && kernel != rtk::kTraceSingleOne) || p.cand_k == 0 ||
        p.local_bands < 2 || ctx->tile_order_mode == RT_TILE_ORDER_OFF)
        return RT_OK;
    const uint64_t gen = ctx->cand_gen;
    if (ctx->band_gen != gen) {
        if (ctx->band_seen_gen != gen) {        // first launch of this generation
            ctx->band_seen_gen = gen;
            return RT_OK;
        }
        ctx->band_gen = gen;
        ctx->wg_pix = 0;
        ctx->wg_parts = 0;
    }
    const uint32_t pix = kernel == rtk::kTraceSingle ? rtk::single_pix() : 1u;
    const uint32_t per = rtk::single_wg_tiles(pix);
    const uint64_t units = (uint64_t)((((p.width + 7u) >> 3) + per - 1u) / per) * p.local_bands;
    if (units > ctx->wg_cap) {
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        (void)hipFree(ctx->wg_buf);
        ctx->wg_buf = nullptr;
        ctx->wg_cap = 0;
        e = hipMalloc(&ctx->wg_buf, (2 * units + 1) * sizeof(uint32_t));
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(workgroup order)");
        ctx->wg_cap = units;
        ctx->wg_pix = 0;
    }
    if (ctx->wg_pix != pix || ctx->wg_parts != parts) {
        hipError_t e = rtk::launch_wg_order(p.cand, (p.width + 7u) >> 3, p.local_bands, pix,
                                            ctx->wg_buf, ctx->wg_buf + units, stream, parts);
        if (e != hipSuccess) return hip_fail(e, "workgroup order launch");
        ctx->wg_pix = pix;
        ctx->wg_parts = parts;
        ctx->wg_builds++;
    }
    p.wg_order = ctx->wg_buf + units;
    return RT_OK;
}

// Split bounce launches (rt_kernels.hip kBounceSplit; RT_PATHS_SPLIT, or AUTO for small
// launches): each tile's frames in S chunks traced by separate waves.  A share of a few
// waves per SIMD in per-wave mode ends with SIMDs idle behind its costliest tiles' 64-frame
// chains (an 8-rank K5 share's longest waves last 0.91-1.0 of the launch, 4.75
// waves resident per SIMD on average); S times as many, S times shorter waves keep them
// busy to the end.  S = 4 up to kSplit4MaxTiles tiles per launch, 2 up to kSplit2MaxTiles,
// else 1 (per wave; RT_PATHS_SPLIT forces at least 2); never more chunks than frames.
// RT_BOUNCE_SPLIT (environment, diagnostic) overrides S.  With a measured tile order only the
// costliest tiles split (the unit order below).  Measured (tools/k5_ab.py, 64-frame K5
// launches, the modes interleaved launch by launch): every tile split, first build
// (profiles/r04/k5_ab_r04e.jsonl): 8-rank share per wave 4 635 µs, S = 2 4 422, S = 4 4 821,
// S = 8 4 970; 4-rank per wave 8 010, S = 2 8 388 — the chunks' hand-off traffic, merges and
// extra wave starts cost more than the shorter tail saves.  The unit order
// (profiles/r04/r04l_k5_unit_order.jsonl, 7 launches each): 8-rank share per wave 4 593, every
// tile in 2 chunks 4 447, the unit order with S = 4 and alpha 0.25 4 253 (0.879 of the 1-GPU
// per-wave rate); 4-rank per wave 7 896 against 8 008, whole image 29 911 against 30 185 — so
// AUTO splits (S = 4, unit order) shares of at most 20 000 tiles and runs larger ones per wave.
// Against S = 8 and other alphas (profiles/r04/r04e2_k5_chunks_alpha.jsonl, 8-rank share):
// AUTO 4 248, S = 8 alpha 0.25 / 0.5 4 318 / 4 391, S = 4 alpha 0.125 / 0.5 4 686 / 4 264.
#ifndef RT_SPLIT4_MAX_TILES
#define RT_SPLIT4_MAX_TILES 20000
#endif
#ifndef RT_SPLIT2_MAX_TILES
#define RT_SPLIT2_MAX_TILES 20000
#endif
constexpr uint64_t kSplit4MaxTiles = RT_SPLIT4_MAX_TILES, kSplit2MaxTiles = RT_SPLIT2_MAX_TILES;
// Only the costliest tiles split: the first ceil(tiles * kSplitFrac) slots of the cost order
// (a launch without an order: its first slots in raster order).  RT_SPLIT_FRAC (environment,
// diagnostic) overrides the fraction.
#ifndef RT_SPLIT_FRAC
#define RT_SPLIT_FRAC 1.0
#endif
// alpha: a tile splits when its recorded cost exceeds alpha times the launch's ideal span
// (the sum of all costs over the device's resident waves); 0.25 measured best with S = 4
#ifndef RT_SPLIT_ALPHA
#define RT_SPLIT_ALPHA 0.25
#endif
// The bounce instance's table of scatter random numbers (TraceParams::hint_rs_dev) for the
// hinted frames of a launch: the context's buffer, filled on the stream by launch_bounce.
rt_status plan_hint_rs(rt_ctx* ctx, rtk::TraceParams& p, int kernel) {
    p.hint_rs_dev = nullptr;
    p.hint_rs_dev_frames = 0;
    if (kernel != rtk::kTraceBounce || p.hint_acc_frames == 0 || p.depth == 0 ||
        p.depth > rtk::kHintRsDepth)
        return RT_OK;
    if (!ctx->d_hint_rs) {
        const hipError_t e = hipMalloc(&ctx->d_hint_rs, sizeof(float4) * rtk::kHintFrames *
                                                            rtk::kHintRsDepth);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(hint table)");
    }
    p.hint_rs_dev = ctx->d_hint_rs;
    p.hint_rs_dev_frames = p.hint_acc_frames;
    return RT_OK;
}

rt_status plan_split(rt_ctx* ctx, rtk::TraceParams& p, int kernel, hipStream_t stream) {
    p.split = 1;
    p.split_tiles = 0;
    p.unit_order = nullptr;
    p.unit_count = nullptr;
    p.split_col = nullptr;
    p.split_cnt = nullptr;
    const int mode = ctx->path_compaction;
    if (kernel != rtk::kTraceBounce || (mode != RT_PATHS_AUTO && mode != RT_PATHS_SPLIT))
        return RT_OK;
    const uint64_t tiles = (uint64_t)((p.width + 7u) >> 3) * p.local_bands;
    uint32_t S = tiles <= kSplit4MaxTiles ? 4u : tiles <= kSplit2MaxTiles ? 2u : 1u;
    if (mode == RT_PATHS_SPLIT) S = std::max(S, 2u);
    if (const char* e = std::getenv("RT_BOUNCE_SPLIT")) S = (uint32_t)std::max(1L, std::atol(e));
    S = std::min(std::min(S, p.frames), 8u);   // a unit-order entry holds chunks 0-7
    // a power of two: rt_unit_order_kernel moves a split tile's cost bucket by 4·log2 S
    // places (cost / S), and launches of 3, 5, 6 or 7 frames would otherwise give S = 3..7
    while (S & (S - 1u)) S &= S - 1u;
    // AUTO splits only with a measured order (the unit order below): a launch without one runs
    // per wave, so the costs it records are whole tiles', not a chunk's scaled by S
    if (mode == RT_PATHS_AUTO && !p.tile_order && !std::getenv("RT_SPLIT_FRAC")) S = 1u;
    if (S <= 1u || tiles == 0) {
        p.compact = 0u;
        return RT_OK;
    }
    const uint64_t bytes = tiles * p.frames * 1024ull;
    if (bytes > ctx->split_col_bytes || tiles > ctx->split_cnt_tiles) {
        hipError_t e = hipStreamSynchronize(stream);    // the old buffers may be in use
        if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        if (bytes > ctx->split_col_bytes) {
            (void)hipFree(ctx->split_col);
            ctx->split_col = nullptr;
            ctx->split_col_bytes = 0;
            e = hipMalloc(&ctx->split_col, bytes);
            if (e != hipSuccess) return hip_fail(e, "hipMalloc(split colours)");
            ctx->split_col_bytes = bytes;
        }
        if (tiles > ctx->split_cnt_tiles) {
            (void)hipFree(ctx->split_cnt);
            ctx->split_cnt = nullptr;
            ctx->split_cnt_tiles = 0;
            e = hipMalloc(&ctx->split_cnt, tiles * sizeof(uint32_t));
            // (zero once: every launch leaves the arrival counters at zero)
            if (e == hipSuccess) e = hipMemsetAsync(ctx->split_cnt, 0, tiles * sizeof(uint32_t), stream);
            if (e != hipSuccess) return hip_fail(e, "hipMalloc(split counters)");
            ctx->split_cnt_tiles = tiles;
        }
    }
    // With a measured tile order: the unit order (longest-processing-time-first over the
    // units; tiles above alpha times the launch's ideal span split).  RT_SPLIT_FRAC (the
    // first fraction of the tile order splits, no unit order) and RT_SPLIT_ALPHA: diagnostic.
    const char* frac_env = std::getenv("RT_SPLIT_FRAC");
    if (p.tile_order && !frac_env && p.local_bands < 4096u && ((p.width + 7u) >> 3) < 65536u) {
        double alpha = RT_SPLIT_ALPHA;
        if (const char* e = std::getenv("RT_SPLIT_ALPHA")) alpha = std::atof(e);
        const uint64_t cap = tiles * S;
        if (cap + 1 > ctx->unit_cap) {
            hipError_t e = hipStreamSynchronize(stream);   // the old order may be in use
            if (e == hipSuccess) {
                (void)hipFree(ctx->unit_order);
                ctx->unit_order = nullptr;
                ctx->unit_cap = 0;
                e = hipMalloc(&ctx->unit_order, (cap + 1) * sizeof(uint32_t));
            }
            if (e != hipSuccess) return hip_fail(e, "hipMalloc(unit order)");
            ctx->unit_cap = cap + 1;
            ctx->unit_key[0] = ~0ull;
        }
        // (resident waves of the launch: every SIMD of the context's device at 8 waves)
        if (ctx->cus == 0) {
            int n = 0;
            if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, ctx->device) !=
                    hipSuccess || n <= 0)
                n = 256;
            ctx->cus = n;
        }
        const int cus = ctx->cus;
        const float k_thr = (float)(alpha / (cus * 4.0 * 8.0));
        uint32_t kbits;
        std::memcpy(&kbits, &k_thr, 4);
        const uint64_t key[5] = {ctx->order_gen, ctx->order_frames, tiles, S, kbits};
        if (!std::equal(key, key + 5, ctx->unit_key)) {
            hipError_t e = rtk::launch_unit_order(ctx->tile_cost, ctx->unit_order,
                                                  ctx->unit_order + cap, (uint32_t)tiles,
                                                  (p.width + 7u) >> 3, S, k_thr, stream);
            if (e != hipSuccess) return hip_fail(e, "rt_unit_order_kernel launch");
            std::copy(key, key + 5, ctx->unit_key);
        }
        p.compact = 3u;
        p.split = S;
        p.split_tiles = 0;
        p.split_col = ctx->split_col;
        p.split_cnt = ctx->split_cnt;
        p.unit_order = ctx->unit_order;
        p.unit_count = ctx->unit_order + cap;
        return RT_OK;
    }
    double frac = RT_SPLIT_FRAC;
    if (frac_env) frac = std::atof(frac_env);
    const uint64_t st = std::min<uint64_t>(tiles, (uint64_t)std::ceil(tiles * std::max(0.0, frac)));
    if (st == 0) {
        p.compact = 0u;
        return RT_OK;
    }
    p.compact = 3u;
    p.split = S;
    p.split_tiles = (uint32_t)st;
    p.split_col = ctx->split_col;
    p.split_cnt = ctx->split_cnt;
    return RT_OK;
}

// After a launch that recorded tile costs.
void finish_tile_order(rt_ctx* ctx, const rtk::TraceParams& p) {
    if (!p.tile_cost) return;
    ctx->cost_gen = ctx->cand_gen;
    ctx->cost_frames = p.frames;
    const uint32_t key[6] = {p.width, p.height, p.band_first, p.band_step, p.local_bands,
                             ctx->cost_group};
    std::copy(key, key + 6, ctx->cost_key);
    ctx->cost_key_ok = true;
}

// Per-column / per-row halves of the pixel-invariant seed hash (wgsl:309-310), built on
// the host once per image size: one buffer, hash(x*73) for x < rtk::hy_offset(w), then
// hash(y*51) for y < h (the trace kernel derives the row table from the column table's
// pointer and the width: one preloaded pointer for both).
rt_status ensure_hash_tables(rt_ctx* ctx, uint32_t w, uint32_t h, hipStream_t stream) {
    const uint32_t xpad = rtk::hy_offset(w);
    if (ctx->d_hx && ctx->hx_len == xpad && ctx->hy_len >= h) return RT_OK;
    const uint32_t ylen = std::max(h, ctx->hx_len == xpad ? ctx->hy_len : 0u);
    std::vector<uint32_t> v((size_t)xpad + ylen);
    for (uint32_t i = 0; i < xpad; ++i) v[i] = rtd::hash(i * 73u);
    for (uint32_t i = 0; i < ylen; ++i) v[xpad + i] = rtd::hash(i * 51u);
    uint32_t* d = nullptr;
    hipError_t e = hipMalloc(&d, v.size() * sizeof(uint32_t));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(hash table)");
    e = hipMemcpyAsync(d, v.data(), v.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);  // also retires old readers
    if (e != hipSuccess) {
        (void)hipFree(d);
        return hip_fail(e, "hipMemcpyAsync(hash table)");
    }
    (void)hipFree(ctx->d_hx);
    ctx->d_hx = d;
    ctx->hx_len = xpad;
    ctx->hy_len = ylen;
    return RT_OK;
}

// ---- sample-count hints (TraceParams::hint_n) ------------------------------------------
bool lookup_count(const rt_ctx* ctx, const void* image, const rtk::TraceParams& p,
                  uint32_t& n) {
    for (const rt_ctx::CountRecord& r : ctx->counts)
        if (r.image == image && r.w == p.width && r.h == p.height && r.first == p.band_first &&
            r.step == p.band_step && r.bands == p.local_bands) {
            n = r.n;
            return true;
        }
    return false;
}

void forget_count(rt_ctx* ctx, const void* image) {
    for (size_t i = 0; i < ctx->counts.size(); ++i)
        if (ctx->counts[i].image == image) {
            ctx->counts.erase(ctx->counts.begin() + (long)i);
            return;
        }
}

void record_count(rt_ctx* ctx, const void* image, const rtk::TraceParams& p, uint32_t n) {
    forget_count(ctx, image);
    if (ctx->counts.size() >= 16) ctx->counts.erase(ctx->counts.begin());
    ctx->counts.push_back({image, p.width, p.height, p.band_first, p.band_step, p.local_bands, n});
}

// The count a pixel holds after frame f of the kernel's loop, given the count before it
// (wgsl:352-362, including the f32 round trip of the stored count).
uint32_t next_count(uint32_t n, uint32_t spp) {
    return host_f2u((float)(n < spp ? n + 1u : n));
}

// Fills p.hint_* for a launch whose input pixels all hold count n_in (frame 0 of a reset
// launch: 0) and returns the count every pixel holds after the launch.
uint32_t fill_hint(rtk::TraceParams& p, uint32_t n_in) {
    const uint32_t spp = p.spp, depth = p.depth;
    const uint32_t af = std::min<uint32_t>(p.frames, rtk::kHintFrames);
    uint32_t hf = af;
    if (depth > 0) hf = std::min<uint32_t>(hf, rtk::kHintEntries / depth);
    p.hint_frames = hf;
    p.hint_acc_frames = af;
    uint32_t n = n_in;
    for (uint32_t f = 0; f < p.frames; ++f) {
        if (f < af) {
            p.hint_n[f] = n;
            // RN32(1 / f32(n + 1)) (exact integer for n + 1 <= 2^24, where the kernels use it)
            p.hint_rcp[f] = 1.0f / (float)(n + 1u);
            p.hint_cnt[f] = (float)(n < spp ? n + 1u : n);
        }
        if (f < hf) {
            const uint32_t B = p.seed_b[f];
            for (uint32_t i = 0; i < depth; ++i) {
                // wgsl:268 with seed + 1 = n + B + 2 (wgsl:353, 358)
                const uint32_t sb = rtd::hash(n + B + 2u + i * 1000u);
                const float r_sb = rtd::rf(sb);
                const rtd::v3 u = rtd::random_unit_vector(r_sb, sb);
                p.hint_rs[f * depth + i] = make_float4(r_sb, u.x, u.y, u.z);
            }
        }
        n = next_count(n, spp);
    }
    return n;
}

// Sets the hint of one launch from what the context knows about `in` and records the
// count of `out` afterwards (or forgets it when unknown).
void plan_hint(rt_ctx* ctx, rtk::TraceParams& p, const void* in, const void* out) {
    uint32_t n_in = 0;
    const bool known = p.reset_first || lookup_count(ctx, in, p, n_in);
    if (!known) {
        p.hint_frames = 0;
        p.hint_acc_frames = 0;
        forget_count(ctx, out);
        return;
    }
    record_count(ctx, out, p, fill_hint(p, p.reset_first ? 0u : n_in));
}

void fill_camera(rtk::TraceParams& p, const rt_scene_camera& c) {
    for (int i = 0; i < 3; ++i) {
        p.center[i] = c.center[i];
        p.vul[i] = c.viewport_upper_left[i];
        p.pdu[i] = c.pixel_delta_u[i];
        p.pdv[i] = c.pixel_delta_v[i];
        p.ddu[i] = c.defocus_disk_u[i];
        p.ddv[i] = c.defocus_disk_v[i];
    }
    p.defocus_angle = c.defocus_angle;
    p.depth = host_f2u(c.max_depth);
    p.spp = host_f2u(c.samples_per_pixel);
}

// The round-robin stripes of rank / nranks as a band set (band b -> rank b mod nranks).
rt_band_set stripe_set(uint32_t h, uint32_t rank, uint32_t nranks) {
    const uint32_t bands = (h + RT_STRIPE_ROWS - 1) / RT_STRIPE_ROWS;
    return {rank, nranks, bands > rank ? (bands - rank + nranks - 1) / nranks : 0u};
}

// A band set the kernels can run: inside the image, step >= 1, and (for two or more bands)
// first and step within the packed stripe map's 16 / 15 bits (rtk::pack_bands).
rt_status check_band_set(uint32_t h, const rt_band_set& bs) {
    const uint32_t bands = (h + RT_STRIPE_ROWS - 1) / RT_STRIPE_ROWS;
    if (bs.step == 0) return fail(RT_ERR_INVALID_ARGUMENT, "band set step is 0");
    if (bs.count == 0) return RT_OK;
    if (bs.first >= bands || (uint64_t)bs.first + (uint64_t)(bs.count - 1u) * bs.step >= bands)
        return fail(RT_ERR_INVALID_ARGUMENT, "band set reaches past the image");
    if (bs.first > 0xFFFFu || (bs.count >= 2u && bs.step >= 0x7FFFu))
        return fail(RT_ERR_INVALID_ARGUMENT, "band set first / step out of range");
    return RT_OK;
}

// Common setup of every trace launch: argument checks, scene upload, kernel parameters
// (camera, stripe map, scan-mode data such as the candidate lists).
rt_status prepare(rt_ctx* ctx, const void* in, const void* out, uint32_t w, uint32_t h,
                  const rt_band_set& bs, const rt_scene_camera* cam,
                  const rt_sphere* spheres, uint32_t count, const float* seeds,
                  hipStream_t stream, rtk::TraceParams& p) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!in || !out || !cam) return fail(RT_ERR_INVALID_ARGUMENT, "NULL image or camera");
    if (rt_status s = check_image(w, h)) return s;
    if (rt_status s = check_band_set(h, bs)) return s;
    if (!seeds) return fail(RT_ERR_INVALID_ARGUMENT, "random_seeds is NULL");
    if (rt_status s = upload_spheres(ctx, spheres, count, stream)) return s;

    std::memset(&p, 0, sizeof(p));
    p.geom = ctx->d_geom;
    p.sph = ctx->d_sph;
    p.width = w;
    p.height = h;
    p.count = count;
    p.normal_rn = ctx->normal_rn ? 1u : 0u;
    p.roots_fast = ctx->scene_bound <= 0x1p40 ? 1u : 0u;
    p.band_first = bs.first;
    p.band_step = bs.step;
    p.local_bands = bs.count;
    fill_camera(p, *cam);
    // bounce instance mode (rt_kernels.hip rt_bounce_kernel: 0 per wave, 1 compact, 2 pairs)
    p.compact = ctx->path_compaction == RT_PATHS_COMPACT ? 1u
                : ctx->path_compaction == RT_PATHS_PAIR  ? 2u
                                                         : 0u;
    if (rt_status s = ensure_hash_tables(ctx, w, h, stream)) return s;
    p.hx = ctx->d_hx;
    p.hy = ctx->d_hx + rtk::hy_offset(w);
    if (ctx->scan_mode == RT_SCAN_CULLED) {
        // Camera rays use the per-tile candidate lists; the LDS copy of the records only
        // serves the per-wave cone culling of bounce rays, so it is skipped at depth <= 1
        // (tiles without a list then read the records from L2).
        const uint32_t padded = (count + 63u) & ~63u;   // <= count + 63 < count + kScanPad
        const bool bounces = cam->max_depth >= 2.0f;
        // (the per-wave bounce instance runs one-wave workgroups: no LDS copy, which each
        // of them would stage)
        p.lds_records = (bounces && padded <= rtk::kLdsMaxRecords &&
                         ctx->path_compaction == RT_PATHS_COMPACT)
                            ? padded
                            : 0u;
        if (rt_status s = ensure_candidates(ctx, p, stream)) return s;
        if (bounces && ctx->grid.nx) {
            const rt_ctx::Grid& g = ctx->grid;
            const unsigned char* base = static_cast<const unsigned char*>(ctx->d_grid);
            const size_t cells = (size_t)g.nx * g.nz;
            p.grid_cells = reinterpret_cast<const uint2*>(base);
            const size_t geom_off = (cells * 8 + 15) & ~(size_t)15;     // as build_grid
            p.grid_geom = reinterpret_cast<const float4*>(base + geom_off);
            p.grid_items = reinterpret_cast<const uint32_t*>(base + geom_off + g.items * 16ull);
            p.grid_big = p.grid_items + g.items;
            p.grid_nx = g.nx;
            p.grid_nz = g.nz;
            p.grid_nbig = g.nbig;
            p.grid_x0 = g.x0;
            p.grid_z0 = g.z0;
            p.grid_s = g.s;
            p.grid_inv_s = g.inv_s;
            p.grid_ylo = g.ylo;
            p.grid_yhi = g.yhi;
            p.grid_cx = g.cx;
            p.grid_cy = g.cy;
            p.grid_cz = g.cz;
            p.grid_reach = g.reach;
            p.grid_m = g.m;
            p.grid_e = g.e;
        }
    }
    return RT_OK;
}

// Concurrent parts of a one-frame update (rt_set_update_queues).  AUTO by the launch's
// tiles (profiles/r03/r03e_ab_queues.log, r03/r03e_rank_sim_k3_q*.jsonl; µs per K3 update at 1 / 2
// / 3 / 4 parts: whole image 22.7 / 19.6 / 19.6 / 19.0, K2 15.9 / 13.6 / 13.5 / 13.5; a
// 2-rank share 12.5 / 11.4 / 11.5; 4-rank 7.8 / 7.5 / 9.7; 8-rank 5.9 / 7.9 / 10.9): each
// part costs the host one more launch (2.7-4.4 µs each on the boxes measured,
// profiles/r03/r03g_launch_rate.jsonl, r03/r03h_launch_rate.jsonl), which small shares cannot hide,
// and a slow host turns 4 parts into a host-bound chain (the driver's 20-step command:
// 72-77 G rays/s at 4 parts, 87-90 at 2, 81-85 at 1, profiles/r03/r03h_bench_driver_q*.json).
constexpr uint64_t kQueues4MinTiles = ~0ull, kQueues2MinTiles = 12000;
uint32_t update_parts(const rt_ctx* ctx, const rtk::TraceParams& p, int kernel) {
    if ((kernel != rtk::kTraceSingle && kernel != rtk::kTraceSingleOne) || p.frames != 1u)
        return 1u;
    uint32_t q = ctx->update_queues;
    if (q == 0) {
        const uint64_t tiles = (uint64_t)((p.width + 7u) >> 3) * p.local_bands;
        q = tiles >= kQueues4MinTiles ? 4u : tiles >= kQueues2MinTiles ? 2u : 1u;
    }
    return std::max(1u, std::min(q, p.local_bands));
}

// Parts of a one-frame update submitted as AQL packets: a packet costs the host ≈0.25 µs
// (profiles/r03/r03r_aql_probe.txt), so the host never bounds the parts; but four HSA queues
// beside HIP's own measured 38.7 µs per K3 update against 20.4 with two
// (profiles/r03/r03s_ab_aql_nckarg.log): AUTO takes 2 from 2 000 tiles, else 1
// (rt_set_update_queues overrides).
constexpr uint64_t kAqlQueues4MinTiles = ~0ull, kAqlQueues2MinTiles = 2000;
uint32_t update_parts_aql(const rt_ctx* ctx, const rtk::TraceParams& p) {
    uint32_t q = ctx->update_queues;
    if (q == 0) {
        const uint64_t tiles = (uint64_t)((p.width + 7u) >> 3) * p.local_bands;
        q = tiles >= kAqlQueues4MinTiles ? 4u : tiles >= kAqlQueues2MinTiles ? 2u : 1u;
    }
    return std::max(1u, std::min(q, p.local_bands));
}

// The context's extra streams and fork/join events (created on first use, on ctx->device).
rt_status ensure_aux_streams(rt_ctx* ctx, uint32_t n) {
    if (!ctx->fork_ev) {
        hipError_t e = hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming);
        if (e != hipSuccess) return hip_fail(e, "hipEventCreateWithFlags");
    }
    for (uint32_t k = 0; k < n; ++k) {
        if (!ctx->aux[k]) {
            hipError_t e = hipStreamCreateWithFlags(&ctx->aux[k], hipStreamNonBlocking);
            if (e != hipSuccess) return hip_fail(e, "hipStreamCreateWithFlags");
        }
        if (!ctx->join_ev[k]) {
            hipError_t e = hipEventCreateWithFlags(&ctx->join_ev[k], hipEventDisableTiming);
            if (e != hipSuccess) return hip_fail(e, "hipEventCreateWithFlags");
        }
    }
    return RT_OK;
}


// `stream` waits for everything issued on aux[0..n) so far
rt_status join_aux(rt_ctx* ctx, uint32_t n, hipStream_t stream) {
    hipError_t e = hipSuccess;
    for (uint32_t k = 0; e == hipSuccess && k < n; ++k) {
        e = hipEventRecord(ctx->join_ev[k], ctx->aux[k]);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, ctx->join_ev[k], 0);
    }
    return e == hipSuccess ? RT_OK : hip_fail(e, "join (hipEventRecord / hipStreamWaitEvent)");
}

void note_launch(rt_ctx* ctx, const rtk::TraceParams& p, int kernel, uint32_t frames,
                 uint32_t parts = 1u, bool aql = false) {
    ctx->last.launches += parts;
    ctx->last.queues = parts;
    ctx->last.submit = aql ? RT_SUBMIT_AQL : RT_SUBMIT_HIP;
    ctx->last.frames += frames;
    ctx->last.max_frames_per_launch = std::max(ctx->last.max_frames_per_launch, frames);
    ctx->last.normal_rn = p.normal_rn;
    ctx->last.kernel = kernel != rtk::kTraceBounce ? kernel
                       : p.compact == 3u             ? RT_KERNEL_BOUNCE_SPLIT
                                                     : RT_KERNEL_BOUNCE + (int)p.compact;
}

// A chain failure (a go wait that gave up, so a segment's frames were dropped; a queue
// error; a segment that did not complete in time) is returned once, by the context's next
// call (rt_update_frames, rt_destroy, rt_update_submit_status); the context runs HIP launches
// from then on.  No synchronisation: the flags live in host memory.
rt_status chain_report(rt_ctx* ctx) {
    if (!ctx->chain || ctx->chain_reported || !rtc::chain_failed(ctx->chain)) return RT_OK;
    ctx->chain_reported = true;
    const char* why = "";
    (void)rtc::chain_ok(ctx->chain, &why);
    return fail(RT_ERR_HIP, std::string("AQL submission failed earlier (") + why +
                                "); the context runs HIP launches from now on");
}

// The context's AQL chain if one-frame updates go through it (rt_set_update_submit AQL, or
// AUTO inside [kAqlAutoMinTiles, kAqlAutoMaxTiles) tiles — an empty range since round 4:
// AQL submission is opt-in): created on first use; AQL fails the call with the reason when
// the machine does not offer it, AUTO falls back to HIP launches, and after a chain failure
// every mode runs HIP launches.  Round 3 measured AQL faster only on mid-sized rank shares
// of per-dispatch updates (a 4-rank K3 share 6.76 against 7.54-7.68 µs per update,
// profiles/r03/r03zd_rank_sim_*.jsonl; whole images and 2-rank shares alike either way, 8-rank
// shares slower); rank shares now run fused frame chains in one launch instead
// (rt_set_frame_images), and no multi-GPU record of AQL submission exists.
#ifndef RT_AQL_AUTO_MIN_TILES
#define RT_AQL_AUTO_MIN_TILES 0
#endif
#ifndef RT_AQL_AUTO_MAX_TILES
#define RT_AQL_AUTO_MAX_TILES 0
#endif
constexpr uint64_t kAqlAutoMinTiles = RT_AQL_AUTO_MIN_TILES,
                   kAqlAutoMaxTiles = RT_AQL_AUTO_MAX_TILES;
rt_status usable_chain(rt_ctx* ctx, const rtk::TraceParams& p, rtc::Chain** out) {
    *out = nullptr;
    if (ctx->update_submit == RT_SUBMIT_HIP || ctx->chain_reported) return RT_OK;
    if (ctx->update_submit == RT_SUBMIT_AUTO) {
        const uint64_t tiles = (uint64_t)((p.width + 7u) >> 3) * p.local_bands;
        if (tiles < kAqlAutoMinTiles || tiles >= kAqlAutoMaxTiles) return RT_OK;
    }
    const bool aql = ctx->update_submit == RT_SUBMIT_AQL;
    if (!ctx->chain_tried) {
        ctx->chain_tried = true;
        rt_status st = RT_OK;
        ctx->chain = rtc::chain_create(ctx->device, &st);
        // (AUTO: a chain that could not be set up leaves the call on HIP launches)
        if (st != RT_OK && aql) return st;
    }
    const char* why = "";
    // AUTO also needs the queues of its parts up front: no failure once frames are packed
    if (rtc::chain_ok(ctx->chain, &why) && (aql || rtc::chain_queues(ctx->chain, 2u))) {
        *out = ctx->chain;
        return RT_OK;
    }
    if (aql) return fail(RT_ERR_HIP, std::string("AQL submission unavailable: ") + why);
    return RT_OK;
}

// Whether plan_wg_order would issue work on the stream or reallocate for this launch (an
// open AQL segment still reads the current order: it is closed first).
bool wg_order_pending(const rt_ctx* ctx, const rtk::TraceParams& p, int kernel) {
    const uint32_t parts = p.parts > 1u ? p.parts : 1u;
    if ((kernel != rtk::kTraceSingle && kernel != rtk::kTraceSingleOne) || p.cand_k == 0 ||
        p.local_bands < 2 || ctx->tile_order_mode == RT_TILE_ORDER_OFF)
        return false;
    const uint64_t gen = ctx->cand_gen;
    if (ctx->band_gen != gen) return ctx->band_seen_gen == gen;   // builds on this launch
    const uint32_t pix = kernel == rtk::kTraceSingle ? rtk::single_pix() : 1u;
    const uint32_t per = rtk::single_wg_tiles(pix);
    const uint64_t units = (uint64_t)((((p.width + 7u) >> 3) + per - 1u) / per) * p.local_bands;
    return units > ctx->wg_cap || ctx->wg_pix != pix || ctx->wg_parts != parts;
}

// Shared body of rt_update / rt_render / rt_render_stripes: `frames` accumulated in
// launches of up to kMaxFramesPerLaunch frames each.
rt_status trace(rt_ctx* ctx, const float* in, float* out, uint32_t w, uint32_t h,
                uint32_t rank, uint32_t nranks, const rt_scene_camera* cam,
                const rt_sphere* spheres, uint32_t count, uint32_t frames,
                const float* seeds, void* stream_v) {
    if (frames == 0) return ctx ? RT_OK : fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipStream_t stream = static_cast<hipStream_t>(stream_v);
    if (nranks == 0 || rank >= nranks) return fail(RT_ERR_INVALID_ARGUMENT, "bad rank/nranks");
    rtk::TraceParams p;
    if (rt_status s = prepare(ctx, in, out, w, h, stripe_set(h, rank, nranks), cam, spheres,
                              count, seeds, stream, p))
        return s;
    const float4* src = reinterpret_cast<const float4*>(in);
    float4* dst = reinterpret_cast<float4*>(out);
    ctx->last = {0, 0, 0, -1, 0, 0, 0};
    for (uint32_t f0 = 0; f0 < frames; f0 += rtk::kMaxFramesPerLaunch) {
        const uint32_t nf = std::min<uint32_t>(frames - f0, rtk::kMaxFramesPerLaunch);
        p.in = src;
        p.out = dst;
        p.frames = nf;
        p.reset_first = (f0 == 0 && cam->camera_has_moved > 0.5f) ? 1u : 0u;
        for (uint32_t f = 0; f < nf; ++f) p.seed_b[f] = host_f2u(seeds[f0 + f] * 4294967296.0f);
        plan_hint(ctx, p, src, dst);
        const int kernel = single_or(ctx, p, trace_kernel_for(ctx, p));
        if (rt_status s = plan_tile_order(ctx, p, kernel, stream)) return s;
        if (rt_status s = plan_wg_order(ctx, p, kernel, stream)) return s;
        if (rt_status s = plan_split(ctx, p, kernel, stream)) return s;
        if (rt_status s = plan_hint_rs(ctx, p, kernel)) return s;
        hipError_t e = rtk::launch_trace(p, kernel, stream);
        if (e != hipSuccess) return hip_fail(e, "rt_trace_kernel launch");
        finish_tile_order(ctx, p);
        note_launch(ctx, p, kernel, nf);
        src = dst;  // later launches continue the accumulation in place
    }
    return RT_OK;
}

}  // namespace

extern "C" {

uint32_t rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_last_error(void) { return g_last_error.c_str(); }

const char* rt_kernel_name(int which) {
    static const char* const names[] = {"rt_trace_kernel<0>",      "rt_trace_kernel<1>",
                                        "rt_trace_kernel<2>",      "rt_trace_kernel<3>",
                                        "rt_trace_kernel<4>",      "rt_bounce_kernel<0>",
                                        "rt_bounce_kernel<1>",     "rt_bounce_kernel<2>",
                                        rtk::single_kernel_name(0),
                                        rtk::single_kernel_name(1),
                                        "rt_bounce_kernel<3>",     "rt_tpair_kernel<2>",
                                        "rt_tpair_kernel<4>"};
    if (which >= 0 && which < (int)(sizeof(names) / sizeof(names[0]))) return names[which];
    return rtk::trace_kernel_name();
}

rt_status rt_last_launch_info(const rt_ctx* ctx, rt_launch_info* out) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = ctx->last;
    return RT_OK;
}

rt_status rt_candidate_stats(rt_ctx* ctx, uint64_t out[5]) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "out is NULL");
    for (int i = 0; i < 5; ++i) out[i] = 0;
    out[4] = rtk::kCandMax;
    if (!ctx->cand || ctx->cand_live == 0) return RT_OK;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    // the count is the first word of each tile's kCandStride-float4 block
    std::vector<uint32_t> cnt(ctx->cand_live);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess)
        e = hipMemcpy2D(cnt.data(), sizeof(uint32_t), ctx->cand, rtk::kCandStride * sizeof(float4),
                        sizeof(uint32_t), cnt.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy2D(candidate counts)");
    out[0] = cnt.size();
    for (uint32_t c : cnt) {
        if (c == rtk::kCandNone) {
            out[1]++;
        } else {
            out[2] += c;
            out[3] = std::max<uint64_t>(out[3], c);
        }
    }
    return RT_OK;
}

rt_status rt_create(int device, rt_ctx** out_ctx) {
    if (!out_ctx) return fail(RT_ERR_INVALID_ARGUMENT, "out_ctx is NULL");
    *out_ctx = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    if (device < 0 || device >= n) return fail(RT_ERR_INVALID_DEVICE, "no such HIP device");
    rt_ctx* ctx = new (std::nothrow) rt_ctx();
    if (!ctx) return fail(RT_ERR_NO_MEMORY, "out of host memory");
    ctx->device = device;
    *out_ctx = ctx;
    return RT_OK;
}

rt_status rt_destroy(rt_ctx* ctx) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    rt_status st = RT_OK;
    {
        DeviceGuard guard(ctx->device);
        if (ctx->d_geom || ctx->d_sph || ctx->cand) (void)hipDeviceSynchronize();
        (void)hipFree(ctx->d_geom);
        (void)hipFree(ctx->d_sph);
        (void)hipFree(ctx->d_flag);
        (void)hipFree(ctx->d_hint_rs);
        (void)hipFree(ctx->d_band_src);
        for (hipEvent_t ev : ctx->time_ev)
            if (ev) (void)hipEventDestroy(ev);
        (void)hipFree(ctx->d_srgb);
        (void)hipFree(ctx->d_hx);
        (void)hipFree(ctx->tile_cost);
        (void)hipFree(ctx->tile_order);
        (void)hipFree(ctx->d_grid);
        (void)hipFree(ctx->wg_buf);
        (void)hipFree(ctx->split_col);
        (void)hipFree(ctx->split_cnt);
        (void)hipFree(ctx->unit_order);
        free_candidates(ctx);
        for (uint32_t k = 0; k + 1 < RT_MAX_UPDATE_QUEUES; ++k) {
            if (ctx->aux[k]) (void)hipStreamDestroy(ctx->aux[k]);
            if (ctx->join_ev[k]) (void)hipEventDestroy(ctx->join_ev[k]);
        }
        if (ctx->fork_ev) (void)hipEventDestroy(ctx->fork_ev);
        st = chain_report(ctx);
        // (a segment still outstanding after the bound leaves the chain's resources in place)
        if (rt_status d = rtc::chain_destroy(ctx->chain)) st = d;
    }
    delete ctx;
    return st;
}

rt_status rt_set_scan_mode(rt_ctx* ctx, int mode) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (mode != RT_SCAN_EXHAUSTIVE && mode != RT_SCAN_CULLED)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown scan mode");
    ctx->scan_mode = mode;
    return RT_OK;
}

rt_status rt_set_frames_per_launch(rt_ctx* ctx, uint32_t frames_per_launch) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    ctx->frames_per_launch = frames_per_launch;
    return RT_OK;
}

rt_status rt_set_frame_pairs(rt_ctx* ctx, int mode) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (mode != RT_FRAME_PAIRS_AUTO && mode != RT_FRAME_PAIRS_OFF && mode != RT_FRAME_PAIRS_ON &&
        mode != RT_FRAME_PAIRS_QUAD && mode != RT_FRAME_PAIRS_ON2 && mode != RT_FRAME_PAIRS_QUAD2)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown frame-pair mode");
    ctx->frame_pairs = mode;
    return RT_OK;
}

rt_status rt_set_path_compaction(rt_ctx* ctx, int mode) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (mode != RT_PATHS_AUTO && mode != RT_PATHS_PER_WAVE && mode != RT_PATHS_COMPACT &&
        mode != RT_PATHS_PAIR && mode != RT_PATHS_SPLIT)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown path-compaction mode");
    ctx->path_compaction = mode;
    return RT_OK;
}

rt_status rt_set_single_kernel(rt_ctx* ctx, int mode) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (mode != RT_SINGLE_AUTO && mode != RT_SINGLE_OFF && mode != RT_SINGLE_PAIR &&
        mode != RT_SINGLE_ONE)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown single-kernel mode");
    ctx->single_kernel = mode;
    return RT_OK;
}

rt_status rt_set_update_queues(rt_ctx* ctx, uint32_t queues) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (queues > RT_MAX_UPDATE_QUEUES)
        return fail(RT_ERR_INVALID_ARGUMENT, "queues above RT_MAX_UPDATE_QUEUES");
    ctx->update_queues = queues;
    return RT_OK;
}

rt_status rt_set_update_submit(rt_ctx* ctx, int mode) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (mode != RT_SUBMIT_AUTO && mode != RT_SUBMIT_HIP && mode != RT_SUBMIT_AQL)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown submit mode");
    ctx->update_submit = mode;
    return RT_OK;
}

rt_status rt_update_submit_status(rt_ctx* ctx, int* aql_available, uint32_t* go_give_ups,
                                  uint64_t* packets) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    if (!ctx->chain_tried) {
        // (sets the chain up without any HSA queue: queues are created by the first segment)
        ctx->chain_tried = true;
        rt_status st = RT_OK;
        ctx->chain = rtc::chain_create(ctx->device, &st);
        if (st != RT_OK) return st;
    }
    uint32_t gave_up = 0;
    if (ctx->chain && !rtc::chain_failed(ctx->chain))
        if (rt_status s = rtc::chain_errors(ctx->chain, &gave_up)) return s;
    if (rt_status s = chain_report(ctx)) return s;
    const char* why = "";
    const bool ok = rtc::chain_ok(ctx->chain, &why);
    if (aql_available) *aql_available = ok ? 1 : 0;
    if (packets) *packets = rtc::chain_packets(ctx->chain);
    if (go_give_ups) *go_give_ups = (ctx->chain && rtc::chain_failed(ctx->chain)) ? 1u : gave_up;
    if (!ok) fail(RT_OK, std::string("AQL submission unavailable: ") + why);
    return RT_OK;
}

rt_status rt_set_frame_images(rt_ctx* ctx, int mode) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (mode != RT_FRAME_IMAGES_LAST_TWO && mode != RT_FRAME_IMAGES_EVERY)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown frame-images mode");
    ctx->frame_images = mode;
    return RT_OK;
}

rt_status rt_set_tile_order(rt_ctx* ctx, int mode) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (mode != RT_TILE_ORDER_AUTO && mode != RT_TILE_ORDER_OFF)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown tile-order mode");
    ctx->tile_order_mode = mode;
    return RT_OK;
}

rt_status rt_get_frames_per_launch(const rt_ctx* ctx, const rt_scene_camera* cam,
                                   uint32_t* out) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!cam || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL camera or out");
    rtk::TraceParams p;
    std::memset(&p, 0, sizeof(p));
    fill_camera(p, *cam);
    *out = frames_per_launch_for(ctx, p);
    return RT_OK;
}

rt_status rt_set_spheres(rt_ctx* ctx, const rt_sphere* spheres, uint32_t count, void* stream) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    return upload_spheres(ctx, spheres, count, static_cast<hipStream_t>(stream));
}

rt_status rt_init_image(rt_ctx* ctx, float* out, uint32_t w, uint32_t h, void* stream) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "out_rgba is NULL");
    if (rt_status s = check_image(w, h)) return s;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipError_t e = rtk::launch_init(reinterpret_cast<float4*>(out), (uint64_t)w * h,
                                    static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "rt_init_kernel launch");
    // every pixel now holds count 0 (for a whole-image update of this size)
    rtk::TraceParams p;
    std::memset(&p, 0, sizeof(p));
    p.width = w;
    p.height = h;
    p.band_step = 1;
    record_count(ctx, out, p, 0u);
    return RT_OK;
}

rt_status rt_update(rt_ctx* ctx, const float* in, float* out, uint32_t w, uint32_t h,
                    const rt_scene_camera* cam, const rt_sphere* spheres, uint32_t count,
                    void* stream) {
    if (in != nullptr && in == out)
        return fail(RT_ERR_INVALID_ARGUMENT, "rt_update: in and out must not alias");
    if (!cam) return fail(RT_ERR_INVALID_ARGUMENT, "camera is NULL");
    const float seed = cam->random_seed;
    return trace(ctx, in, out, w, h, 0, 1, cam, spheres, count, 1, &seed, stream);
}

rt_status rt_render(rt_ctx* ctx, const float* in, float* out, uint32_t w, uint32_t h,
                    const rt_scene_camera* cam, const rt_sphere* spheres, uint32_t count,
                    uint32_t frames, const float* seeds, void* stream) {
    return trace(ctx, in, out, w, h, 0, 1, cam, spheres, count, frames, seeds, stream);
}

}  // extern "C"

namespace {

rt_status update_frames(rt_ctx* ctx, float* image_a, float* image_b, uint32_t w, uint32_t h,
                        const rt_band_set& bands, const rt_scene_camera* cam,
                        const rt_sphere* spheres, uint32_t count, uint32_t frames,
                        const float* seeds, void* stream_v, int* out_newest) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (image_a == image_b) return fail(RT_ERR_INVALID_ARGUMENT, "image_a and image_b alias");
    DeviceGuard guard(ctx->device);
    CALL_STAMP(1);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    // an earlier call's AQL segment that failed is reported here, once
    if (rt_status s = chain_report(ctx)) return s;
    hipStream_t stream = static_cast<hipStream_t>(stream_v);
    rtk::TraceParams p;
    if (rt_status s = prepare(ctx, image_a, image_b, w, h, bands, cam, spheres, count, seeds,
                              stream, p))
        return s;
    CALL_STAMP(2);
    float4* img[2] = {reinterpret_cast<float4*>(image_a), reinterpret_cast<float4*>(image_b)};
    // Frames per launch (frames_per_launch_for).  Fusing removes the per-launch fill, tail
    // and kernel boundary (≈ 6 µs of a 30-µs K3 frame): the camera-ray-only instances
    // (max_depth <= 1) and the bounce instance (max_depth >= 2) run up to kHintFrames
    // frames per launch, the hint's reach; rt_set_frames_per_launch caps both (1 = one
    // dispatch per frame, the reference's structure).  The exhaustive and general culled
    // instances run one frame per launch.
    const uint32_t per = frames_per_launch_for(ctx, p);
    int cur = 0;
    ctx->last = {0, 0, 0, -1, 0, 0, 0};
    // What the call has in flight beside the caller's stream, closed on every exit path (an
    // error return included): an AQL segment still being packed is dropped (nothing of it has
    // been submitted), and the context's aux streams are joined back into `stream`, so the
    // caller's later work stays ordered after everything the call issued.
    struct InFlight {
        rt_ctx* ctx;
        hipStream_t stream;
        rtc::Chain* chain = nullptr;
        bool seg_open = false;      // an AQL segment of this call is open
        uint32_t aux_live = 0;      // aux streams with work of this call not yet joined
        ~InFlight() {
            if (seg_open) rtc::chain_abort(chain);
            for (uint32_t k = 0; k < aux_live; ++k)   // (errors here: the call already failed)
                if (hipEventRecord(ctx->join_ev[k], ctx->aux[k]) == hipSuccess)
                    (void)hipStreamWaitEvent(stream, ctx->join_ev[k], 0);
        }
    } fl{ctx, stream};
    bool forked = false;        // aux streams ordered after the last work on `stream`
    // One-frame launches of the one-frame instances go out as AQL packets when the call has
    // two or more of them (rt_set_update_submit; a single update gains nothing from it).
    if (per == 1u && frames >= 2u)
        if (rt_status s = usable_chain(ctx, p, &fl.chain)) return s;
    rtc::Chain* const chain = fl.chain;
    uint32_t seg_parts = 0, seg_packets = 0;
    // launch timing (rt_set_launch_timing): armed for this call's fused launches, disarmed on
    // every exit path
    struct Timing {
        rt_ctx* ctx;
        explicit Timing(rt_ctx* c) : ctx(c) {
            if (ctx->timing) rtk::arm_launch_events(ctx->time_ev[0], ctx->time_ev[1]);
        }
        ~Timing() {
            if (ctx->timing) ctx->timed_launches = rtk::disarm_launch_events();
        }
    } timing_scope{ctx};
    for (uint32_t f0 = 0; f0 < frames; f0 += per) {
        const uint32_t nf = std::min<uint32_t>(per, frames - f0);
        p.in = img[cur];
        p.out = img[1 - cur];
        p.out2 = img[cur];
        // (nf == 1: the plain single-frame store; else the ping-pong images of the last two
        // frames, or of every frame: rt_set_frame_images)
        p.store_each = nf == 1u ? 0u : ctx->frame_images == RT_FRAME_IMAGES_EVERY ? 2u : 1u;
        p.frames = nf;
        p.reset_first = (f0 == 0 && cam->camera_has_moved > 0.5f) ? 1u : 0u;
        for (uint32_t f = 0; f < nf; ++f) p.seed_b[f] = host_f2u(seeds[f0 + f] * 4294967296.0f);
        // the counts both buffers hold afterwards (hint bookkeeping, see plan_hint)
        uint32_t n_in = 0;
        const bool known = p.reset_first || lookup_count(ctx, p.in, p, n_in);
        uint32_t n_prev = 0, n_last = 0;
        if (known) {
            n_last = fill_hint(p, p.reset_first ? 0u : n_in);
            // the frame before the last: what the other buffer holds when nf >= 2
            n_prev = p.reset_first ? 0u : n_in;
            for (uint32_t f = 0; f + 1u < nf; ++f) n_prev = next_count(n_prev, p.spp);
        } else {
            p.hint_frames = 0;
            p.hint_acc_frames = 0;
        }
        // Frame groups (several waves per tile, alternate frames) whenever every frame of
        // the launch is hinted: faster at every rank count measured.
        int kernel = trace_kernel_for(ctx, p);
        const bool pairable = kernel == rtk::kTraceList && p.store_each && known &&
                              p.hint_frames == nf;
        if (pairable && ctx->frame_pairs != RT_FRAME_PAIRS_OFF) {
            // AUTO: four waves per tile when the share is small (a few tiles per SIMD), four
            // per pair of tiles up to twice that, two per pair above (rt_kernels.h
            // kQuadMaxTiles / kQuad2MaxTiles; DESIGN.md §5 "Frame groups over tile pairs")
            const int mode = ctx->frame_pairs;
            const uint64_t tiles = (uint64_t)((w + 7u) >> 3) * p.local_bands;
            const bool automode = mode == RT_FRAME_PAIRS_AUTO;
            // (the tile-pair instances read the candidate blocks: lists required)
            const bool tpair = p.cand && (mode == RT_FRAME_PAIRS_ON2 || mode == RT_FRAME_PAIRS_QUAD2 ||
                                          (automode && tiles > rtk::kQuadMaxTiles));
            const bool quad = mode == RT_FRAME_PAIRS_QUAD || mode == RT_FRAME_PAIRS_QUAD2 ||
                              (automode && (tiles <= rtk::kQuadMaxTiles ||
                                            (tpair && tiles <= rtk::kQuad2MaxTiles)));
            kernel = quad ? (tpair ? rtk::kTraceListQuad2 : rtk::kTraceListQuad)
                          : (tpair ? rtk::kTraceListPair2 : rtk::kTraceListPair);
        }
        kernel = single_or(ctx, p, kernel);
        const bool aql = chain && nf == 1u &&
                         (kernel == rtk::kTraceSingle || kernel == rtk::kTraceSingleOne);
        const uint32_t parts = aql ? update_parts_aql(ctx, p) : update_parts(ctx, p, kernel);
        p.parts = parts;
        p.part = 0;
        // A new workgroup order (built on the stream by plan_wg_order) changes which pixels
        // each part owns, and rewrites the order buffer the parts may still be reading: the
        // parts in flight are joined into `stream` first and forked again after it.
        const bool new_order = wg_order_pending(ctx, p, kernel);
        if (fl.seg_open && (!aql || parts != seg_parts || new_order ||
                            seg_packets + parts > rtc::kMaxSegmentPackets)) {
            fl.seg_open = false;
            if (rt_status s = rtc::chain_end(chain, stream)) return s;
        }
        if ((parts == 1u || aql || new_order) && fl.aux_live) {  // wait for the parts
            if (rt_status s = join_aux(ctx, fl.aux_live, stream)) return s;
            fl.aux_live = 0;
            forked = false;
        }
        CALL_STAMP(3);
        if (rt_status s = plan_tile_order(ctx, p, kernel, stream)) return s;
        if (rt_status s = plan_wg_order(ctx, p, kernel, stream)) return s;
        if (rt_status s = plan_split(ctx, p, kernel, stream)) return s;
        if (rt_status s = plan_hint_rs(ctx, p, kernel)) return s;
        CALL_STAMP(4);
        if (aql) {
            // frame f of part k is a packet on the chain's queue k, after part k's frame f - 1
            if (!fl.seg_open) {
                if (rt_status s = rtc::chain_begin(chain, stream, parts)) return s;
                fl.seg_open = true;
                seg_parts = parts;
                seg_packets = 0;
            }
            for (uint32_t k = 0; k < parts; ++k) {
                p.part = k;
                if (rt_status s = rtc::chain_frame(chain, p, kernel, k)) return s;
            }
            seg_packets += parts;
        } else if (parts > 1u) {
            // every part's next frame reads only the pixels its own previous frame wrote;
            // what `stream` prepared (lists, order, the input image) is forked to the others
            if (rt_status s = ensure_aux_streams(ctx, parts - 1u)) return s;
            // The fork: the aux streams wait for an event recorded on `stream` — unless
            // `stream` has nothing left to run (a new call on an idle stream: then everything
            // it was given is complete and the aux streams, joined into it at the end of the
            // previous call, are idle too), which spares the host the event record and the
            // waits (two HIP calls; the GPU time measured the same either way,
            // profiles/r05/r05b_region_k3.jsonl).  Part 0 goes out before the waits.
            bool wait_fork = false;
            if (!forked) {
                if (hipStreamQuery(stream) != hipSuccess) {
                    hipError_t e = hipEventRecord(ctx->fork_ev, stream);
                    if (e != hipSuccess) return hip_fail(e, "fork (hipEventRecord)");
                    wait_fork = true;
                }
                forked = true;
            }
            for (uint32_t k = 0; k < parts; ++k) {
                p.part = k;
                if (k == 1u && wait_fork)
                    for (uint32_t j = 0; j + 1u < parts; ++j) {
                        hipError_t e = hipStreamWaitEvent(ctx->aux[j], ctx->fork_ev, 0);
                        if (e != hipSuccess) return hip_fail(e, "fork (hipStreamWaitEvent)");
                    }
                hipError_t e = rtk::launch_trace(p, kernel, k ? ctx->aux[k - 1] : stream);
                if (e != hipSuccess) return hip_fail(e, "rt_single_kernel launch");
                if (k) fl.aux_live = std::max(fl.aux_live, k);
            }
        } else {
            hipError_t e = rtk::launch_trace(p, kernel, stream);
            if (e != hipSuccess) return hip_fail(e, "rt_trace_kernel launch");
        }
        CALL_STAMP(5);
        finish_tile_order(ctx, p);
        note_launch(ctx, p, kernel, nf, parts, aql);
        // frame f of the launch wrote img[(cur + 1 + f) % 2]
        const int newest = (nf & 1u) ? 1 - cur : cur;
        if (known) {
            record_count(ctx, img[newest], p, n_last);
            if (nf >= 2) record_count(ctx, img[1 - newest], p, n_prev);
        } else {
            forget_count(ctx, img[newest]);
            if (nf >= 2) forget_count(ctx, img[1 - newest]);
        }
        cur = newest;
    }
    if (fl.seg_open) {   // the call's work ends on the caller's stream
        fl.seg_open = false;
        if (rt_status s = rtc::chain_end(chain, stream)) return s;
    }
    if (fl.aux_live) {
        const uint32_t n = fl.aux_live;
        fl.aux_live = 0;
        if (rt_status s = join_aux(ctx, n, stream)) return s;
    }
    if (out_newest) *out_newest = cur;
    CALL_STAMP(6);
#ifdef RT_CALL_STAMPS
    std::fprintf(stderr, "RT_CALL_STAMPS %u %llu %llu %llu %llu %llu %llu\n", frames,
                 g_call_stamp[1] - g_call_stamp[0], g_call_stamp[2] - g_call_stamp[0],
                 g_call_stamp[3] - g_call_stamp[0], g_call_stamp[4] - g_call_stamp[0],
                 g_call_stamp[5] - g_call_stamp[0], g_call_stamp[6] - g_call_stamp[0]);
#endif
    return RT_OK;
}

// gathered row of every output band: band_src[b] = the row (in rows_per_rank-row rank
// buffers back to back) where band b's first row lies; false if the sets do not cover every
// band exactly once or a set exceeds rows_per_rank
bool band_sources(uint32_t h, uint32_t nranks, const rt_band_set* sets, uint32_t rows_per_rank,
                  std::vector<uint32_t>& out) {
    const uint32_t bands = (h + RT_STRIPE_ROWS - 1) / RT_STRIPE_ROWS;
    out.assign(bands, ~0u);
    uint64_t seen = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
        const rt_band_set& bs = sets[r];
        if (check_band_set(h, bs) != RT_OK) return false;
        if ((uint64_t)bs.count * RT_STRIPE_ROWS > rows_per_rank) return false;
        for (uint32_t j = 0; j < bs.count; ++j) {
            const uint32_t b = bs.first + j * bs.step;
            if (out[b] != ~0u) return false;          // two owners
            out[b] = (uint32_t)((uint64_t)r * rows_per_rank + (uint64_t)j * RT_STRIPE_ROWS);
            ++seen;
        }
    }
    return seen == bands;
}

}  // namespace

namespace rti {
bool band_sets_cover(uint32_t h, uint32_t nranks, const rt_band_set* sets,
                     uint32_t rows_per_rank) {
    std::vector<uint32_t> src;
    return band_sources(h, nranks, sets, rows_per_rank, src);
}
}  // namespace rti

extern "C" {

rt_status rt_update_frames(rt_ctx* ctx, float* image_a, float* image_b, uint32_t w, uint32_t h,
                           uint32_t rank, uint32_t nranks, const rt_scene_camera* cam,
                           const rt_sphere* spheres, uint32_t count, uint32_t frames,
                           const float* seeds, void* stream_v, int* out_newest) {
    CALL_STAMP(0);
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (nranks == 0 || rank >= nranks) return fail(RT_ERR_INVALID_ARGUMENT, "bad rank/nranks");
    return update_frames(ctx, image_a, image_b, w, h, stripe_set(h, rank, nranks), cam, spheres,
                         count, frames, seeds, stream_v, out_newest);
}

rt_status rt_update_frames_bands(rt_ctx* ctx, float* image_a, float* image_b, uint32_t w,
                                 uint32_t h, const rt_band_set* bands,
                                 const rt_scene_camera* cam, const rt_sphere* spheres,
                                 uint32_t count, uint32_t frames, const float* seeds,
                                 void* stream_v, int* out_newest) {
    CALL_STAMP(0);
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!bands) return fail(RT_ERR_INVALID_ARGUMENT, "bands is NULL");
    return update_frames(ctx, image_a, image_b, w, h, *bands, cam, spheres, count, frames,
                         seeds, stream_v, out_newest);
}

rt_status rt_set_launch_timing(rt_ctx* ctx, int enable) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    if (enable && !ctx->time_ev[0]) {
        for (int i = 0; i < 2; ++i) {
            hipError_t e = hipEventCreate(&ctx->time_ev[i]);
            if (e != hipSuccess) return hip_fail(e, "hipEventCreate(launch timing)");
        }
    }
    ctx->timing = enable != 0;
    ctx->timed_launches = 0;
    return RT_OK;
}

rt_status rt_last_call_kernel_time(rt_ctx* ctx, float* out_ms, uint32_t* out_launches) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!out_ms) return fail(RT_ERR_INVALID_ARGUMENT, "out_ms is NULL");
    if (!ctx->timing || ctx->timed_launches == 0)
        return fail(RT_ERR_INVALID_ARGUMENT, "the last call carried no timed launch");
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipError_t e = hipEventSynchronize(ctx->time_ev[1]);
    if (e == hipSuccess) e = hipEventElapsedTime(out_ms, ctx->time_ev[0], ctx->time_ev[1]);
    if (e != hipSuccess) return hip_fail(e, "hipEventElapsedTime(launch timing)");
    if (out_launches) *out_launches = ctx->timed_launches;
    return RT_OK;
}

rt_status rt_band_costs(rt_ctx* ctx, uint32_t w, uint32_t h, const rt_band_set* bands,
                        double* out_cost) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!bands || !out_cost) return fail(RT_ERR_INVALID_ARGUMENT, "NULL bands or out_cost");
    const uint32_t group = ctx->cost_key[5];
    const uint32_t want[5] = {w, h, bands->first, bands->step, bands->count};
    // (and for the lists the context holds now: another camera geometry, scene or share
    // since then starts a new generation, whose costs are not measured yet)
    if (!ctx->cost_key_ok || !ctx->tile_cost || !std::equal(want, want + 5, ctx->cost_key) ||
        ctx->cost_gen != ctx->cand_gen)
        return fail(RT_ERR_INVALID_ARGUMENT, "no tile costs recorded for this share");
    const uint32_t tiles_x = (((w + 7u) >> 3) + group - 1u) / group;
    const uint64_t units = (uint64_t)tiles_x * bands->count;
    std::vector<uint32_t> c(units);
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    if (units) {
        hipError_t e = hipMemcpy(c.data(), ctx->tile_cost, units * sizeof(uint32_t),
                                 hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy(tile costs)");
    }
    for (uint32_t j = 0; j < bands->count; ++j) {
        double sum = 0.0;
        for (uint32_t x = 0; x < tiles_x; ++x) sum += c[(uint64_t)j * tiles_x + x];
        out_cost[j] = sum;
    }
    return RT_OK;
}

rt_status rt_partition_bands(const double* cost, uint32_t nbands, uint32_t nranks,
                             rt_band_set* out) {
    if (!cost || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL band_cost or out");
    if (nranks == 0) return fail(RT_ERR_INVALID_ARGUMENT, "nranks is 0");
    if (nbands > 65536u) return fail(RT_ERR_INVALID_SIZE, "more than 65536 bands");
    for (uint32_t b = 0; b < nbands; ++b)
        if (!(cost[b] >= 0.0) || !std::isfinite(cost[b]))
            return fail(RT_ERR_INVALID_ARGUMENT, "band costs must be finite and >= 0");
    // The smallest largest-range cost B* over all cuts into at most nranks contiguous ranges
    // (a range's cost: the difference of prefix sums), by bisection over B with the greedy
    // test "ranges as long as they fit under B" (O(bands) per step, memory O(bands)).  The
    // test is monotone in B and changes only at range costs, so once lo < hi are adjacent
    // doubles with hi feasible and lo not, B* = hi exactly.  The cut under hi then takes
    // ranges as long as fit but always leaves one band for each rank still to come, so it
    // uses min(nranks, nbands) ranges: once that bound binds, every later range is one band,
    // which fits (B* >= every band's cost).
    std::vector<double> pre(nbands + 1, 0.0);
    for (uint32_t b = 0; b < nbands; ++b) pre[b + 1] = pre[b] + cost[b];
    auto cuts = [&](double B, std::vector<uint32_t>* starts) -> uint64_t {
        uint64_t n = 0;
        for (uint32_t i = 0; i < nbands;) {
            uint32_t j = i + 1;                      // a range holds at least one band
            if (pre[j] - pre[i] > B) return UINT64_MAX;
            // (the final cut: leave a band for each of the ranks after this one)
            const uint64_t left = starts && nranks > n + 1 ? nranks - n - 1 : 0;
            const uint32_t jmax = left >= nbands ? i + 1
                                                 : std::max<uint32_t>(i + 1, nbands - (uint32_t)left);
            while (j < jmax && pre[j + 1] - pre[i] <= B) ++j;
            if (starts) starts->push_back(i);
            ++n;
            i = j;
        }
        return n;
    };
    double lo = 0.0, hi = pre[nbands];
    for (uint32_t b = 0; b < nbands; ++b) lo = std::max(lo, cost[b]);
    if (cuts(lo, nullptr) <= nranks) {
        hi = lo;
    } else {
        for (int it = 0; it < 2200; ++it) {              // (2^-1074 steps cover any range)
            const double mid = lo + (hi - lo) / 2.0;
            if (!(mid > lo && mid < hi)) break;
            if (cuts(mid, nullptr) <= nranks) hi = mid; else lo = mid;
        }
    }
    std::vector<uint32_t> starts;
    cuts(hi, &starts);
    starts.push_back(nbands);
    for (uint32_t r = 0; r < nranks; ++r) {
        if (r + 1 < starts.size())
            out[r] = {starts[r], 1u, starts[r + 1] - starts[r]};
        else
            out[r] = {0u, 1u, 0u};   // no band left (more ranks than ranges)
    }
    return RT_OK;
}

rt_status rt_deinterleave_bands(rt_ctx* ctx, const float* gathered, float* out, uint32_t w,
                                uint32_t h, uint32_t nranks, const rt_band_set* sets,
                                uint32_t rows_per_rank, void* stream_v) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!gathered || !out || !sets) return fail(RT_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (gathered == out) return fail(RT_ERR_INVALID_ARGUMENT, "gathered and out alias");
    if (nranks == 0) return fail(RT_ERR_INVALID_ARGUMENT, "nranks is 0");
    if (rt_status s = check_image(w, h)) return s;
    std::vector<uint32_t> src;
    if (!band_sources(h, nranks, sets, rows_per_rank, src))
        return fail(RT_ERR_INVALID_ARGUMENT,
                    "band sets must cover every band once, each within rows_per_rank rows");
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipStream_t stream = static_cast<hipStream_t>(stream_v);
    if (src != ctx->band_src) {
        // (the previous table may still be read by a queued de-interleave)
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        if (src.size() > ctx->band_src.size() || !ctx->d_band_src) {
            (void)hipFree(ctx->d_band_src);
            ctx->d_band_src = nullptr;
            ctx->band_src.clear();
            e = hipMalloc(&ctx->d_band_src, src.size() * sizeof(uint32_t));
            if (e != hipSuccess) return hip_fail(e, "hipMalloc(band table)");
        }
        e = hipMemcpy(ctx->d_band_src, src.data(), src.size() * sizeof(uint32_t),
                      hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy(band table)");
        ctx->band_src = src;
    }
    hipError_t e = rtk::launch_deinterleave_bands(
        reinterpret_cast<const float4*>(gathered), reinterpret_cast<float4*>(out), w, h,
        ctx->d_band_src, stream);
    return e == hipSuccess ? RT_OK : hip_fail(e, "rt_deinterleave_bands_kernel launch");
}

uint32_t rt_stripe_local_rows(uint32_t height, uint32_t rank, uint32_t nranks) {
    if (nranks == 0 || rank >= nranks) return 0;
    const uint32_t bands = (height + RT_STRIPE_ROWS - 1) / RT_STRIPE_ROWS;
    const uint32_t local = bands > rank ? (bands - rank + nranks - 1) / nranks : 0;
    return local * RT_STRIPE_ROWS;
}

rt_status rt_render_stripes(rt_ctx* ctx, const float* in, float* out, uint32_t w, uint32_t h,
                            uint32_t rank, uint32_t nranks, const rt_scene_camera* cam,
                            const rt_sphere* spheres, uint32_t count, uint32_t frames,
                            const float* seeds, void* stream) {
    return trace(ctx, in, out, w, h, rank, nranks, cam, spheres, count, frames, seeds, stream);
}

rt_status rt_deinterleave_stripes(rt_ctx* ctx, const float* gathered, float* out, uint32_t w,
                                  uint32_t h, uint32_t nranks, void* stream) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!gathered || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (gathered == out) return fail(RT_ERR_INVALID_ARGUMENT, "gathered and out alias");
    if (nranks == 0) return fail(RT_ERR_INVALID_ARGUMENT, "nranks is 0");
    if (rt_status s = check_image(w, h)) return s;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipError_t e = rtk::launch_deinterleave(
        reinterpret_cast<const float4*>(gathered), reinterpret_cast<float4*>(out), w, h,
        nranks, rt_stripe_local_rows(h, 0, nranks), static_cast<hipStream_t>(stream));
    return e == hipSuccess ? RT_OK : hip_fail(e, "rt_deinterleave_kernel launch");
}

rt_status rt_selftest_fastmath(rt_ctx* ctx, uint64_t n_random, uint64_t out[5]) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "out is NULL");
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc(&d, 5 * sizeof(unsigned long long));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(selftest)");
    unsigned long long h[5] = {0, 0, 0, 0, 0};
    e = hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rtk::launch_selftest(d, n_random, nullptr);
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "rt_selftest_kernel");
    for (int i = 0; i < 5; ++i) out[i] = h[i];
    return RT_OK;
}

void rt_srgb_thresholds(float out[256]) {
    out[0] = 0.0f;
    for (int j = 1; j < 256; ++j) {
        const double v = (j - 0.5) / 255.0;  // encoded boundary between j-1 and j
        const double lin = v <= 0.04045 ? v / 12.92 : std::pow((v + 0.055) / 1.055, 2.4);
        float f = (float)lin;
        if ((double)f < lin) f = std::nextafter(f, 2.0f);
        out[j] = f;
    }
}

rt_status rt_present_rgba8(rt_ctx* ctx, const float* in, uint8_t* out, uint32_t w, uint32_t h,
                           int encoding, void* stream_v) {
    if (!ctx) return fail(RT_ERR_INVALID_CONTEXT, "ctx is NULL");
    if (!in || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL image");
    if (encoding != RT_ENCODE_LINEAR && encoding != RT_ENCODE_SRGB)
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown encoding");
    if (rt_status s = check_image(w, h)) return s;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return fail(RT_ERR_INVALID_DEVICE, "hipSetDevice failed");
    hipStream_t stream = static_cast<hipStream_t>(stream_v);
    if (encoding == RT_ENCODE_SRGB && !ctx->d_srgb) {
        float t[256];
        rt_srgb_thresholds(t);
        float* d = nullptr;
        hipError_t e = hipMalloc(&d, sizeof(t));
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(sRGB table)");
        e = hipMemcpy(d, t, sizeof(t), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(d);
            return hip_fail(e, "hipMemcpy(sRGB table)");
        }
        ctx->d_srgb = d;
    }
    hipError_t e = rtk::launch_present(reinterpret_cast<const float4*>(in),
                                       reinterpret_cast<uchar4*>(out), (uint64_t)w * h,
                                       encoding == RT_ENCODE_SRGB ? ctx->d_srgb : nullptr,
                                       stream);
    return e == hipSuccess ? RT_OK : hip_fail(e, "rt_present_kernel launch");
}

}  // extern "C"
