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
// Per-tile candidate blocks of camera rays (culled scan), kCandStride float4 (1 KB) per
// tile: [0] the count (u32 bits of .x; kCandNone = no list), [kCandRecOff + j] the scan
// record of entry j (index order; the record slots past the count are zero up to a whole
// chunk of 4 and anything after — the scans read whole chunks and a chunk ahead, but only
// consider indices < count), [kCandSphOff + 2j, +1] entry j's 32-B sphere record.  A wave
// can fetch its tile's whole list with one 16-B load per lane.
constexpr uint32_t kCandStride = 64;
constexpr uint32_t kCandMax = 19;
constexpr uint32_t kCandRecOff = 1;
constexpr uint32_t kCandSphOff = 21;
constexpr uint32_t kCandNone = 0xFFFFFFFFu;
static_assert(kCandRecOff + ((kCandMax + 3u) & ~3u) <= kCandSphOff, "record chunks fit");
static_assert(kCandSphOff + 2u * kCandMax <= kCandStride, "sphere records fit");
// Sample-count hint (see TraceParams::hint_n): per-(frame, bounce) random numbers of the
// scatter step for at most kHintEntries (frame, bounce) pairs of the first kHintFrames
// frames of a launch.
#ifndef RT_HINT_FRAMES
#define RT_HINT_FRAMES 64   // 16 / 32 / 64: 24.4 / 24.1 / 24.0 us per K3 frame
#endif
constexpr uint32_t kHintFrames = RT_HINT_FRAMES;
constexpr uint32_t kHintEntries = RT_HINT_FRAMES;
// the bounce instance's device table of scatter random numbers (TraceParams::hint_rs_dev):
// up to kHintFrames frames of up to kHintRsDepth bounces
constexpr uint32_t kHintRsDepth = 16;

// Everything the `update` kernel needs, passed by value (kernarg -> SGPRs).
struct TraceParams {
    const float4* in;    // local image (compact stripes), row pitch = width
    float4* out;
    // store_each (rt_update_frames): frame f of the launch stores its image to out for
    // even f and to out2 (the input buffer) for odd f — the ping-pong of chained `update`
    // dispatches (lib.rs:366-374), with the accumulator kept in registers.  1: only the last
    // two frames' images survive the launch, so only they are written; 2: every frame's
    // image is written (rt_set_frame_images EVERY).
    float4* out2;
    uint32_t store_each;
    const float4* geom;  // per sphere: (cx, cy, cz, r*r) — the scan's 16-B record
    const float4* sph;   // per sphere: the 32-B GpuSphere as two float4 (pos+r, color)
    uint32_t width, height, count;
    uint32_t band_first, band_step, local_bands;  // stripe map (RT_STRIPE_ROWS rows/band)
    uint32_t frames;       // accumulation frames in this launch (1 = one `update`)
    uint32_t reset_first;  // camera_has_moved > 0.5 applies to frame 0 only
    uint32_t lds_records;  // culled scan: records staged in LDS (0 = read from HBM/L2)
    uint32_t cand_k;       // per-tile candidate list capacity (0 = no lists)
    const float4* cand;    // [tile][kCandStride] candidate blocks (see kCandStride)
    // one-frame launches (rt_single_kernel): workgroup u traces (band << 16 | column group)
    // wg_order[u] (launch_wg_order), null = natural order
    const uint32_t* wg_order;
    // one-frame launches: this launch is part `part` of `parts` concurrent parts of the
    // update (rt_set_update_queues), each on its own stream: the wg_order list's sub-list
    // `part` (launch_wg_order with `parts`), or without an order every parts-th local band
    // from band `part`.  parts <= 1: the whole update.
    uint32_t part, parts;
    // Uniform XZ grid over the small spheres for bounce rays (rt_kernels.hip scan_grid;
    // built by rt_abi.cpp build_grid): per cell the range of its items, each item a copy
    // of the sphere's scan record and its index (every small sphere is registered in the
    // cells near its centre); grid_big lists the other spheres.  grid_nx == 0: no grid.
    const uint2* grid_cells;     // [grid_nx * grid_nz] (first item, end)
    const float4* grid_geom;     // [items] scan records (cx, cy, cz, r*r)
    const uint32_t* grid_items;  // [items] sphere indices
    const uint32_t* grid_big;    // sphere indices
    uint32_t grid_nx, grid_nz, grid_nbig;
    float grid_x0, grid_z0, grid_s, grid_inv_s;
    float grid_ylo, grid_yhi;    // slab of the gridded spheres, padded
    // a ray may use the grid only if 2.5e-3 * (|o - grid_c| + grid_reach) <= grid_m (the
    // f32 margin of the discriminant stays inside the registration padding)
    float grid_cx, grid_cy, grid_cz, grid_reach, grid_m;
    float grid_e;                // bound on the walk's f32 position error (also in the padding)
    const uint32_t* hx;    // [width]  hash(x * 73)  (wgsl:309, pixel-invariant)
    const uint32_t* hy;    // [height] hash(y * 51)  (wgsl:310)
    float center[3], vul[3], pdu[3], pdv[3], ddu[3], ddv[3];
    float defocus_angle;
    // u32(max_depth), u32(samples_per_pixel) (camera.rs:343, wgsl:343, 268) and per frame
    // B = u32(random_seed * 4294967296.0) (wgsl:311, 353), converted on the host with the
    // kernel's own f32 -> u32 rule.
    uint32_t depth, spp;
    // Sample-count hint.  The scatter step's random numbers depend only on the pixel's
    // sample count n, the frame seed and the bounce (sb = hash(n + B + 2 + 1000 i),
    // wgsl:268, 353), not on the pixel.  When the host knows the count every pixel of `in`
    // holds (it wrote the image, or the frame resets it), hint_n[f] is that count at
    // frame f and hint_rs[f * depth + i] = (rf(sb), random_unit_vector(sb)) for the
    // first hint_frames frames.  Waves whose live pixels all hold hint_n[f] use these
    // values and a scalar camera seed; the accumulator load is then only awaited after
    // the sample is traced, and any pixel whose loaded count differs is traced again with
    // its own count — so the hint never changes a bit of the result.
    // Tile order (camera-ray-only instances, one tile per workgroup): workgroup i of the
    // launch traces tile tile_order[i] = (local band << 16) | column instead of tile i;
    // null = natural order.  tile_cost (non-null): each tile's wave 0 stores its
    // s_memtime duration there, for launch_tile_order.
    const uint32_t* tile_order;
    uint32_t* tile_cost;
    // bounce instance (kTraceBounce): compact live paths across the workgroup's waves
    // after every bounce (1), let each wave keep its own paths (0), frame pairs (2), or
    // split each tile's frames into `split` chunks traced by separate waves (3)
    uint32_t compact;
    // compact == 3: chunks per tile, each chunk's per-frame colours in split_col (one 1-KB
    // row of 64 float4 per tile and frame, [tile][frame][lane]), arrivals per tile in
    // split_cnt (zero between launches: the last arriver resets it)
    uint32_t split;
    uint32_t split_tiles;  // the leading slots of the order that split (the rest: one unit)
    float4* split_col;
    uint32_t* split_cnt;
    // compact == 3 with a measured order: the launch's units costliest first (launch_unit_order:
    // entry = split << 31 | chunk << 28 | band << 16 | column), *unit_count of them; the grid
    // has tiles * split workgroups and those past the count exit at once
    const uint32_t* unit_order;
    const uint32_t* unit_count;
    // 1: one Markstein step from rcp_refined(R) is the IEEE (p - C) / R for every radius of
    // the scene (rt_rcp_check_kernel at upload: exhaustive over the numerators' significands)
    uint32_t normal_rn;
    uint32_t hint_frames;  // 0 = no hint
    // hint_n / hint_rcp hold frames [0, hint_acc_frames) (hint_frames <= hint_acc_frames:
    // hint_rs has room for fewer frames at depth > 1); 0 = no hint
    uint32_t hint_acc_frames;
    // The scene's |C| + |R| stay within 2^40 (rt_abi.cpp scene_bound): with roots_fast_wave's
    // per-wave check of the rays, the root test's sqrt and divisions may run on the fast cores
    uint32_t roots_fast;
    // The scatter step's random numbers of the bounce instance (hint_rs for every hinted
    // frame and bounce: hint_rs holds too few entries at depth > 1): row f * depth + i of a
    // device table that rt_hint_rs_kernel fills from hint_n and seed_b before the launch, for
    // frames [0, hint_rs_dev_frames); 0 = none (depth > kHintRsDepth, or no hint)
    float4* hint_rs_dev;
    uint32_t hint_rs_dev_frames;
    uint32_t hint_n[kHintFrames];
    // RN32(1 / f32(hint_n[f] + 1)): the accumulator's division by f32(n + 1) as a Markstein
    // division (rtd::div_rn; exact for integer n + 1 < 2^22, rt_kernels.hip kAccRnMax)
    float hint_rcp[kHintFrames];
    // f32 of the count after frame f: f32(hint_n[f] + 1) where the frame accumulates
    // (hint_n[f] < spp: also the divisor k of wgsl:356), else f32(hint_n[f]) — the image's
    // alpha (wgsl:362) and k as scalar operands, no per-frame conversion in the kernels
    float hint_cnt[kHintFrames];
    float4 hint_rs[kHintEntries];
    uint32_t seed_b[kMaxFramesPerLaunch];
};

// Trace kernel instances: the reference's exhaustive scan; per-tile candidate lists for
// camera rays + wave-level cone culling for bounce rays; lists + exhaustive fallback only
// (max_depth <= 1: no bounce rays, so the culling code and its registers are left out).
constexpr int kTraceExhaustive = 0;
constexpr int kTraceCulled = 1;
constexpr int kTraceList = 2;
// Camera-ray-only, two waves per tile tracing alternate frames (rt_update_frames on small
// per-rank images; see rt_kernels.hip, trace_pair).
constexpr int kTraceListPair = 3;
// The same with four waves per tile: for small per-rank shares (few tiles per SIMD), where
// shorter per-wave frame chains keep more waves resident (rt_abi.cpp picks it).
constexpr int kTraceListQuad = 4;
// The frame groups over tile pairs: two pixels per lane (rt_tpair_kernel<2 / 4>).
constexpr int kTraceListPair2 = 11;
constexpr int kTraceListQuad2 = 12;
static_assert(kTraceListPair2 == RT_KERNEL_LIST_PAIR2 && kTraceListQuad2 == RT_KERNEL_LIST_QUAD2,
              "instance ids are the ABI's RT_KERNEL_LIST_*2");
static_assert(kTraceExhaustive == RT_KERNEL_EXHAUSTIVE && kTraceCulled == RT_KERNEL_CULLED &&
                  kTraceList == RT_KERNEL_LIST && kTraceListPair == RT_KERNEL_LIST_PAIR &&
                  kTraceListQuad == RT_KERNEL_LIST_QUAD,
              "instance ids are the ABI's RT_KERNEL_* values");
// Bounce rays (max_depth >= 2) over several frames per launch, live paths compacted across
// the workgroup's waves after every bounce (rt_kernels.hip, rt_bounce_kernel).
constexpr int kTraceBounce = 5;
constexpr uint32_t kBounceWaves = 4;   // tiles (waves) per bounce workgroup
// One frame per launch of the camera-ray-only case (rt_update / a one-frame rt_update_frames
// launch with the kTraceList conditions): rt_kernels.hip, rt_single_kernel.
constexpr int kTraceSingle = 8;
// the same with one tile per wave (small per-rank shares)
constexpr int kTraceSingleOne = 9;
static_assert(kTraceSingle == RT_KERNEL_SINGLE && kTraceSingleOne == RT_KERNEL_SINGLE_ONE,
              "instance ids are the ABI's RT_KERNEL_SINGLE*");
// Tiles per launch below which one-frame launches use one tile per wave (kTraceSingleOne).
// (K3 per-update rank shares, profiles/r02_rank_sim_k3_single_*.jsonl: two tiles per wave
// 24.1 / 14.4 / 9.8 / 8.6 us at 1 / 2 / 4 / 8 ranks, one tile 26.6 / 15.0 / 9.6 / 7.1)
#ifndef RT_SINGLE_ONE_MAX_TILES
#define RT_SINGLE_ONE_MAX_TILES 9000
#endif
constexpr uint64_t kSingleOneMaxTiles = RT_SINGLE_ONE_MAX_TILES;
constexpr bool is_group_kernel(int k) {
    return k == kTraceListPair || k == kTraceListQuad;
}
constexpr bool is_list_kernel(int k) { return k == kTraceList || is_group_kernel(k); }
// Waves (tiles) per workgroup of the one-wave-per-tile instances (kTraceExhaustive,
// kTraceList): four-wave workgroups dispatch faster than one-wave ones (K3 single-frame
// update 29.9 -> 29.1 us, K2 23.0 -> 22.1, profiles/r02_ab_single_frame.log).
#ifndef RT_WG_WAVES
#define RT_WG_WAVES 4
#endif
// Instances that run cost-ordered tiles (one tile per workgroup): the frame groups, and
// kTraceList when its workgroups are one wave.
constexpr bool trace_ordered(int k) {
    return k == kTraceListQuad2 || k == kTraceListPair2 ||
           (is_list_kernel(k) && (is_group_kernel(k) || RT_WG_WAVES == 1));
}
// AUTO's frame groups by tiles per launch (rank 0's K3 share, 20-frame chains, wall µs per
// frame, profiles/r06/r06al/, r06an/): up to kQuadMaxTiles four waves per tile
// (rt_trace_kernel<4>; 8 ranks, 4 080 tiles: 3.08, four per tile pair 3.05, two per tile
// 3.12); up to kQuad2MaxTiles four waves per pair of tiles (rt_tpair_kernel<4>; 3 ranks,
// 10 800 tiles: 5.65 against 5.83 / 5.80 two per tile / pair; 4 ranks, 8 160 tiles: 4.61
// against 4.72 / 5.04); above it two per pair (rt_tpair_kernel<2>; the whole image).  With
// the tile pairs' accumulation split over their two tiles' waves (late round 6,
// profiles/r06/r06bj/) four per pair also won at 2 ranks (16 320 tiles: 7.75-7.80 against
// 8.04-8.13 two per pair), so the bound now covers 2 ranks (was 12 288).  The tile-pair
// instances need candidate lists; without them the same sizes run one tile per group.
constexpr uint64_t kQuadMaxTiles = 6144;
constexpr uint64_t kQuad2MaxTiles = 20000;
// The seed-hash tables share one buffer: hash(x*73) for x < hy_offset(width), then
// hash(y*51) per row (TraceParams::hy == hx + hy_offset(width)).
constexpr uint32_t hy_offset(uint32_t width) { return (width + 63u) & ~63u; }
// Stripe map packed for rt_trace_kernel's preloaded arguments: band_first (16 bits),
// min(band_step, 0x7FFF) (15 bits; exact: a rank with two or more bands has band_step <
// bands <= 8192) and bit 31 = TraceParams::tile_order is set.
constexpr uint32_t pack_bands(uint32_t first, uint32_t step, bool ordered) {
    return first | ((step < 0x7FFFu ? step : 0x7FFFu) << 16) | (ordered ? 1u << 31 : 0u);
}
hipError_t launch_trace(const TraceParams& p, int kernel, hipStream_t stream);
// Launch timing (rt_set_launch_timing): arm two timing events for this host thread's next
// fused launches (rt_trace_kernel / rt_tpair_kernel / rt_bounce_kernel: start on the first,
// stop on every one); disarm returns how many launches carried them.
void arm_launch_events(hipEvent_t start, hipEvent_t stop);
uint32_t disarm_launch_events();
// out[y][x] = gathered[band_src[y / 8] + y % 8][x] (rt_deinterleave_bands)
hipError_t launch_deinterleave_bands(const float4* gathered, float4* out, uint32_t width,
                                     uint32_t height, const uint32_t* band_src,
                                     hipStream_t stream);
hipError_t launch_init(float4* out, uint64_t texels, hipStream_t stream);
// Builds the per-tile candidate blocks for p's camera/scene/stripes (p.cand_k entries at
// most per tile).
hipError_t launch_candidates(const TraceParams& p, float4* cand, hipStream_t stream);
// wg_order for one-frame launches of `pix` tiles per wave: the workgroups by decreasing
// candidate-list load (per tile 4 + count for a tile with a list, 64 for a tile without
// one), sorted by launch_tile_order's buckets;
// wg_cost is scratch of one word per workgroup.
// parts > 1: dealt round-robin into `parts` contiguous sub-lists (part_range).
hipError_t launch_wg_order(const float4* cand, uint32_t tiles_x, uint32_t bands, uint32_t pix,
                           uint32_t* wg_cost, uint32_t* wg_order, hipStream_t stream,
                           uint32_t parts);
// [first, first + len) of sub-list k of n entries dealt round-robin into `parts` sub-lists
inline void part_range(uint32_t n, uint32_t parts, uint32_t k, uint32_t& first, uint32_t& len) {
    first = k * (n / parts) + (k < n % parts ? k : n % parts);
    len = n / parts + (k < n % parts ? 1u : 0u);
}
uint32_t single_wg_tiles(uint32_t pix);
uint32_t single_pix();   // tiles per wave of kTraceSingle
// Frame chains (rt_chain.cpp): one-frame launches submitted as AQL packets.  The chain
// kernels (rt_chain_kernel / rt_chain_reset_kernel for one tile or kTraceSingle's tiles per
// wave, the go and the done packet's kernels), a part of each mangled name to find them
// among the code object's symbols, and the packet's kernel arguments for one part of a
// one-frame launch (chain_args: bytes written, 0 = the part has no workgroup).
constexpr int kChainPix1 = 0, kChainPix1Reset = 1, kChainPix = 2, kChainPixReset = 3,
              kChainGo = 4, kChainDone = 5, kChainKernels = 6;
constexpr uint32_t kHiddenArgsBytes = 256;   // code object v5 hidden arguments
hipError_t chain_load_kernels();
const char* chain_kernel_symbol(int which);
uint32_t chain_args(const TraceParams& p, int kernel, const uint32_t* abort, unsigned char* out,
                    uint32_t cap, uint32_t grid[2], uint32_t* group_threads, int* which);
hipError_t launch_deinterleave(const float4* gathered, float4* out, uint32_t width,
                               uint32_t height, uint32_t nranks, uint32_t max_local_rows,
                               hipStream_t stream);
// 8-bit presentation of a float image (rt_present_rgba8); srgb_t = device T[256] or null
// for the linear encoding.
hipError_t launch_present(const float4* in, uchar4* out, uint64_t texels,
                          const float* srgb_t, hipStream_t stream);
const char* trace_kernel_name();
// "rt_single_kernel<p>": p = pix tiles per wave (0: kTraceSingle's)
const char* single_kernel_name(uint32_t pix);
// tile_order for launch_trace: the local tiles by decreasing recorded cost (quantised
// log2 of tile_cost), so the slowest tiles start first and the cheap ones fill the tail.
hipError_t launch_tile_order(const uint32_t* tile_cost, uint32_t* tile_order, uint32_t tiles,
                             uint32_t tiles_x, hipStream_t stream, uint32_t parts = 1);
// The bounce split schedule's unit order (rt_kernels.hip rt_unit_order_kernel): a tile whose
// recorded cost exceeds k_thr times the sum of all costs runs as `split` chunks of a
// 1/split share each, and all units are ordered by their own cost, costliest first.
hipError_t launch_unit_order(const uint32_t* tile_cost, uint32_t* unit_order,
                             uint32_t* unit_count, uint32_t tiles, uint32_t tiles_x,
                             uint32_t split, float k_thr, hipStream_t stream);
// Exact fast-path self-test (rt_selftest_fastmath): cnt[5] device counters, zeroed.
hipError_t launch_selftest(unsigned long long* cnt, uint64_t n_rand, hipStream_t stream);
// bad[0] |= 1 unless div_rn(a, R, rcp_refined(R)) == a / R for every numerator significand
// (binades 2^0 and 2^-100) and each of the n distinct radii (device array)
hipError_t launch_rcp_check(const float* radii, uint32_t n, uint32_t* bad, hipStream_t stream);

}  // namespace rtk
