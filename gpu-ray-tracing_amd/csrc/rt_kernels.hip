// rt_kernels.hip — gfx950 kernels for the per-pixel ray tracer.
//
// Replaces the reference's WGSL compute kernels (assets/compute_shader.wgsl):
//   rt_trace_kernel   == `update` (wgsl:333-364), optionally fused over several frames
//   rt_init_kernel    == `init`   (wgsl:65-70)
//   rt_deinterleave   root-side scatter of gathered stripe tiles (multi-GPU)
//
// Mapping onto CDNA4: one wave64 = one 8x8 pixel tile (the reference's 8x8 workgroup,
// wgsl:333), four waves per 256-thread workgroup.  The sphere scan (wgsl:164-221) walks
// a wave-uniform index, so the 16-byte scan records are fetched with scalar loads into
// SGPRs and consumed directly as VALU operands — no VGPRs and no LDS traffic per test.
// The 32-byte material record is fetched only for the winning hit.  Each lane keeps its
// pixel's accumulator in registers across fused frames and writes it back with one
// coalesced 16-byte store (one HBM read + one write per pixel per launch).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_kernels.h"

#include <cstddef>
#include <cstring>

// The device code is written for gfx950 only.  Two of its hand-offs between workgroups (the
// split bounce schedule's chunk colours, the AQL chain's frames) rely on that target's cache
// policy bits — the buffer intrinsics' aux = 16 is sc1: write-through stores and L1-bypassing
// loads — and on the drained-`sc1` forms MI355X_MICROARCH.md measures for it (inter-workgroup
// visibility, "Valid forms") in place of agent-scope release / acquire fences.  Another
// target would need those re-checked (or the fences), so it does not compile.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "rt_kernels.hip targets gfx950 only (cache-policy bits of the sc1 hand-offs)"
#endif

namespace rtk {

using namespace rtd;

// ---- diagnostic wave trace (RT_WAVE_TRACE=1 builds only; never in the product) -------
// Per wave of the camera-ray-only and bounce instances: start and end s_memrealtime, HW_ID, XCC_ID,
// indexed by workgroup * 4 + wave (tools/wave_trace.py reads them via rt_diag_wave_trace).
#ifndef RT_WAVE_TRACE
#define RT_WAVE_TRACE 0
#endif
#if RT_WAVE_TRACE
constexpr uint32_t kTraceWaves = 1u << 18;
__device__ unsigned long long g_wave_t[kTraceWaves][2];
__device__ unsigned g_wave_id[kTraceWaves][2];
__device__ __forceinline__ void wave_trace(int end) {
    const uint32_t gw = (blockIdx.y * gridDim.x + blockIdx.x) * 4u + (threadIdx.x >> 6);
    if ((threadIdx.x & 63u) == 0 && gw < kTraceWaves) {
        g_wave_t[gw][end] = __builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide
        if (end) {
            g_wave_id[gw][0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
            g_wave_id[gw][1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
        }
    }
}
#define WAVE_TRACE(e) wave_trace(e)
#else
#define WAVE_TRACE(e) ((void)0)
#endif

// ---- diagnostic bounce counters (RT_BOUNCE_COUNTS=1 builds only; never in the product) ---
// BCOUNT(k): the wave's first active lane adds 1 to g_bcount[k] and the active lanes' count
// to g_bcount[k + 1] — wave-level trips and lane-level work of a code region
// (tools/bounce_counts.py reads them via rt_diag_bounce_counts).
#ifndef RT_BOUNCE_COUNTS
#define RT_BOUNCE_COUNTS 0
#endif
#if RT_BOUNCE_COUNTS
__device__ unsigned long long g_bcount[32];
__device__ __forceinline__ void bcount(int k) {
    const uint64_t ex = __builtin_amdgcn_read_exec();
    if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(ex)) {
        atomicAdd(&g_bcount[k], 1ull);
        atomicAdd(&g_bcount[k + 1], (unsigned long long)__builtin_popcountll(ex));
    }
}
#define BCOUNT(k) bcount(k)
#else
#define BCOUNT(k) ((void)0)
#endif

// ---- diagnostic phase stamps of the one-frame kernel (RT_SSTAMPS=1 builds only) ------
// Per wave of rt_single_kernel: s_memtime when each phase's result is available (the asm
// consumes the value, so the stamp waits for it): 0 entry, 1 workgroup order resolved,
// 2 seed tables + candidate counts arrived, 3 camera rays built, 4 list walk done, 5 hit
// shading + sky done, 6 accumulator consumed, 7 stores issued; 8 / 9 s_memrealtime at entry
// / end (100 MHz), 10 HW_ID, 11 XCC_ID.  tools/stamps_single.py reads them
// (rt_diag_single_stamps).
#ifndef RT_SSTAMPS
#define RT_SSTAMPS 0
#endif
#if RT_SSTAMPS
constexpr uint32_t kSStampWaves = 1u << 17;
__device__ unsigned long long g_sst[kSStampWaves][12];
__device__ __forceinline__ uint32_t sst_wave() {
    return (blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
}
__device__ __forceinline__ void sst_put(int k, unsigned long long t) {
    const uint32_t gw = sst_wave();
    if ((threadIdx.x & 63u) == 0u && gw < kSStampWaves) g_sst[gw][k] = t;
}
#define SST_V(k, dep)                                        \
    do {                                                     \
        asm volatile("" ::"v"(dep));                         \
        sst_put((k), __builtin_amdgcn_s_memtime());          \
    } while (0)
#define SST_S(k, dep)                                        \
    do {                                                     \
        asm volatile("" ::"s"(dep));                         \
        sst_put((k), __builtin_amdgcn_s_memtime());          \
    } while (0)
#elif defined(RT_MARKS)
// (asm-inspection builds: a comment in the code at each phase boundary, after its value)
#define SST_V(k, dep) asm volatile(";MARK " #k ::"v"(dep))
#define SST_S(k, dep) asm volatile(";MARK " #k ::"s"(dep))
#else
#define SST_V(k, dep) ((void)0)
#define SST_S(k, dep) ((void)0)
#endif

// Wave ballot of a per-lane condition.  HIP's __ballot(int) takes the predicate as an int,
// and the bool -> int -> bool round trip costs a v_cndmask + v_cmp per ballot on gfx950;
// the builtin takes the condition's lane mask as it is.
__device__ __forceinline__ unsigned long long rt_ballot(bool x) {
    return __builtin_amdgcn_ballot_w64(x);
}
// The one-frame kernel's (and normalize_w's) wave-uniform decisions come from lane masks
// (mask_*) instead of ballots: lane masks straight from one compare (llvm.amdgcn.icmp /
// fcmp: the v_cmp's SGPR result), combined with & and | as 64-bit scalars.  A ballot of a
// boolean that crosses blocks or combines earlier booleans compiles to a v_cndmask 0/1 +
// v_cmp_ne round trip (two 4-cycle VALU operations) at every use; these do not (round 3:
// K3 19.5-19.8 -> 18.9-19.1 µs, K2 13.6-13.8 -> 13.4 µs per update,
// profiles/r03/r03t_ab_single_masks_all.log).
__device__ __forceinline__ uint64_t mask_ult(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_uicmp(a, b, 36);          // ICMP_ULT
}
__device__ __forceinline__ uint64_t mask_uge(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_uicmp(a, b, 35);          // ICMP_UGE
}
__device__ __forceinline__ uint64_t mask_ne(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_uicmp(a, b, 33);          // ICMP_NE
}
__device__ __forceinline__ uint64_t mask_sge(int a, int b) {
    return __builtin_amdgcn_sicmp(a, b, 39);          // ICMP_SGE
}
__device__ __forceinline__ uint64_t mask_not_lt(float a, float b) {
    return __builtin_amdgcn_fcmpf(a, b, 11);          // FCMP_UGE: !(a < b)
}

// Constant address space (read-only for the whole launch; eligible for scalar loads).
// (The host pass of hipcc also parses device code; there the qualifier is dropped.)
#if defined(__HIP_DEVICE_COMPILE__)
#define kconst __attribute__((address_space(4)))
#else
#define kconst
#endif

// min(|x|, |y|, |z|) (v_min3_f32 with abs modifiers; NaN channels ignored, as IEEE minNum)
__device__ __forceinline__ float min_abs3(v3 v) {
    return fminf(fminf(fabsf(v.x), fabsf(v.y)), fabsf(v.z));
}

struct Hit {
    int idx;     // winning sphere, -1 = miss
    float t;     // its root
};

// sphere_list_hit (wgsl:164-180) + sphere_hit (wgsl:182-201) without the hit record:
// only the closest root and its index are tracked; the record (p, normal, face,
// material) is rebuilt once for the winner, bit-identical to the WGSL's last assignment.
//
// The scan walks the list in chunks of 4 spheres.  The 16-byte scan records of the next
// chunk are fetched with scalar loads while the current chunk is computed (the index is
// wave-uniform, so the records live in SGPRs and feed the VALU directly).  Per sphere the
// common (miss) path is 12 VALU ops for the discriminant; the chunk's four "!(D < 0)"
// tests collapse into one integer max + compare on the float bit patterns (exact: D is
// never -0, see below), so the root-finding path is entered once per chunk at most.

// Discriminant of wgsl:183-187 for one sphere record g = (center, r*r).
__device__ __forceinline__ float discriminant(const float4 g, v3 o, v3 d, float a, float& h) {
    const float ocx = g.x - o.x;                                        // wgsl:183
    const float ocy = g.y - o.y;
    const float ocz = g.z - o.z;
    h = fmaf(ocz, d.z, fmaf(ocy, d.y, ocx * d.x));                      // wgsl:185
    const float c = fmaf(ocz, ocz, fmaf(ocy, ocy, ocx * ocx)) - g.w;    // wgsl:186
    return fmaf(h, h, -(a * c));                                        // wgsl:187
}

// Root selection of wgsl:189-201 for sphere i, given its discriminant.  (Callers only
// pass indices < count.)  The IEEE sqrt and divisions are kept as the compiler emits them:
// exact unscaled fast paths with per-lane domain checks measured slower here (the checks
// and their branches cost more SALU/VALU issue than the shorter sequences save).
__device__ __forceinline__ void consider(float disc, float h, float a, uint32_t i, float& tmax,
                                         int& idx) {
    if (!(disc < 0.0f)) {                                               // wgsl:189
        const float q = sqrtf(disc);
        float root = (h - q) / a;
        if (root <= 0x1.0624dep-10f || tmax <= root) {                  // wgsl:196
            root = (h + q) / a;
            if (root <= 0x1.0624dep-10f || tmax <= root) return;        // wgsl:198
        }
        tmax = root;
        idx = (int)i;
    }
}

// consider() for camera rays whose domain the host has proven (camera_rays_bounded in
// rt_abi.cpp): a = |d|^2 in [2^-11, 2^20] and |h|, sqrt(D) <= 2^53 for every sphere.  Then
// sqrt_core(D + 2^-126) and div_core (ya = the shared reciprocal of a) give the IEEE bits
// wherever the bits matter: for D >= 2^-96 adding 2^-126 (< half an ulp of D) changes
// nothing; for D in [0, 2^-96) both sqrt(D) and sqrt_core(D + 2^-126) are below 2^-47, so
// h -+ q rounds to h when |h| >= 2^-22, and below that both roots are under 0.001 (rejected)
// with either q; |h -+ q| < 2^-100 gives a root under 2^-89 (rejected) with either quotient;
// every other quotient is inside div_core's exact domain.  A first root above 0.001 and at
// or beyond tmax also rejects the second: h + q >= h - q and a > 0 make that root larger
// still.  The device self-test replays both functions on random grazing and ordinary
// cases (rt_selftest_fastmath, out[4]).
__device__ __forceinline__ void consider_fast(float disc, float h, float a, float ya,
                                              uint32_t i, float& tmax, int& idx) {
    if (!(disc < 0.0f)) {                                               // wgsl:189
        const float q = sqrt_core(disc + 0x1p-126f);
        float root = div_core(h - q, a, ya);
        if (root <= 0x1.0624dep-10f) {                                  // wgsl:196
            root = div_core(h + q, a, ya);
            if (root <= 0x1.0624dep-10f || tmax <= root) return;        // wgsl:198
        } else if (tmax <= root) {
            return;
        }
        tmax = root;
        idx = (int)i;
    }
}

// "!(D < 0)" for any of K discriminants, on the bit patterns: a float is < 0 exactly
// when its int32 view is <= 0xFF800000 (-inf) and it is not -0.  D = fma(h, h, -(a*c))
// with h*h >= +0 and a >= +0 cannot round to -0, so the test is one max-tree and one
// compare per chunk (max_bits below).

// Exhaustive scan: the reference's linear walk over every sphere (wgsl:169-177).

// max over the int32 views of K discriminants
template <int K>
__device__ __forceinline__ int max_bits(const float (&dd)[K]) {
    int m = __float_as_int(dd[0]);
#pragma unroll
    for (int k = 1; k < K; ++k) m = max(m, __float_as_int(dd[k]));
    return m;
}

// Chunk sizes: a full-list walk is 4 spheres per s_load_dwordx16 (267 us at K3 against
// 330 us one sphere at a time).  The list-only kernel (max_depth <= 1) walks the short
// per-tile candidate lists (2.7 spheres on average at K3) 2 at a time, testing fewer
// padding records (-2 % at K3; mixing both sizes in one kernel measured slower).
#ifndef RT_SCAN_CHUNK
#define RT_SCAN_CHUNK 4
#endif
#ifndef RT_LIST_CHUNK
#define RT_LIST_CHUNK 2
#endif
// the bounce instance's camera rays over their tile's list (K5: 2.1 entries per tile)
#ifndef RT_BOUNCE_LIST_CHUNK
#define RT_BOUNCE_LIST_CHUNK 2
#endif
template <int kScan>
constexpr int scan_chunk() { return is_list_kernel(kScan) ? RT_LIST_CHUNK : RT_SCAN_CHUNK; }
// Per-frame stores of fused launches (TraceParams::store_each) in rt_trace_kernel exist in
// the camera-ray-only instances alone (the culled instance would spill registers for them
// and runs one frame per launch); the bounce instance (rt_bounce_kernel) has its own
// two-last-frames stores and fuses frames too (rt_abi.cpp frames_per_launch_for).
template <int kScan>
constexpr bool kStoreEach = is_list_kernel(kScan);
// Exact fast division / sqrt cores (rt_device.h) in the camera-ray-only instances, which
// rt_abi.cpp selects only for cameras and scenes inside the proven domain
// (camera_rays_bounded): bit 1 the roots of the scan, 2 the normal, 4 the sky, 8 the
// metal / dielectric normalisations (the last three behind a wave-wide check of their
// operands), 16 the defocus disk's reciprocal table (disk_unit).  K3 per frame (fused): 21.7 us without, 20.9 / 20.1 / 20.1 us with bits
// 1 / 1-2 / 1-4; the accumulator's three divisions by f32(n + 1) the same way (checked
// numerators in [2^-88, 2^88)) measured +0.75 us and are left to the compiler.
// The accumulator's division by f32(n + 1) (wgsl:356) where every pixel of the wave holds
// the hinted count n (the one-frame kernel, the frame groups of trace_pair): a Markstein
// division by k = f32(n + 1) with y = RN32(1 / k) from the host (acc_rn: a multiply and two
// fmas per channel; round 5, against round 2's RN32(num * RN64(1 / k)), acc_f64: two
// conversions and an f64 multiply per channel, each a 4-cycle VALU form).  Exactness: for
// an integer k < 2^22 (kAccRnMax below), div_rn (rt_device.h) returns the IEEE quotient
// whenever num and the quotient are normal; numerators in (0, 2^-102) could give subnormal quotients and take the
// IEEE division (acc_ok: one unsigned compare per channel on the bit patterns; zero passes).
// Zero, inf and NaN numerators need no exclusion in this use: num = col - c with the sample
// colour col finite (|col| <= 1: a product of albedos in [0, 1] and the sky's [0.5, 1]) or
// NaN (a degenerate refraction); -0 / k comes out +0, but num = -0 needs c = +0 and c + (+-0)
// is +0 either way; num = +-inf needs c = -+inf, and c + num / k and c + div_rn(...) are NaN
// both (inf - inf); NaN propagates through both.  rt_selftest_fastmath replays it on random
// accumulators and colours.
constexpr uint32_t kBits2m102 = 0x0C800000u;   // 2^-102
// The Markstein step by k = f32(n + 1) is the IEEE quotient for integer k < 2^22 even where
// q = RN(num y) is 1.5 ulp off (Markstein's hypothesis needs one): num - mid k is a nonzero
// multiple of ulp(num / k) / 2 for every rounding midpoint mid, so |num / k - mid| >=
// ulp / (2 k) > 2^-23 ulp, more than the corrected quotient's error |q - num / k| |k y - 1|
// <= 1.5 ulp 2^-24 (round-5 ADVICE).  Counts of 2^22 or more take the IEEE division.
constexpr uint32_t kAccRnMax = 1u << 22;
// |x| >= 2^-102 or x == +-0 (NaN, inf pass) as one unsigned compare per channel on
// 2 (abs_bits(x) - 1) mod 2^32 = (bits << 1) - 2: the sign shifted out, one v_lshl_add per
// channel instead of an and and an add (x = +-0 wraps to 0xFFFFFFFE, above the bound, as
// abs_bits(x) - 1 wraps to 0xFFFFFFFF; otherwise the doubling is exact, abs_bits < 2^31)
constexpr uint32_t kAccOkDbl = 2u * (kBits2m102 - 1u);
__device__ __forceinline__ uint32_t dbl_m2(float x) { return (__float_as_uint(x) << 1) - 2u; }
// (acc_ok(num) == acc_min_bits(num) >= kAccOkDbl)
__device__ __forceinline__ uint32_t acc_min_bits(v3 num) {
    return min(min(dbl_m2(num.x), dbl_m2(num.y)), dbl_m2(num.z));
}
__device__ __forceinline__ bool acc_ok(v3 num) { return acc_min_bits(num) >= kAccOkDbl; }
// c + num / k with y = RN32(1 / k)
__device__ __forceinline__ v3 acc_rn(v3 c, v3 num, float k, float y) {
    return mk(c.x + div_rn(num.x, k, y), c.y + div_rn(num.y, k, y), c.z + div_rn(num.z, k, y));
}
template <int kScan>
constexpr bool fast_core(int bit) { return is_list_kernel(kScan); }
// The defocus disk's normalisation in the camera-ray-only trace instances (disk_unit)
constexpr int kTraceDisk = 3;

// Scan records are read through the constant address space: they do not change during a
// launch, and only then may the compiler use scalar loads (s_load_dwordx8/16 into SGPRs)
// in kernels that store images inside the frame loop.  (The single-frame list instance
// keeps vector loads: its SGPRs are short, scalar records measured +0.6 us per update.)
template <bool kScalar>
__device__ __forceinline__ float4 load_rec(const float4* __restrict__ geom, uint32_t i) {
    if (kScalar) return ((const kconst float4*)geom)[i];
    return geom[i];
}

// A tile's candidate count through the constant address space: a scalar load (the lists do
// not change during a launch), not a vector load + readfirstlane.
__device__ __forceinline__ uint32_t load_cnt(const float4* cand, uint32_t tile) {
    return ((const kconst uint32_t*)cand)[(size_t)tile * (4u * kCandStride)];
}

// kFast: camera rays in the host-proven domain (consider_fast).  kScalar: read the records
// through the constant address space (below).
template <int K, bool kFast = false, bool kScalar = true>
__device__ __forceinline__ Hit scan_exhaustive(const float4* __restrict__ geom, uint32_t count,
                                               v3 o, v3 d) {
    float tmax = 0x1.05ed2ep+118f;             // 3.4e35 (wgsl:266)
    int idx = -1;
    if (count == 0) return Hit{idx, tmax};
    const float a = dot(d, d);                 // wgsl:184 (ray-invariant)
    const float ya = kFast ? rcp_refined(a) : 0.0f;
    // The record list is zero-padded to whole chunks plus one chunk more (rt_abi.cpp), so
    // every chunk (and the one-ahead prefetch) is a full scalar load; padding records are
    // never accepted (consider() is only called for indices < count).
    float4 cur[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cur[k] = load_rec<kScalar>(geom, k);
    for (uint32_t i = 0; i < count; i += K) {
        float4 nxt[K];
#pragma unroll
        for (int k = 0; k < K; ++k) nxt[k] = load_rec<kScalar>(geom, i + K + k);
        float hh[K], dd[K];
#pragma unroll
        for (int k = 0; k < K; ++k) dd[k] = discriminant(cur[k], o, d, a, hh[k]);
        if (__builtin_expect(max_bits<K>(dd) > (int)0xFF800000, 0)) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (i + k < count) {
                    if (kFast)
                        consider_fast(dd[k], hh[k], a, ya, i + k, tmax, idx);
                    else
                        consider(dd[k], hh[k], a, i + k, tmax, idx);
                }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) cur[k] = nxt[k];
    }
    return Hit{idx, tmax};
}

// ---- Exact wave-level culling --------------------------------------------------------
//
// The 64 rays of a wave (one 8x8 tile, plus lens offsets) are nearly coherent.  Bound all
// of the wave's live rays by one double cone: apex = centroid of the origins, every
// origin within r_O of it, every unit direction within angle theta of the axis A (either
// sign).  For sphere (C, R) with v = C - apex, t = v.A, p = |v - tA|, every ray line is at
// distance >= p cos(theta) - |t| sin(theta) - r_O from C.  In exact arithmetic
// D = |d|^2 (R^2 - dist^2), and the f32 evaluation of wgsl:183-187 errs by less than
// ~32 eps |d|^2 (|oc|^2 + R^2) (eps = 2^-24), so the computed D is certainly negative when
// dist > R + m with m = 2.5e-3 (|oc| + |R|) >= 2.5x sqrt(16 eps)|oc| + sqrt(6 eps)|R|, and
// |oc| <= |t| + p + r_O + d_max (DESIGN.md §5 has the derivation).
// Such a sphere can never be the hit of any lane and is skipped; every other sphere goes
// through the exact per-lane test in list order, so the closest-hit result (including
// the first-index-wins tie rule) is bit-identical to the exhaustive scan.  One sphere
// per lane is tested against the cone (64 spheres per VALU instruction); survivors are
// picked from the ballot mask in increasing index order.  Bounce rays walk the sphere grid
// instead when the scene has one (scan_grid below); non-finite or degenerate rays, wide
// cones (theta >~ 60 deg) and short lists use the exhaustive scan.
constexpr uint32_t kCullMinSpheres = 32;

// Wave-wide reductions on the VALU: row_ror DPP inside each 16-lane row, then the four
// row results are read into SGPRs (v_readlane) and combined, so every lane receives the
// same (uniform) value.  Rounding order does not matter here: the cone only needs to be
// conservative, and the margins of cone_misses() dwarf these errors.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int kRowRor8 = 0x128, kRowRor4 = 0x124, kRowRor2 = 0x122, kRowRor1 = 0x121;
__device__ __forceinline__ float lane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp<kRowRor8>(v);
    v += dpp<kRowRor4>(v);
    v += dpp<kRowRor2>(v);
    v += dpp<kRowRor1>(v);
    return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp<kRowRor8>(v));
    v = fmaxf(v, dpp<kRowRor4>(v));
    v = fmaxf(v, dpp<kRowRor2>(v));
    v = fmaxf(v, dpp<kRowRor1>(v));
    return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ bool finite3(v3 v) {
    return __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z);
}

struct Cone {
    v3 apex, axis;
    float cos_t, sin_t, r_o, d_max;
};

// Builds the cone of the live lanes' rays; false when culling cannot be used.  Must be
// called with the whole wave active (it reduces across lanes).  The apex is the centroid
// of the points q = o + d: for camera rays these are the sample points on the focus
// plane, where the beam of a tile is narrowest; r_o bounds |q - apex| and d_max bounds
// |d| (so |o - apex| <= r_o + d_max for the rounding margin).
__device__ __forceinline__ bool wave_cone(v3 o, v3 d, bool live, Cone& k) {
    const float dd = dot(d, d);
    const v3 q = add(o, d);
    const bool bad = live && !(finite3(o) && finite3(q) && dd > 0.0f && __builtin_isfinite(dd));
    const unsigned long long lm = rt_ballot(live);
    if (lm == 0ull || rt_ballot(bad)) return false;
    // Axis and apex come from the first live lane (v_readlane: no cross-lane reduction);
    // the half-angle, the apex radius and max |d| are then exact max-reductions.
    const int L = (int)__builtin_ctzll(lm);
    const float inv = rsqrtf(dd);
    const v3 u = mk(d.x * inv, d.y * inv, d.z * inv);
    k.axis = mk(lane_f(u.x, L), lane_f(u.y, L), lane_f(u.z, L));
    k.apex = mk(lane_f(q.x, L), lane_f(q.y, L), lane_f(q.z, L));
    const v3 du = sub(u, k.axis), dq = sub(q, k.apex);
    const float s = wave_max(live ? __builtin_amdgcn_sqrtf(dot(du, du)) : 0.0f);  // chord
    const float r = wave_max(live ? __builtin_amdgcn_sqrtf(dot(dq, dq)) : 0.0f);
    const float dm = wave_max(live ? __builtin_amdgcn_sqrtf(dd) : 0.0f);
    const float su = s * 1.001f + 1e-6f;
    if (!(su < 1.0f)) return false;                                  // theta >~ 60 degrees
    k.cos_t = 1.0f - 0.5f * su * su;
    k.sin_t = su * __builtin_amdgcn_sqrtf(1.0f - 0.25f * su * su) * 1.001f;
    k.r_o = r * 1.001f + 1e-6f * (fabsf(k.apex.x) + fabsf(k.apex.y) + fabsf(k.apex.z));
    k.d_max = dm * 1.001f;
    return true;
}

// True when sphere record g = (center, r*r) provably misses every ray of the cone.
// lhs bounds the distance of every ray line from C from below (less 1e-5 of the magnitudes
// for its own f32 evaluation); the computed discriminant is certainly negative when
// dist^2 > R^2 + E, E = eps (16 |oc|^2 + 6 R^2), and m^2 >= 6.25e-6 (|oc|^2 +
// R^2) >= E, so the test is dist > sqrt(R^2 + m^2) — round 4 used R + m, which is larger by
// up to m, about a fifth of a small sphere's radius at the K3 camera's distances (K3's
// candidate lists 2.68 -> 2.22 entries per tile, profiles/r05/r05t/).
__device__ __forceinline__ bool cone_misses(const Cone& k, float4 g) {
    const v3 v = mk(g.x - k.apex.x, g.y - k.apex.y, g.z - k.apex.z);
    const float t = dot(v, k.axis);
    const float p = __builtin_amdgcn_sqrtf(fmaxf(fmaf(-t, t, dot(v, v)), 0.0f));
    const float at = fabsf(t), R = __builtin_amdgcn_sqrtf(g.w) * 1.0001f;
    const float mag = at + p + k.r_o;
    const float lhs = fmaf(p, k.cos_t, -at * k.sin_t) - k.r_o - 1e-5f * mag;
    const float m = 2.5e-3f * (mag + k.d_max + R);
    return lhs > R && lhs * lhs > fmaf(R, R, m * m) * 1.0001f;   // NaN anywhere -> keep
}

// Scan records staged in LDS by the workgroup (culled scan, lists up to kLdsMaxRecords).
extern __shared__ float4 lds_recs[];

// kLds: read the cull records from the workgroup's LDS copy (else from the global array);
// both hold count records zero-padded to a multiple of 64.
// ---- Exact grid walk for incoherent bounce rays ---------------------------------------
//
// The closest hit of the linear scan (consider() in index order: a later sphere wins only
// if strictly nearer) is the minimum over spheres of c_i = root1 if root1 > 0.001, else
// root2 if root2 > 0.001, with ties going to the lower index: a sphere whose first root is
// valid but not below the running tmax has a second root at least as large (h + q >= h - q,
// a > 0), and a tie keeps the earlier index.  So the spheres may be tested in any order with
// consider_any's rule.  A sphere can be accepted only at a root t > 0 whose point lies
// within sqrt(R^2 + m^2) of its centre (m the f32 margin of the discriminant, as in the cone
// test), so the grid walk visits every cell the ray passes through for t >= 0 inside the
// gridded spheres' slab, and each sphere is registered in every cell within
// sqrt(R^2 + grid_m^2) + grid_e of its centre (rt_abi.cpp): no sphere that could be accepted
// is skipped.
// (items: the grid's item index array — the sphere index items[i] is loaded only for a root
// that is accepted or ties; null: i is the sphere index)
__device__ __forceinline__ void consider_any(float disc, float h, float a, uint32_t i,
                                             float& tmax, int& idx,
                                             const uint32_t* items = nullptr) {
    if (!(disc < 0.0f)) {                                               // wgsl:189
        const float q = sqrtf(disc);
        float root = (h - q) / a;
        if (root <= 0x1.0624dep-10f) {                                  // wgsl:196
            root = (h + q) / a;
            if (root <= 0x1.0624dep-10f) return;                        // wgsl:198
        }
        if (root <= tmax) {
            const int si = (int)(items ? items[i] : i);
            if (root < tmax || si < idx) {
                tmax = root;
                idx = si;
            }
        }
    }
}
// consider_any with consider_fast's arithmetic (sqrt_core of D + 2^-126, div_core with the
// shared reciprocal ya of a): the IEEE roots wherever they decide anything, on consider_fast's
// domain (a in [2^-11, 2^20], |h| and sqrt(D) <= 2^53), which roots_fast_wave checks per wave.
__device__ __forceinline__ void consider_any_fast(float disc, float h, float a, float ya,
                                                  uint32_t i, float& tmax, int& idx,
                                                  const uint32_t* items = nullptr) {
    if (!(disc < 0.0f)) {                                               // wgsl:189
        const float q = sqrt_core(disc + 0x1p-126f);
        float root = div_core(h - q, a, ya);
        if (root <= 0x1.0624dep-10f) {                                  // wgsl:196
            root = div_core(h + q, a, ya);
            if (root <= 0x1.0624dep-10f) return;                        // wgsl:198
        }
        if (root <= tmax) {
            const int si = (int)(items ? items[i] : i);
            if (root < tmax || si < idx) {
                tmax = root;
                idx = si;
            }
        }
    }
}
// Whether every live ray of the wave is in consider_fast's domain against every sphere of a
// scene with |C| + |R| <= 2^40 (scene_ok: TraceParams::roots_fast): a = |d|^2 in
// [2^-11, 2^20] and |o|'s components below 2^39.  Then |oc| <= |C| + |o| < 2^41,
// |h| <= |d| |oc| < 2^51 and, with c = |oc|^2 - R^2 >= -R^2, sqrt(D) <= sqrt(h^2 + a R^2)
// < 2^52.  NaN or infinite a / o fail the test.  (Bounce rays and the bounce instance's camera
// rays: the camera-ray-only instances have the host's camera_rays_bounded instead.)
__device__ __forceinline__ bool roots_fast_wave(uint32_t scene_ok, v3 o, float a, bool live) {
    const uint32_t om = max(max(abs_bits(o.x), abs_bits(o.y)), abs_bits(o.z));
    const bool ok = __float_as_uint(a) - 0x3A000000u <= 0x49800000u - 0x3A000000u &&  // a
                    om < 0x53000000u;                                               // 2^39
    return scene_ok != 0u && rt_ballot(live && !ok) == 0ull;
}
// The grid's launch parameters (TraceParams grid_*), as one value: built from the kernel
// argument, or (rt_bounce_kernel) re-read from the kernarg segment at every use so that they
// do not stay live in SGPRs across the frame loop.
struct GridP {
    const uint2* cells;
    const float4* geom;
    const uint32_t* items;
    const uint32_t* big;
    const float4* sgeom;     // TraceParams::geom (the big spheres' records)
    uint32_t nx, nz, nbig;
    float x0, z0, s, inv_s, ylo, yhi, cx, cy, cz, reach, m, e;
    uint32_t roots_fast;     // TraceParams::roots_fast
};
template <typename P>
__device__ __forceinline__ GridP grid_params(const P& p) {
    GridP g;
    g.roots_fast = p.roots_fast;
    g.cells = p.grid_cells;
    g.geom = p.grid_geom;
    g.items = p.grid_items;
    g.big = p.grid_big;
    g.sgeom = p.geom;
    g.nx = p.grid_nx;
    g.nz = p.grid_nz;
    g.nbig = p.grid_nbig;
    g.x0 = p.grid_x0;
    g.z0 = p.grid_z0;
    g.s = p.grid_s;
    g.inv_s = p.grid_inv_s;
    g.ylo = p.grid_ylo;
    g.yhi = p.grid_yhi;
    g.cx = p.grid_cx;
    g.cy = p.grid_cy;
    g.cz = p.grid_cz;
    g.reach = p.grid_reach;
    g.m = p.grid_m;
    g.e = p.grid_e;
    return g;
}
// kFast: the roots by consider_any_fast (the wave passed roots_fast_wave; same bits).
// The walk's own t values (slab and box entry / exit, cell-boundary crossings and their
// steps) are products with refined reciprocals of d's components (rcp_refined: one Newton
// step from v_rcp_f32) rather than IEEE quotients: they only steer the traversal, whose cells
// are padded by e (build_grid).  Each such product is within 1 ulp (<= 2 eps, eps = 2^-24) of
// its exact value instead of half an ulp, so a crossing after k steps is off by at most
// (4 + 6k) eps x the coordinate magnitudes (the start and the k additions of the step,
// each step's own error included), inside e's (k + 16) x 8 eps.  A zero component keeps its
// branch; a subnormal one gives an infinite or huge reciprocal, i.e. an axis the ray does not
// cross (it moves less than 2^-60 along it inside the box), or a NaN t that fminf / fmaxf /
// the compares skip the same way.
// walk: this lane walks the grid (false: a far ray that misses every small sphere, which only
// tests the big list; grid_usable).
template <bool kFast>
__device__ __forceinline__ Hit scan_grid_t(const GridP& p, v3 o, v3 d, bool live, bool walk) {
    const float a = dot(d, d);
    const float ya = kFast ? rcp_refined(a) : 0.0f;
    float tmax = 0x1.05ed2ep+118f;             // 3.4e35 (wgsl:266)
    int idx = -1;
    auto test = [&](float disc, float h, uint32_t i, const uint32_t* items) {
        if (kFast)
            consider_any_fast(disc, h, a, ya, i, tmax, idx, items);
        else
            consider_any(disc, h, a, i, tmax, idx, items);
    };
    // spheres outside the grid (the ground, large ones): every live lane tests them
    for (uint32_t b = 0; b < p.nbig; ++b) {
        const uint32_t i = p.big[b];
        const float4 g = p.sgeom[i];
        float h;
        const float disc = discriminant(g, o, d, a, h);
        if (live) test(disc, h, i, nullptr);
    }
    BCOUNT(26);
    if (!live || !walk) return Hit{idx, tmax};
    BCOUNT(kFast ? 0 : 14);
    // t range of the ray inside the slab and the grid box (t >= 0)
    const float rx = rcp_refined(d.x), ry = rcp_refined(d.y), rz = rcp_refined(d.z);
    float t0 = 0.0f, t1 = 0x1.05ed2ep+118f;
    auto clip = [&](float oc, float dc, float rc, float lo, float hi) {
        if (dc != 0.0f) {
            const float ta = (lo - oc) * rc, tb = (hi - oc) * rc;
            t0 = fmaxf(t0, fminf(ta, tb));
            t1 = fminf(t1, fmaxf(ta, tb));
        } else if (oc < lo || oc > hi) {
            t1 = -1.0f;
        }
    };
    const float xhi = p.x0 + p.s * (float)p.nx;
    const float zhi = p.z0 + p.s * (float)p.nz;
    clip(o.y, d.y, ry, p.ylo, p.yhi);
    clip(o.x, d.x, rx, p.x0, xhi);
    clip(o.z, d.z, rz, p.z0, zhi);
    if (!(t0 <= t1)) return Hit{idx, tmax};
    // 2-D DDA over the cells from P(t0) to P(t1)
    const int nx = (int)p.nx, nz = (int)p.nz;
    int ix = (int)floorf((fmaf(t0, d.x, o.x) - p.x0) * p.inv_s);
    int iz = (int)floorf((fmaf(t0, d.z, o.z) - p.z0) * p.inv_s);
    ix = min(max(ix, 0), nx - 1);
    iz = min(max(iz, 0), nz - 1);
    const int sx = d.x > 0.0f ? 1 : -1, sz = d.z > 0.0f ? 1 : -1;
    const float inf = 0x1.05ed2ep+118f;
    float tx = d.x != 0.0f ? (p.x0 + p.s * (float)(ix + (sx > 0)) - o.x) * rx : inf;
    float tz = d.z != 0.0f ? (p.z0 + p.s * (float)(iz + (sz > 0)) - o.z) * rz : inf;
    const float dtx = d.x != 0.0f ? p.s * fabsf(rx) : inf;
    const float dtz = d.z != 0.0f ? p.s * fabsf(rz) : inf;
    const float slack = 2.0f * p.e * rsqrtf(a) * 1.01f;
    for (int step = 0; step < nx + nz + 2; ++step) {
        BCOUNT(2);
        const uint2 range = p.cells[iz * nx + ix];
        for (uint32_t k = range.x; k < range.y; ++k) {
            BCOUNT(4);
            float h;
            const float disc = discriminant(p.geom[k], o, d, a, h);
            test(disc, h, k, p.items);
        }
        // A cell entered beyond t1, or beyond the closest hit so far, holds no better hit;
        // slack: the walk's position error (grid_e, as t) and 1e-4 of t.
        const float tn = fminf(tx, tz);
        if (tn > fminf(t1, tmax) * 1.0001f + slack) break;
        if (tx < tz) {
            ix += sx;
            tx += dtx;
            if (ix < 0 || ix >= nx) break;
        } else {
            iz += sz;
            tz += dtz;
            if (iz < 0 || iz >= nz) break;
        }
    }
    return Hit{idx, tmax};
}
__device__ __forceinline__ Hit scan_grid(const GridP& p, v3 o, v3 d, bool live, bool walk) {
    if (roots_fast_wave(p.roots_fast, o, dot(d, d), live))
        return scan_grid_t<true>(p, o, d, live, walk);
    return scan_grid_t<false>(p, o, d, live, walk);
}

// The wave may walk the grid: every live ray finite and within reach of the grid margin.
// A ray farther out (walk false) may still share the wave's walk when it certainly misses
// every small sphere: it tests the big list only.  The small spheres lie in the ball B(c,
// reach); sphere i's discriminant is certainly negative where the line passes farther than
// sqrt(R_i^2 + m_i^2) from C_i, m_i = 2.5e-3 (|o - C_i| + R_i) <= m_far = 2.5e-3 (|o - c| +
// reach) (the cone test's margin), so a line at least reach + m_far from c misses them all
// (|C_i - c| + R_i <= reach), and so does a ray whose origin lies past the whole ball (c's
// projection t < -(reach + m_far): both roots of every small sphere negative).  Evaluated with
// a 1.01 / 1.001 widening and 1e-5 |o - c| for the f32 rounding of t and of |o - c|^2 - t^2.
// (K5: 0.038 of every wave-frame fell back to the 500-sphere exhaustive scan for the
// far ground's bounce rays, profiles/r06/r06v/.)
__device__ __forceinline__ bool grid_usable(const GridP& p, v3 o, v3 d, bool live, bool& walk) {
    if (p.nx == 0u) return false;
    const v3 oc = mk(o.x - p.cx, o.y - p.cy, o.z - p.cz);
    const float vv = dot(oc, oc);
    const float dist = __builtin_amdgcn_sqrtf(vv);
    const float dd = dot(d, d);
    const bool fin = finite3(o) && finite3(d) && dd >= 0x1p-20f && dd <= 0x1p20f;
    walk = 2.5e-3f * 1.01f * (dist + p.reach) <= p.m;
    bool far_miss = false;
    if (fin && !walk) {
        const float t = -dot(oc, d) * __builtin_amdgcn_rsqf(dd);   // c along the unit ray
        const float thr = (p.reach + 2.5e-3f * 1.01f * (dist + p.reach)) * 1.001f + 1e-5f * dist;
        far_miss = fmaf(-t, t, vv) > fmaf(1e-5f, vv, thr * thr * 1.0001f) || t < -thr;
    }
    return rt_ballot(live && !(fin && (walk || far_miss))) == 0ull;
}

template <bool kLds>
__device__ __forceinline__ Hit scan_culled(const GridP& gp, const float4* __restrict__ geom,
                                           uint32_t count, v3 o, v3 d, bool live, bool bounce) {
    const float4* recs = kLds ? lds_recs : geom;
    // Bounce rays walk the grid whenever the wave may (measured faster than the cone
    // culling even for coherent specular waves); camera rays of tiles without a candidate
    // list keep the cone, whose rays share a narrow beam.
    bool walk;
    if (bounce && count >= kCullMinSpheres && grid_usable(gp, o, d, live, walk))
        return scan_grid(gp, o, d, live, walk);
    (void)bounce;
    (void)gp;
    Cone k;
    if (count < kCullMinSpheres || !wave_cone(o, d, live, k)) {
        BCOUNT(bounce ? 18 : 20);
        return scan_exhaustive<RT_SCAN_CHUNK>(geom, count, o, d);
    }
    BCOUNT(bounce ? 22 : 24);
    const uint32_t lane = threadIdx.x & 63u;
    const float a = dot(d, d);
    float tmax = 0x1.05ed2ep+118f;
    int idx = -1;
    for (uint32_t base = 0; base < count; base += 64u) {
        const float4 g = recs[base + lane];
        const bool keep = (base + lane < count) && !cone_misses(k, g);
        unsigned long long mask = rt_ballot(keep);
        while (mask) {                                    // survivors, in index order
            const int j = __builtin_ctzll(mask);
            mask &= mask - 1ull;
            const float4 gs = recs[base + (uint32_t)j];   // broadcast read
            float h;
            const float disc = discriminant(gs, o, d, a, h);
            consider(disc, h, a, base + (uint32_t)j, tmax, idx);
        }
    }
    return Hit{idx, tmax};
}

// ---- Per-tile candidate lists for camera rays -----------------------------------------
//
// Every camera ray of a tile passes through the tile's footprint on the focus plane
// (pc = vul + pdu*sx + pdv*sy with sx in [x0, x0+8], sy in [y0, y0+8] for any jitter, since
// rounding is monotonic) and through the lens disk (|o - center| <= |(px,py)| *
// sqrt(|ddu|^2 + |ddv|^2)), whatever the frame seed.  That gives a cone valid for ALL
// frames of a camera: apex = footprint centre Pc, r_O = footprint radius, axis =
// Pc - center, sin(theta) <= (r_O + r_lens) / (|Pc - center| - r_O - r_lens).  Spheres
// that cone_misses() rejects can never be hit by a camera ray of the tile; the others are
// listed (records + indices, in index order) once per camera/scene by
// rt_candidates_kernel, and each frame's camera rays test only that list.
__device__ __forceinline__ float len3(v3 v) { return __builtin_amdgcn_sqrtf(dot(v, v)); }

// The cone of the camera rays through the focus-plane rectangle of pixel columns [x0, x1)
// and rows [y0, y1) (one tile: 8 x 8).
__device__ __forceinline__ bool footprint_cone(const TraceParams& p, float x0, float x1,
                                               float y0, float y1, Cone& k) {
    const v3 vul = mk(p.vul[0], p.vul[1], p.vul[2]), pdu = mk(p.pdu[0], p.pdu[1], p.pdu[2]),
             pdv = mk(p.pdv[0], p.pdv[1], p.pdv[2]);
    const v3 ctr = mk(p.center[0], p.center[1], p.center[2]);
    const v3 pc = fmas(0.5f * (y0 + y1), pdv, fmas(0.5f * (x0 + x1), pdu, vul));
    float rq = 0.0f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const v3 q = fmas(c & 2 ? y1 : y0, pdv, fmas(c & 1 ? x1 : x0, pdu, vul));
        rq = fmaxf(rq, len3(sub(q, pc)));
    }
    float rl = 0.0f;
    if (p.defocus_angle > 0.0f) {
        const v3 du = mk(p.ddu[0], p.ddu[1], p.ddu[2]), dv = mk(p.ddv[0], p.ddv[1], p.ddv[2]);
        rl = __builtin_amdgcn_sqrtf(dot(du, du) + dot(dv, dv));
    }
    const float mag = fabsf(pc.x) + fabsf(pc.y) + fabsf(pc.z) + fabsf(ctr.x) + fabsf(ctr.y) +
                      fabsf(ctr.z);
    rq = rq * 1.001f + 1e-5f * mag;                 // f32 evaluation of pc and o = pc - d + d
    rl = rl * 1.001f + 1e-5f * mag;
    const v3 w = sub(pc, ctr);
    const float L = len3(w), delta = rq + rl;
    if (!(L > 4.0f * delta) || !__builtin_isfinite(L + mag)) return false;
    k.axis = mk(w.x / L, w.y / L, w.z / L);
    k.apex = pc;
    k.sin_t = delta / (L - delta) * 1.01f;
    k.cos_t = __builtin_amdgcn_sqrtf(1.0f - k.sin_t * k.sin_t) * 0.999f;
    k.r_o = rq;
    k.d_max = (L + delta) * 1.001f;
    return true;
}

struct Cam {
    v3 center, vul, pdu, pdv, ddu, ddv;
    float defocus_angle;
    float k1s = -0x1.9943f2p-13f, k1c = 0x1.99eb9cp-16f;   // sincos_k's leading coefficients
};
template <typename P>
__device__ __forceinline__ Cam cam_params(const P& p) {
    Cam cam;
    cam.center = mk(p.center[0], p.center[1], p.center[2]);
    cam.vul = mk(p.vul[0], p.vul[1], p.vul[2]);
    cam.pdu = mk(p.pdu[0], p.pdu[1], p.pdu[2]);
    cam.pdv = mk(p.pdv[0], p.pdv[1], p.pdv[2]);
    cam.ddu = mk(p.ddu[0], p.ddu[1], p.ddu[2]);
    cam.ddv = mk(p.ddv[0], p.ddv[1], p.ddv[2]);
    cam.defocus_angle = p.defocus_angle;
    return cam;
}

// The defocus disk's normalize((cos, sin)) (wgsl:327-331).  Over all 2^32 values of
// hash(seed + 1), len2 = sa^2 + ca^2 takes only the eight f32 values of
// [1 - 6*2^-24, 1 + 2^-23], |sa| >= 2^-30 or sa == +0 and |ca| >= 2^-27 (checked
// exhaustively by rt_selftest_fastmath), so sqrtf(len2) = 1 - m 2^-24 with
// m = (0x3F800001 - bits(len2)) >> 1 in {3, 3, 2, 2, 1, 1, 0, 0}.
// kTable: 0 = sqrt_core / div_core (exact on this domain);
// 3 = all-f32: len = sqrtf(len2) = 1 - m 2^-24 (bits 0x3F800000 - m) and y = RN32(1 / len)
// = 1 + ((m + 1) >> 1) 2^-23 (m = 1: 1 + 2^-24 + 2^-48 rounds up; m = 3: 1 + 1.5 ulp + 9
// 2^-48 rounds to 2 ulp) from the bits of len2, then one Markstein step — q0 = RN(a y), the
// exact residual r = fma(-len, q0, a), q = RN(q0 + r y) — the correctly rounded a / len
// for a correctly rounded y (checked against the IEEE division for all 2^32 seeds by
// rt_selftest_fastmath).  Six f32 operations and four integer ones.  (Rounds 2-4 also had
// an f64 table of RN64(1 / len), per workgroup in LDS or in closed form: the all-f32 form
// replaced it in the one-frame kernel in round 3 and in the frame groups in round 5 — no
// table, no barrier at wave start; an 8-rank K3 chain share 2.69 -> 2.65 us per step,
// profiles/r05/r05h/.)
template <int kTable>
__device__ __forceinline__ void disk_unit(float sa, float ca, float& ux, float& uy) {
    const float len2 = fmaf(sa, sa, ca * ca);
    if (kTable == 3) {
        const uint32_t m = (0x3F800001u - __float_as_uint(len2)) >> 1;
        const float len = __uint_as_float(0x3F800000u - m);
        const float y = __uint_as_float(0x3F800000u + ((m + 1u) >> 1));
        const float qx = ca * y, qy = sa * y;
        ux = fmaf(fmaf(-len, qx, ca), y, qx);
        uy = fmaf(fmaf(-len, qy, sa), y, qy);
    } else {
        const float len = sqrt_core(len2);
        const float y = rcp_refined(len);
        ux = div_core(ca, len, y);
        uy = div_core(sa, len, y);
    }
}

// The lens sample's sincos runs without a NaN guard on its quadrant (the angle is finite):
// K3 14.26 against 14.42 µs per update over three interleaved rounds
// (profiles/r04/r04q_ab_front_fin.txt).
// get_ray (wgsl:305-325) with the pixel-invariant hash(hash(x*73) ^ hash(y*51)) part
// precomputed per pixel: seed = hash(hxy ^ su), su = sample_index*25 + B (wave-uniform
// when every pixel of the wave holds the same sample count).
template <int kTable>
__device__ __forceinline__ void get_ray(const Cam& cam, uint32_t x, uint32_t y, uint32_t hxy,
                                        uint32_t su, v3& o, v3& d,
                                        const v3* c0v = nullptr) {
    const uint32_t seed = hash(hxy ^ su);
    // rf(v) = f32(hash(v)) * 2^-32 is exact (a power-of-two scale of a value >= 1 or 0), so
    // the next rounding is the only one: rf - 0.5 is one fma, 2pi * rf one multiply by
    // 2pi * 2^-32 — the same bits as the two-step forms.
    const float offx = fmaf((float)hash(seed), 0x1p-32f, -0.5f);         // sample_square
    const float offy = fmaf((float)hash(seed * seed), 0x1p-32f, -0.5f);  // wgsl:299-303
    const float sx = ((float)x + 0.5f) + offx;
    const float sy = ((float)y + 0.5f) + offy;
    const v3 pc = fmas(sy, cam.pdv, fmas(sx, cam.pdu, cam.vul));
    // the lens centre in VGPRs (c0v, the copies the lens-less path needs anyway), so that
    // fma(u, ddu, centre) has one scalar operand (gfx950 VALU: one SGPR per instruction)
    // instead of a second copy per component; a caller tracing several pixels per lane
    // passes one copy for all of them
    v3 c0 = c0v ? *c0v : cam.center;
    if (!c0v) asm volatile("" : "+v"(c0.x), "+v"(c0.y), "+v"(c0.z));
    if (cam.defocus_angle > 0.0f) {                     // defocus_disk_sample wgsl:327-331
        const float ang = (float)hash(seed + 1u) * 0x1.921fb4p-30f;  // 2*3.1415926 * rf
        float sa, ca, ux, uy;
        // (ang = f32(hash) * 2pi 2^-32: always finite, so no NaN guard)
        sincos_k(ang, sa, ca, cam.k1s, cam.k1c, true);
        disk_unit<kTable>(sa, ca, ux, uy);
        o = fmas(uy, cam.ddv, fmas(ux, cam.ddu, c0));
    } else {
        // (made here: as a plain copy the compiler hoists it ahead of the branch, three
        // v_mov per pixel on every lens frame)
        o = c0;
        asm volatile("" : "+v"(o.x), "+v"(o.y), "+v"(o.z));
    }
    d = sub(pc, o);
}

// A zero vector materialised where this is called: the frame loops' colour of a frame that
// traces nothing.  As a plain constant the compiler hoists its six v_mov ahead of the branch,
// onto every traced frame (12 per tile-pair frame in rt_tpair_kernel<2>).
__device__ __forceinline__ v3 zero_v3_here() {
    float x, y, z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(x));
    asm volatile("v_mov_b32 %0, 0" : "=v"(y));
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return mk(x, y, z);
}

// component-wise select of two v3 (a select of whole v3 values can leave them in
// scratch memory)
__device__ __forceinline__ v3 sel3(bool c, v3 a, v3 b) {
    return mk(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z);
}

// The reciprocal of |v| in the sky's normalize(d).y and in normalize_w comes from the square
// root's own rsq (sqrt_core_rcp) instead of a second transcendental (v_rcp).  Adopted in
// round 4 with the one-frame kernel's select skipping, the AND sign test and one record per
// tile and step (K3 14.95 -> 14.68 µs per update over three interleaved rounds;
// profiles/r04/r04k_ab_single_variants.txt).
// normalize(v) = v / sqrt(v.v) (WGSL normalize).  kFast: when every active lane's |v|^2 is
// in [2^-20, 2^40] (NaN, 0 and inf are not) and its components are >= 2^-100 in
// magnitude, sqrt_core and div_core with the shared reciprocal of |v| in [2^-10, 2^20]
// (components <= |v|: inside div_core's exact domain); otherwise the IEEE operations.
template <bool kFast>
__device__ __forceinline__ v3 normalize_w(v3 v) {
    if (kFast) {
        const float dd = dot(v, v);
        const uint32_t span = __float_as_uint(dd) - kBits2m20;
        // (a component below 2^-100: min_abs3 and an ordered compare, as in shade_hit)
        if ((mask_uge(span, kBits2p40 - kBits2m20) |
             __builtin_amdgcn_fcmpf(min_abs3(v), 0x1p-100f, 4)) == 0ull) {
            float y;
            const float len = sqrt_core_rcp(dd, y);
            return mk(div_core(v.x, len, y), div_core(v.y, len, y), div_core(v.z, len, y));
        }
    }
    return normalize(v);
}

// ray_color (wgsl:261-297), executed by the whole wave: `live` marks the lanes whose path
// is still being traced; the bounce loop runs while any lane is live, and a lane's
// values are only updated while it is live, so each lane computes exactly its own
// per-pixel result.
// uni (wave-uniform): every live lane of the wave holds the hinted sample count of frame
// f, so the scatter step's random numbers (pixel-independent, see TraceParams::hint_n)
// come from the host-computed hint_rs table instead of three hashes, a sqrt and a sincos
// per lane.
// The hit normal's (p - C) / R (wgsl:209) on div_core's domain (the callers check it),
// y = rcp_refined(R).  rn (wave-uniform, TraceParams::normal_rn): one Markstein step per
// component from y is the IEEE quotient for every numerator of the domain (the numerators
// >= 2^-100, R in [2^-20, 2^20] and |p - C| <= 2^43 keep the quotients normal) — checked
// exhaustively for every distinct radius of the scene on the device at upload
// (rt_rcp_check_kernel); otherwise div_core's two.
__device__ __forceinline__ v3 normal_div(v3 rel, float r, float y, bool rn) {
    if (rn) return mk(div_rn(rel.x, r, y), div_rn(rel.y, r, y), div_rn(rel.z, r, y));
    return mk(div_core(rel.x, r, y), div_core(rel.y, r, y), div_core(rel.z, r, y));
}

// One 16-B buffer load at a byte offset (raw buffer, no format conversion)
__device__ __forceinline__ float4 buf_f4(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                       __uint_as_float(v.w));
}

template <int kScan>
__device__ __forceinline__ v3 ray_color(const TraceParams& p, uint32_t tile, uint32_t ncand,
                                        uint32_t depth, v3 o, v3 d, uint32_t seed, bool live,
                                        bool uni, uint32_t f) {
    v3 cf = mk(1.0f, 1.0f, 1.0f);
    bool black = false;
    for (uint32_t i = 0; i < depth; ++i) {
        if (rt_ballot(live) == 0ull) break;
        // Camera rays of a tile with a candidate list (ncand != kCandNone) test only the
        // listed spheres: their records are in index order and padded like the full list,
        // so the same chunk loop applies; hit.idx then indexes the tile's copy of the
        // sphere records.
        const bool listed = kScan != kTraceExhaustive && i == 0 && ncand != kCandNone;
        const float4* blk = p.cand + (size_t)tile * kCandStride;
        // (one inlined walk for both pointers: two copies measured slower)
        const Hit hit =
            (kScan != kTraceCulled || listed)
                ? scan_exhaustive<scan_chunk<kScan>(), fast_core<kScan>(1), kScan != kTraceList>(
                      listed ? blk + kCandRecOff : p.geom, listed ? ncand : p.count, o, d)
            : p.lds_records ? scan_culled<true>(grid_params(p), p.geom, p.count, o, d, live, i > 0)
                            : scan_culled<false>(grid_params(p), p.geom, p.count, o, d, live, i > 0);
        const float4* hs = listed ? blk + kCandSphOff : p.sph;
        if (!live) continue;
        if (hit.idx < 0) {                                        // wgsl:288-290
            live = false;
            continue;
        }
        // Hit record of the winner (wgsl:205-218).  The two record loads are per-lane and
        // depend on the scan; the scatter's random numbers do not depend on the material
        // (lambertian and metal draw random_unit_vector(sb), dielectric draws rf(sb), its
        // first component), so they are computed while the loads are in flight.
        // (buffer loads here, as in single_sample, measured 1.5 % slower in the 8-rank share
        // kernel: profiles/r06/r06ax/)
        const float4 pr = hs[2 * hit.idx];          // position, radius
        const float4 mat = hs[2 * hit.idx + 1];     // material color
        float r_sb;
        v3 ruv;
        if (uni) {
            const float4 h = p.hint_rs[f * depth + i];
            r_sb = h.x;
            ruv = mk(h.y, h.z, h.w);
        } else {
            const uint32_t sb = hash(seed + i * 1000u);           // wgsl:268
            r_sb = rf(sb);
            ruv = random_unit_vector(r_sb, sb);
        }
        const v3 hp = fmas(hit.t, d, o);
        const v3 C = mk(pr.x, pr.y, pr.z);
        // wgsl:209: (p - C) / R.  Fast core: |R| in [2^-20, 2^20] (host-proven) and every
        // hit lane's three numerators >= 2^-100 in magnitude (they are <= 2^43: the hit
        // lies on a sphere of the bounded scene).
        const v3 rel = sub(hp, C);
        v3 outward;
        if (fast_core<kScan>(2) &&
            rt_ballot(min_abs3(rel) < 0x1p-100f) == 0ull) {    // (see shade_hit)
            const float y = rcp_refined(pr.w);
            outward = normal_div(rel, pr.w, y, p.normal_rn != 0u);
        } else {
            outward = divs(rel, pr.w);
        }
        const bool front = dot(d, outward) < 0.0f;
        const v3 n = sel3(front, outward, neg(outward));
        v3 att = mk(1.0f, 1.0f, 1.0f), nd = d;   // (defined on every path: kept in registers)
        if (mat.w < -1.0f) {                                      // lambertian wgsl:84-93
            const v3 dir = add(n, ruv);
            nd = sel3(dot(dir, dir) < 0x1.0c6f7ap-20f, n, dir);
            att = mk(mat.x, mat.y, mat.z);
        } else if (mat.w <= 1.0f) {                               // metal wgsl:95-100
            constexpr bool kF = fast_core<kScan>(8);
            const v3 refl = fmas(mat.w, ruv, normalize_w<kF>(reflect(d, n)));
            if (!(dot(refl, n) > 0.0f)) {                         // wgsl:277-279
                black = true;
                live = false;
                continue;
            }
            nd = normalize_w<kF>(refl);
            att = mk(mat.x, mat.y, mat.z);
        } else {                                                  // dielectric wgsl:102-135
            att = mk(1.0f, 1.0f, 1.0f);
            const float ratio = front ? 1.0f / mat.x : mat.x;
            constexpr bool kF = fast_core<kScan>(8);
            const v3 u = normalize_w<kF>(d);
            const float cos_t = fminf(dot(neg(u), n), 1.0f);
            const float sin_t = sqrtf(fmaf(-cos_t, cos_t, 1.0f));
            const bool cannot = ratio * sin_t > 1.0f;
            const bool refl = cannot || reflectance(cos_t, ratio) > r_sb;
            nd = normalize_w<kF>(sel3(refl, reflect(u, n), refract(u, n, ratio)));
        }
        cf = mul(cf, att);                                        // wgsl:285-286
        o = hp;
        d = nd;
    }
    if (black) return mk(0.0f, 0.0f, 0.0f);
    // Sky (wgsl:293-296): only normalize(d).y is used.  Fast core when every lane's |d|^2
    // is in [2^-20, 2^40] (NaN and 0 are not): sqrt_core is exact there, and so is
    // div_core(d.y, |d|) for |d.y| >= 2^-100; below that |uy| < 2^-80 and uy + 1 == 1
    // with either quotient.
    const float dd = dot(d, d);
    float uy;
    if (fast_core<kScan>(4) &&
        rt_ballot(__float_as_uint(dd) - kBits2m20 >= kBits2p40 - kBits2m20) == 0ull) {
        // (|d| and its reciprocal from one rsq, as the one-frame kernel's sky: no v_rcp)
        float y;
        const float len = sqrt_core_rcp(dd, y);
        uy = div_core(d.y, len, y);
    } else {
        uy = d.y / sqrtf(dd);
    }
    const float a = 0.5f * (uy + 1.0f);
    const float om = 1.0f - a;
    return mul(cf, mk(fmaf(a, 0.5f, om), fmaf(a, 0x1.666666p-1f, om), fmaf(a, 1.0f, om)));
}

// One wave = one 8x8 tile of the (local) image; lanes are row-major inside the tile.
// Control flow is wave-uniform down to the shading (the culled scan reduces across
// lanes); per-lane conditions of the reference (n < spp, the image bounds) become the
// `live` flag instead of branches.
// a colour's three channels as one vector store (LDS slots of the frame groups)
typedef float f3v __attribute__((ext_vector_type(3)));
struct TileCoord {
    uint32_t x, y;
    size_t idx;
    bool valid;
};

// Launch grid: blockIdx.y = local stripe band, blockIdx.x * 4 + wave = tile column.
__device__ __forceinline__ TileCoord tile_coord(uint32_t width, uint32_t height,
                                                uint32_t band_first, uint32_t band_step,
                                                uint32_t tx, uint32_t lband, uint32_t lane) {
    TileCoord t;
    t.x = tx * 8u + (lane & 7u);
    const uint32_t gband = band_first + lband * band_step;
    t.y = gband * RT_STRIPE_ROWS + (lane >> 3);
    const uint32_t ly = lband * RT_STRIPE_ROWS + (lane >> 3);
    t.valid = (t.x < width) && (t.y < height);
    t.idx = (size_t)ly * width + t.x;
    return t;
}
__device__ __forceinline__ TileCoord tile_coord(const TraceParams& p, uint32_t tx,
                                                uint32_t lband, uint32_t lane) {
    return tile_coord(p.width, p.height, p.band_first, p.band_step, tx, lband, lane);
}

// One sample of one frame for the pixels with `live` set, traced with sample count n
// (wgsl:352-358 without the accumulation).
template <int kScan>
__device__ __forceinline__ v3 sample(const TraceParams& p, const Cam& cam, uint32_t tile,
                                     uint32_t ncand, const TileCoord& tc, uint32_t hxy,
                                     uint32_t n, uint32_t B, uint32_t f, bool live, bool uni) {
    const uint32_t depth = p.depth;
    const uint32_t seed = 1u + n + B;                             // wgsl:353
    v3 o, d;
    get_ray<fast_core<kScan>(16) ? kTraceDisk : 0>(cam, tc.x, tc.y, hxy, seed * 25u + B, o,
                                                  d);                          // wgsl:311
    const v3 col = ray_color<kScan>(p, tile, ncand, depth, o, d, seed + 1u, live, uni, f);
    return col;
}

// acc: the pixel's loaded accumulator (unused when frame 0 resets it).  Without a hint the
// count is taken from acc before the first sample; with a hint the first frame is traced
// with the hinted count while the load is in flight and verified afterwards.
// kHint = false ignores the hint (counts from acc, full per-pixel random numbers): the
// frame-group instance's fallback, kept small so that the instance stays within 64 VGPRs.
template <int kScan, bool kHint = true>
__device__ __forceinline__ float4 trace_pixel(const TraceParams& p, const Cam& cam,
                                              uint32_t tile, uint32_t ncand,
                                              const TileCoord& tc, uint32_t hxy, float4 acc) {
    const uint32_t spp = p.spp;                                   // wgsl:343
    v3 c = mk(0.0f, 0.0f, 0.0f);
    uint32_t n = 0u;
    bool known = p.reset_first != 0u;                             // wgsl:345-350
    if (!known && (!kHint || p.hint_frames == 0u)) {
        c = mk(acc.x, acc.y, acc.z);                              // wgsl:339-341
        n = f2u(acc.w);
        known = true;
    }
    for (uint32_t f = 0; f < p.frames; ++f) {
        const uint32_t B = p.seed_b[f];                           // wgsl:311,353
        if (f == 0 && p.reset_first) {                            // wgsl:345-350
            c = mk(0.0f, 0.0f, 0.0f);
            n = 0u;
        }
        const bool hinted = kHint && f < p.hint_frames;
        uint32_t ng = known ? n : p.hint_n[0];   // count to trace with (unknown: f == 0)
        bool pending = tc.valid;
        for (;;) {
            const bool live = pending && ng < spp;                // wgsl:352
            v3 col = mk(0.0f, 0.0f, 0.0f);
            if (rt_ballot(live) != 0ull) {
                const bool uni = hinted && rt_ballot(live && ng != p.hint_n[f]) == 0ull;
                col = sample<kScan>(p, cam, tile, ncand, tc, hxy, ng, B, f, live, uni);
            }
            bool wrong = false;
            if (!known) {                                         // verify the hint
                c = mk(acc.x, acc.y, acc.z);
                n = f2u(acc.w);
                known = true;
                wrong = pending && n != ng;
            }
            if (pending && !wrong && n < spp) {
                const float k = (float)(n + 1u);                  // wgsl:356
                c = mk(c.x + (col.x - c.x) / k, c.y + (col.y - c.y) / k,
                       c.z + (col.z - c.z) / k);
                n += 1u;
            }
            if (rt_ballot(wrong) == 0ull) break;
            pending = wrong;                                      // retrace these pixels
            ng = n;
        }
        // Chained updates: frame f's image (wgsl:362-363) lands in the other ping-pong
        // buffer; the next frame would read it back (u32(f32(n)), wgsl:341) — here the
        // registers already hold it.  Only the last two frames' images survive the launch
        // (each buffer keeps the last frame written to it, and nothing reads a tile's
        // pixels during the launch but its own wave), so only they are stored — or every
        // frame's (store_each 2, rt_set_frame_images EVERY).
        if (kStoreEach<kScan> && p.store_each && (p.store_each == 2u || f + 2u >= p.frames) &&
            tc.valid)
            ((f & 1u) ? p.out2 : p.out)[tc.idx] = make_float4(c.x, c.y, c.z, (float)n);
        n = f2u((float)n);
    }
    return make_float4(c.x, c.y, c.z, (float)n);                  // wgsl:362
}

// Frame groups (kTraceListPair, rt_update_frames with every pixel at the hinted count):
// kFrameGroup waves own the same tile; wave w traces frames f + w of each group of
// kFrameGroup frames (the samples are independent — the count each one uses is the hinted
// n + f, verified up front), waves 1.. hand their colours to wave 0 through LDS, and wave 0
// accumulates the group's frames in order and stores the surviving images (wgsl:352-363)
// — bit-identical to one wave doing every frame.  More waves, each with a shorter
// sequential chain.
// Called only when every valid pixel's loaded count is the hinted one (rt_trace_kernel).
// Waves per tile: 2 (kTraceListPair) or 4 (kTraceListQuad).  K3 per frame, whole image on
// one GPU: 16.8 / 18.8 us; 8-rank share: 3.13 / 2.95 us (`profiles/r01_rank_sim_groups_k3.txt`).
// Round 5: one more wave per tile that only accumulates and stores, so that every group's
// samplers all trace, measured slower at every size (8-rank share 2.91 against 2.54 us per
// step, whole image 17.2 against 14.6; profiles/r05/r05j/); so did tracing each frame with
// the one-frame kernel's sample (single_sample<1>, records from LDS or by scalar loads:
// profiles/r05/r05h/, r05m/).
template <int kScan>
constexpr uint32_t frame_group() {
    return kScan == kTraceListQuad ? 4u : 2u;
}
// LDS of a frame group: two slots of the producer waves' colours (double-buffered groups)
template <int kScan>
constexpr size_t group_lds_bytes() {
    return (size_t)2u * (frame_group<kScan>() - 1u) * 64u * 16u;
}
template <int kScan>
__device__ __forceinline__ void trace_pair(const TraceParams& p, const Cam& cam, uint32_t tile,
                                           uint32_t ncand, const TileCoord& tc, uint32_t hxy,
                                           float4 acc, uint32_t w) {
    const uint32_t spp = p.spp;                                   // wgsl:343
    v3 c = mk(0.0f, 0.0f, 0.0f);
    if (!p.reset_first) c = mk(acc.x, acc.y, acc.z);              // wgsl:339-341
    // From here every valid pixel holds hint_n[f] before frame f (the host's count
    // bookkeeping, rt_abi.cpp fill_hint): the count arithmetic of wgsl:341-362 is scalar.
    const uint32_t lane = threadIdx.x & 63u;
    constexpr uint32_t kFrameGroup = frame_group<kScan>();
    for (uint32_t f = 0; f < p.frames; f += kFrameGroup) {
        const uint32_t fw = f + w;
        const uint32_t ng = fw < p.frames ? p.hint_n[fw] : spp;  // count before frame fw
        v3 col;
        if (ng < spp && rt_ballot(tc.valid) != 0ull) {             // wgsl:352
            col = sample<kScan>(p, cam, tile, ncand, tc, hxy, ng, p.seed_b[fw], fw, tc.valid,
                                fw < p.hint_frames);
        } else {
            col = zero_v3_here();
        }
        // two LDS slots alternating by group: wave 0 reads group g's slot before it reaches
        // the barrier of group g + 1, so one barrier per group suffices
        float4* slot = lds_recs + ((f / kFrameGroup) & 1u) * (kFrameGroup - 1u) * 64u;
        if (w != 0u)
            *reinterpret_cast<f3v*>(&slot[(w - 1u) * 64u + lane]) = f3v{col.x, col.y, col.z};
        __syncthreads();
        if (w == 0u) {
            const uint64_t valid_m = rt_ballot(tc.valid);
#pragma unroll
            for (uint32_t j = 0; j < kFrameGroup; ++j) {
                const uint32_t fj = f + j;
                if (fj >= p.frames) break;
                if (j != 0) {
                    const float4 cj = slot[(j - 1u) * 64u + lane];
                    col = mk(cj.x, cj.y, cj.z);
                }
                const uint32_t nb = p.hint_n[fj];                 // count before frame fj
                // f32(nb + 1) (the divisor k, wgsl:356) or f32(nb): the host's table
                const float cnt = p.hint_cnt[fj];
                if (nb < spp) {                                   // wgsl:352-358
                    const v3 num = sub(col, c);
                    // num / f32(nb + 1) (wgsl:356) as a Markstein division (acc_rn); both
                    // conditions scalar (see rt_tpair_kernel)
                    const bool rn = (nb < kAccRnMax) &
                                    ((mask_ult(acc_min_bits(num), kAccOkDbl) & valid_m) == 0ull);
                    if (rn) {
                        c = acc_rn(c, num, cnt, p.hint_rcp[fj]);
                    } else {
                        const float k = cnt;                      // wgsl:356
                        c = mk(c.x + num.x / k, c.y + num.y / k, c.z + num.z / k);
                    }
                }
                // wgsl:362-363: the images that survive (or every frame's, store_each 2)
                if ((p.store_each == 2u || fj + 2u >= p.frames) && tc.valid)
                    ((fj & 1u) ? p.out2 : p.out)[tc.idx] = make_float4(c.x, c.y, c.z, cnt);
            }
        }
    }
}

// One workgroup = 4 waves = 4 consecutive tiles.  (A persistent grid that walks tiles
// with the next tile's accumulator prefetched — into VGPRs, or into LDS with
// global_load_lds — measured 15-50 % slower: the loop pushes the kernel past 64 VGPRs /
// into scratch, and the hardware dispatcher already overlaps the waves' HBM phases.)
// Minimum waves per SIMD the compiler plans registers for.  7 rather than 8: at 8 it caps
// SGPRs near 80 and spills ~25 of them into VGPR lanes (v_writelane / v_readlane in the
// frame loop); at 7 the instances use 94 SGPRs and, at <= 64 VGPRs, still run 8 waves per
// SIMD (the frame-group instance needs 66 VGPRs: 7 waves).  K3: 29.0 vs 30.3 us per
// single-frame update, 18.2 vs 18.4 us per fused frame.
#ifndef RT_TRACE_MIN_WAVES
#define RT_TRACE_MIN_WAVES 7
#endif
// Kernel-argument prefetch (single-frame list instance, one tile per wave): the launch
// parameters a wave reads are spread over ~12 cache lines of the 2.6-KB kernarg segment and
// the compiler loads each just before its use — a chain of dependent scalar-cache misses at
// every wave start.  One scalar load per line, all in flight together and awaited once,
// brings them into the scalar cache first (K3 single-frame 30.56 -> 30.28 us, K2 23.72 ->
// 23.40, profiles/r02_ab_single_frame.log).  Adding the first lines of the tile's candidate
// and sphere records to it measured +1.0 us (the wave then waits for two HBM misses before
// its first instruction of ray setup).
// Leading scalar arguments of rt_trace_kernel (before the TraceParams block): what a wave
// needs before its first ray — the tile's candidate count, the seed-hash tables, the
// accumulator and the tile geometry.  Built with -mllvm -amdgpu-kernarg-preload-count=9
// (Makefile), the command processor places these 9 dwords in SGPRs at wave launch, so the
// count, hash and accumulator loads issue at once, together with the kernel-argument
// prefetch, instead of after a kernarg round trip (K3 single-frame 30.7 -> 29.6 us, K2 23.7
// -> 22.9, profiles/r02_ab_single_frame.log).  TraceParams (alignment 16) starts at byte 48.
constexpr uint32_t kParamsOff = 48;
__device__ __forceinline__ void karg_prefetch() {
    const char kconst* kp =
        (const char kconst*)__builtin_amdgcn_kernarg_segment_ptr() + kParamsOff;
    uint32_t d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10;
    asm volatile(
        "s_load_dword %0, %11, 0x0\n\t"
        "s_load_dword %1, %11, 0x40\n\t"
        "s_load_dword %2, %11, 0x80\n\t"
        "s_load_dword %3, %11, 0xc0\n\t"
        "s_load_dword %4, %11, 0x100\n\t"
        "s_load_dword %5, %11, 0x140\n\t"
        "s_load_dword %6, %11, 0x180\n\t"
        "s_load_dword %7, %11, %12\n\t"
        "s_load_dword %8, %11, %13\n\t"
        "s_load_dword %9, %11, %14\n\t"
        "s_load_dword %10, %11, %15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(d0), "=&s"(d1), "=&s"(d2), "=&s"(d3), "=&s"(d4), "=&s"(d5), "=&s"(d6),
          "=&s"(d7), "=&s"(d8), "=&s"(d9), "=&s"(d10)
        : "s"(kp), "i"(offsetof(TraceParams, hint_n)), "i"(offsetof(TraceParams, hint_rcp)),
          "i"(offsetof(TraceParams, hint_rs)), "i"(offsetof(TraceParams, seed_b))
        : "memory");
    (void)d0; (void)d1; (void)d2; (void)d3; (void)d4; (void)d5;
    (void)d6; (void)d7; (void)d8; (void)d9; (void)d10;
}

// Waves (tiles) per workgroup: the culled instance shares the LDS copy of the records among
// 4 waves; a frame-group instance is one tile's group; the others RT_WG_WAVES (rt_kernels.h).
template <int kScan>
constexpr uint32_t wg_waves() {
    return kScan == kTraceCulled ? 4u : is_group_kernel(kScan) ? frame_group<kScan>() : RT_WG_WAVES;
}


// Cost-ordered tiles (TraceParams::tile_order / tile_cost) in the camera-ray-only
// instances, whose workgroups are one tile each.

template <int kScan>
constexpr bool kOrdered = trace_ordered(kScan);
// (the start time is parked in tile_cost itself: no register stays live for it)
template <int kScan>
__device__ __forceinline__ void cost_start(const TraceParams& p, uint32_t tile, uint32_t wave,
                                           uint32_t lane) {
    if (kOrdered<kScan> && p.tile_cost && wave == 0u && lane == 0u)
        p.tile_cost[tile] = (uint32_t)__builtin_amdgcn_s_memtime();
}
template <int kScan>
__device__ __forceinline__ void record_cost(const TraceParams& p, uint32_t tile, uint32_t wave,
                                            uint32_t lane) {
    if (kOrdered<kScan> && p.tile_cost && wave == 0u && lane == 0u)
        p.tile_cost[tile] = (uint32_t)__builtin_amdgcn_s_memtime() - p.tile_cost[tile];
}

template <int kScan>
__global__ __launch_bounds__(64 * wg_waves<kScan>(), RT_TRACE_MIN_WAVES) void rt_trace_kernel(
    const float4* __restrict__ a_cand, const uint32_t* __restrict__ a_hx,
    const float4* __restrict__ a_in, uint32_t a_width, uint32_t a_height, uint32_t a_bands,
    const TraceParams p) {
    WAVE_TRACE(0);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t tiles_x = (a_width + 7u) >> 3;
    // The wave index is uniform, but the compiler's divergence analysis does not know it;
    // readfirstlane makes the tile (and the candidate-list pointers and counts derived from
    // it) scalar, so list records are read with s_load into SGPRs.
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // (frame groups: all waves of the workgroup own the same tile)
    uint32_t tx = is_group_kernel(kScan) ? blockIdx.x : blockIdx.x * wg_waves<kScan>() + wave;
    uint32_t lband = blockIdx.y;
    const uint32_t band_first = a_bands & 0xFFFFu, band_step = (a_bands >> 16) & 0x7FFFu;
    if (kOrdered<kScan> && (a_bands >> 31)) {         // costliest tiles first (tile_order)
        const uint32_t slot = blockIdx.y * gridDim.x + blockIdx.x;
        // (readfirstlane: the loaded value is uniform, but only the scalar form keeps the
        // list pointer and records in SGPRs — s_load chunks instead of vector loads)
        const uint32_t t = __builtin_amdgcn_readfirstlane(p.tile_order[slot]);
        tx = t & 0xFFFFu;
        lband = t >> 16;
    }
    const bool wave_in = tx < tiles_x;
    const TileCoord tc = tile_coord(a_width, a_height, band_first, band_step, tx, lband, lane);
    const uint32_t tile = lband * tiles_x + tx;
    // the tile's candidate count (kCandNone: no list), the accumulator (wgsl:339; a frame-0
    // reset discards it: no load) and hash(x*73) ^ hash(y*51) (wgsl:309-310) from the
    // per-column / per-row tables: issued from the preloaded arguments, before the
    // kernel-argument prefetch below is awaited
    const uint32_t ncand = (kScan != kTraceExhaustive && a_cand && wave_in)
                               ? load_cnt(a_cand, tile)
                               : kCandNone;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    // (loaded even when frame 0 resets the pixel or the wave has no tile, so that the load
    // waits for no kernarg read and no branch; the value is discarded then)
    acc = a_in[tc.valid ? tc.idx : 0];
    const uint32_t hxy =
        a_hx[min(tc.x, a_width - 1u)] ^ a_hx[hy_offset(a_width) + min(tc.y, a_height - 1u)];
    if (kScan == kTraceList) karg_prefetch();
    // Culled scan: the workgroup stages the scan records (count padded to 64) in LDS once;
    // the per-block cone test then reads them at LDS latency instead of L2 latency.
    if (kScan == kTraceCulled && p.lds_records) {
        for (uint32_t j = threadIdx.x; j < p.lds_records; j += 512u) {
            const float4 g0 = p.geom[j];
            const float4 g1 = p.geom[j + 256u < p.lds_records ? j + 256u : j];
            lds_recs[j] = g0;
            if (j + 256u < p.lds_records) lds_recs[j + 256u] = g1;
        }
        __syncthreads();
    }
    if (!wave_in) return;                                         // whole wave exits
    cost_start<kScan>(p, tile, wave, lane);

    Cam cam;
    cam.center = mk(p.center[0], p.center[1], p.center[2]);
    cam.vul = mk(p.vul[0], p.vul[1], p.vul[2]);
    cam.pdu = mk(p.pdu[0], p.pdu[1], p.pdu[2]);
    cam.pdv = mk(p.pdv[0], p.pdv[1], p.pdv[2]);
    cam.ddu = mk(p.ddu[0], p.ddu[1], p.ddu[2]);
    cam.ddv = mk(p.ddv[0], p.ddv[1], p.ddv[2]);
    cam.defocus_angle = p.defocus_angle;

    if (is_group_kernel(kScan)) {
        // every frame's image is stored inside; on a count mismatch (every wave sees the
        // same pixels, hence takes the same decision) wave 0 runs the single-wave loop and
        // the others have nothing to do
        if (p.reset_first || rt_ballot(tc.valid && f2u(acc.w) != p.hint_n[0]) == 0ull) {
            trace_pair<kScan>(p, cam, tile, ncand, tc, hxy, acc, wave);
            record_cost<kScan>(p, tile, wave, lane);
            WAVE_TRACE(1);
            return;
        }
        if (wave != 0u) return;
    }
    const float4 res = trace_pixel<kScan, !is_group_kernel(kScan)>(p, cam, tile, ncand, tc,
                                                                   hxy, acc);
    if (tc.valid && !(kStoreEach<kScan> && p.store_each))        // wgsl:363
        p.out[tc.idx] = res;
    record_cost<kScan>(p, tile, wave, lane);
    WAVE_TRACE(1);
}

// ---- Single-frame update (kTraceSingle): one `update` dispatch, camera rays only --------
//
// The reference's step (lib.rs:408-417: one `update` per frame, wgsl:333-364) at
// max_depth <= 1 for cameras in the proven domain (the kTraceList conditions) and one frame
// per launch.  rt_trace_kernel<kTraceList> pays its general machinery (frame loop, retrace
// loop, per-frame kernarg reads spread over a 2.6-KB parameter block) for the one frame;
// this kernel does the one frame only, with its parameters in one compact block, and gives
// each lane kSinglePix pixels — the same column of kSinglePix horizontally adjacent 8x8
// tiles — so that a wave's fixed costs (launch, parameter and list loads, the disk table)
// are shared and its independent pixel chains interleave (more instructions in flight per
// wave while the list and accumulator loads are outstanding).  The per-pixel arithmetic is
// ray_color's (wgsl:261-297) for depth <= 1, operation for operation: the image bits are
// those of rt_trace_kernel (every parity test runs both, rt_set_single_kernel).
struct SingleParams {
    float4* out;
    const float4* geom;    // full scan records (tiles without a candidate list)
    const float4* sph;     // full sphere records
    uint32_t count, depth, spp;
    uint32_t hinted;       // hint_n / hint_rcp / hint_rs of frame 0 are valid
    uint32_t n_hint;       // every pixel's count before the frame (0 on reset)
    uint32_t seed_b;       // B = u32(random_seed * 2^32) (wgsl:311, 353)
    uint32_t hy_off;       // hash(y * 51) table offset in the hx buffer
    float rcp_hint;        // RN32(1 / f32(n_hint + 1)) (acc_rn)
    uint32_t normal_rn;    // TraceParams::normal_rn
    uint32_t reserved[4];  // (the fields after keep round 4's offsets)
    // local bands of a launch in raster order (no a_order): lband = first + blockIdx.y *
    // step, first | step << 16 — one of the update's concurrent parts (launch_single)
    uint32_t lbands;
    float4 rs;             // (rf(sb), random_unit_vector(sb)) of frame 0, bounce 0
    float center[3], vul[3], pdu[3], pdv[3], ddu[3], ddv[3];
    float defocus_angle;
    // the launch's workgroups per row (rt_chain_kernel reads it here instead of the hidden
    // kernel arguments: its packets are written by rt_chain.cpp)
    uint32_t grid_x;
    // rt_chain_kernel only: non-zero once a segment's go wait gave up — the frame's image
    // stores are dropped (rt_chain.cpp; rt_single_kernel ignores it)
    const uint32_t* abort;
};
static_assert(offsetof(SingleParams, lbands) == 76,
              "SingleParams keeps round 4's offsets after rcp_hint");

// Tiles per wave of the two instances: kTraceSingle (whole-image launches) and
// kTraceSingleOne (small per-rank shares, where more, shorter waves fill the chip).
#ifndef RT_SINGLE_PIX
#define RT_SINGLE_PIX 2
#endif
constexpr uint32_t kSinglePix = RT_SINGLE_PIX;
static_assert(kSinglePix >= 1 && kSinglePix <= 4, "1 to 4 tiles per wave");
// Waves per SIMD the one-frame kernel's register plan targets.  The compiler fills the
// SGPR budget the bound allows: at 5 it reached 98 SGPRs (6 resident waves per SIMD on
// gfx950: MI355X_MICROARCH.md, Residency), at 7 it stays at <= 96 (7 waves) without spills.
#ifndef RT_SINGLE_MIN_WAVES
#define RT_SINGLE_MIN_WAVES 7
#endif
// (Knock-out builds of the one-frame kernel — no accumulator load, sphere scan, random
// camera ray, hit shading or image store, for cost attribution — are an experiment-only
// patch: tools/patches/single_knockouts.patch, DESIGN_HISTORY.md §5.)
// waves per workgroup of the one-frame kernel: 2 since round 4 (profiles/r04/r04a2_single_shape.txt,
// r04b2_driver_wg2.txt: 0.2 us per update faster than 4 at K3, same bits)
#ifndef RT_SINGLE_WG
#define RT_SINGLE_WG 2
#endif
constexpr uint32_t kSingleWg = RT_SINGLE_WG;
// The one-frame kernel walks both tiles' candidate lists in one loop, one record of each per
// step (round 4: fewer padding records tested when the two lists differ in length).
// The tiles' 1-KB candidate blocks are loaded whole at wave start (one 16-B load per lane,
// beside the seed and accumulator loads) and kept in LDS: the scan records and the hit
// records are then LDS reads instead of dependent L2/HBM round trips.  It shortens a
// wave's memory chain (8-rank K3 share, one tile per wave: 7.10 -> 6.64 us per update) but
// costs a whole launch more than it saves (K3 24.9 -> 25.8 us, K2 18.3 -> 19.9;
// profiles/r02_ab_single_lds_k*.log): 1 = the one-tile instance only, 2 = both, 0 = none.
#ifndef RT_SINGLE_LDS
#define RT_SINGLE_LDS 1
#endif
// The defocus disk's reciprocal in the one-frame kernel is all-f32 (disk_unit<3>: the length
// and its reciprocal from the bits of len2, one Markstein step; no f64, no LDS table, no
// barrier).  The workgroup's LDS table made every wave wait for wave 0's kernarg read at
// wave start (K3 23.30 -> 22.46 µs per update without it, profiles/r03/r03a_ab_single.log); the
// all-f32 form with the lane masks: profiles/r03/r03t_ab_single_masks_all.log.
constexpr int kSingleDisk = 3;
// hash(x*73) ^ hash(y*51) (wgsl:309-310) of the one-frame kernel: from the per-column /
// per-row tables (two dependent loads behind the order entry) or computed in the wave —
// one hash per lane (lanes [0, 8*kPix) the wave's columns, the next 8 its rows), handed to
// the pixels with ds_bpermute — so the camera rays need no memory at all.  Bit k set =
// computed in the kPix = k + 1 instance.  Default: the one-tile instance (rank shares)
// computes them — 4-rank shares 0.1-0.3 µs faster per update, 8-rank unchanged
// (profiles/r03/r03zn_single_hash1.txt); the two-tile instance (whole images) reads the tables
// (computing them there cost 0.9 µs at K3, profiles/r03/r03e_ab_single_switches.log).
#ifndef RT_SINGLE_HASH
#define RT_SINGLE_HASH 1
#endif

// The one-frame kernel's per-lane selects after the hit shading (hit / miss, the degenerate
// scatter direction, metal absorption) run only in waves whose lanes differ: a wave-uniform
// branch on a lane mask skips them otherwise (round 4, with sqrt_core_rcp above).  The
// sky's |d|^2 (wgsl:294's normalize) is taken from where the direction was made — the
// camera ray's a = d.d (wgsl:184, computed for the scan), the Lambertian scatter's
// |n + ruv|^2 (computed for its degenerate-direction test, wgsl:89), or the normalised metal
// / dielectric direction's own dot — instead of one more dot product per pixel (the same
// operations on the same operands: the same bits; K3 15.93 against 16.37 µs per update in
// the driver's command, profiles/r04/r04p_ab_skydd.txt).

// Shading of a camera ray's hit at depth 1 (ray_color's loop body at i = 0, wgsl:266-286):
// sets the scattered direction and attenuation, or black (metal absorbed).  r_sb / ruv are
// the scatter's random numbers.  Lanes with !hit compute garbage that the caller drops.
__device__ __forceinline__ void shade_hit(float4 pr, float4 mat, float t, v3 o, v3 d,
                                          float r_sb, v3 ruv, bool hit, uint64_t hm,
                                          bool normal_rn, v3& nd, v3& att, bool& black,
                                          bool& took_other, float& ndd) {
    const v3 hp = fmas(t, d, o);
    const v3 rel = sub(hp, mk(pr.x, pr.y, pr.z));
    v3 outward;                                                   // wgsl:209
    // (some |rel| below 2^-100 as one v_min3_f32 on |.| and one ordered compare: the same
    // lanes as the minimum of the abs bit patterns — a NaN channel is never the small one
    // either way, and rel, an arithmetic result, is never a signalling NaN)
    if ((__builtin_amdgcn_fcmpf(min_abs3(rel), 0x1p-100f, 4) & hm) == 0ull) {   // (FCMP_OLT)
        const float y = rcp_refined(pr.w);
        outward = normal_div(rel, pr.w, y, normal_rn);
    } else {
        outward = divs(rel, pr.w);
    }
    const float dno = dot(d, outward);
    const bool front = dno < 0.0f;
    const v3 n = front ? outward : neg(outward);
    // lambertian (wgsl:84-93), computed for every lane; the other materials below
    v3 dir = add(n, ruv);
    const float ddir = dot(dir, dir);
    ndd = ddir;                     // |nd|^2 for the sky (sky_w's dd)
    if ((__builtin_amdgcn_fcmpf(ddir, 0x1.0c6f7ap-20f, 4) & hm) != 0ull) {   // (FCMP_OLT)
        // (the degenerate scatter direction, wgsl:89-91: per-lane selects only in a wave
        // that has one)
        asm volatile("");
        if (ddir < 0x1.0c6f7ap-20f) {
            dir = n;
            ndd = dot(n, n);
        }
    }
    nd = dir;
    att = mk(mat.x, mat.y, mat.z);
    black = false;
    took_other = false;
    const bool other = hit && !(mat.w < -1.0f);
    if ((mask_not_lt(mat.w, -1.0f) & hm) != 0ull)
        took_other = true;
    if ((mask_not_lt(mat.w, -1.0f) & hm) != 0ull && other) {
        if (mat.w <= 1.0f) {                                      // metal wgsl:95-100
            const v3 refl = fmas(mat.w, ruv, normalize_w<true>(reflect(d, n)));
            black = !(dot(refl, n) > 0.0f);                       // wgsl:277-279
            nd = normalize_w<true>(refl);
            ndd = dot(nd, nd);
        } else {                                                  // dielectric wgsl:102-135
            att = mk(1.0f, 1.0f, 1.0f);
            const float ratio = front ? 1.0f / mat.x : mat.x;
            const v3 u = normalize_w<true>(d);
            const float cos_t = fminf(dot(neg(u), n), 1.0f);
            const float sin_t = sqrtf(fmaf(-cos_t, cos_t, 1.0f));
            const bool cannot = ratio * sin_t > 1.0f;
            const bool refl = cannot || reflectance(cos_t, ratio) > r_sb;
            nd = normalize_w<true>(refl ? reflect(u, n) : refract(u, n, ratio));
            ndd = dot(nd, nd);
        }
    }
}

// normalize(d).y of the sky (wgsl:293-296) and its colour times cf
__device__ __forceinline__ v3 sky_w(v3 cf, v3 d, float dd) {
    float uy;
    if (rt_ballot(__float_as_uint(dd) - kBits2m20 >= kBits2p40 - kBits2m20) == 0ull) {
        float y;
        const float len = sqrt_core_rcp(dd, y);
        uy = div_core(d.y, len, y);
    } else {
        uy = d.y / sqrtf(dd);
    }
    const float a = 0.5f * (uy + 1.0f);
    const float om = 1.0f - a;
    return mul(cf, mk(fmaf(a, 0.5f, om), fmaf(a, 0x1.666666p-1f, om), fmaf(a, 1.0f, om)));
}
__device__ __forceinline__ v3 sky_w(v3 cf, v3 d) { return sky_w(cf, d, dot(d, d)); }

// One sample of kSinglePix pixels per lane (get_ray + ray_color at depth <= 1).  seed[s] =
// 1 + n + B (wgsl:353) of pixel s; kUniRs: every live pixel holds the hinted count, and the
// scatter's random numbers come from p.rs.  Tiles: blk[s] = the tile's candidate block,
// ncand[s] its count (kCandNone: the full list; 0 for a tile past the image edge).
template <uint32_t S>
constexpr bool kSingleLds = RT_SINGLE_LDS == 2 || (RT_SINGLE_LDS == 1 && S == 1);
template <uint32_t S, bool kUniRs, typename P>
__device__ __forceinline__ void single_sample(const P& p, const Cam& cam,
                                              const TileCoord (&tc)[S],
                                              const uint32_t (&hxy)[S],
                                              const uint32_t (&seed)[S],
                                              const float4* const (&blk)[S],
                                              const uint32_t (&ncand)[S],
                                              const bool (&live)[S],
                                              const uint64_t (&live_m)[S],
                                              const float4 (&bv)[S], float4* lblk,
                                              v3 (&col)[S]) {
    constexpr int K = 1;    // records per tile and step of the joint list walk
    v3 o[S], d[S];
    // one VGPR copy of the lens centre for the S pixels (get_ray's c0v)
    v3 c0 = cam.center;
    if (S > 1) asm volatile("" : "+v"(c0.x), "+v"(c0.y), "+v"(c0.z));
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {                            // wgsl:311, 305-325
        get_ray<kSingleDisk>(cam, tc[s].x, tc[s].y, hxy[s], seed[s] * 25u + p.seed_b, o[s],
                             d[s], S > 1 ? &c0 : nullptr);
    }
    SST_V(3, d[S - 1].x);
    const uint32_t lane = threadIdx.x & 63u;
    if (kSingleLds<S>) {
        // (this wave's own LDS slots: written and read by this wave only, in order)
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) lblk[s * kCandStride + lane] = bv[s];
    }
    v3 cf[S], dsky[S];
    float ddsky[S];                   // |dsky|^2 (sky_w's dd)
    bool black[S], any_other[S];      // (any_other: wave-uniform, a metal / dielectric hit)
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {
        cf[s] = mk(1.0f, 1.0f, 1.0f);
        dsky[s] = d[s];
        ddsky[s] = dot(d[s], d[s]);   // (wgsl:184's a as well)
        black[s] = false;
        any_other[s] = false;
    }
    if (p.depth != 0u) {                                          // wgsl:264
        // sphere_list_hit over each tile's list, the tiles' chunks interleaved
        float tmax[S], a[S];
        int idx[S];
        bool joint = true;
        uint32_t m = 0;
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) {
            tmax[s] = 0x1.05ed2ep+118f;                           // 3.4e35 (wgsl:266)
            idx[s] = -1;
            a[s] = ddsky[s];
            joint = joint && ncand[s] != kCandNone;
            m = max(m, ncand[s]);
        }
        if (joint) {
            // (walking the common length jointly and the longer list's rest alone measured
            // neutral: profiles/r06/r06av/)
            for (uint32_t i = 0; i < m; i += K) {
                float hh[S][K], dd[S][K];
                // "some discriminant of the step is not negative" as the sign of the AND of
                // their bit patterns (one 2-cycle v_and per record): exact on the camera-ray
                // domain the host proves for these instances — every discriminant is finite
                // (consider_fast) and never -0 (max_bits), so its sign bit is set exactly when
                // it is < 0
                uint32_t an = 0xFFFFFFFFu;
#pragma unroll
                for (uint32_t s = 0; s < S; ++s)
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const float4 g =
                            kSingleLds<S> ? lblk[s * kCandStride + kCandRecOff + i + k]
                                          : load_rec<true>(blk[s] + kCandRecOff, i + k);
                        dd[s][k] = discriminant(g, o[s], d[s], a[s], hh[s][k]);
                        an &= __float_as_uint(dd[s][k]);
                    }
                if (__builtin_expect((int)an >= 0, 0)) {
#pragma unroll
                    for (uint32_t s = 0; s < S; ++s)
#pragma unroll
                        for (int k = 0; k < K; ++k)
                            if (i + k < ncand[s])
                                // (1 / a only where some discriminant is not negative:
                                // waves without candidates, the sky's, skip the v_rcp)
                                consider_fast(dd[s][k], hh[s][k], a[s], rcp_refined(a[s]), i + k, tmax[s],
                                              idx[s]);
                }
            }
        } else {
#pragma unroll
            for (uint32_t s = 0; s < S; ++s) {
                const bool listed = ncand[s] != kCandNone;
                const Hit h = scan_exhaustive<K, true, true>(
                    listed ? blk[s] + kCandRecOff : p.geom, listed ? ncand[s] : p.count, o[s],
                    d[s]);
                idx[s] = h.idx;
                tmax[s] = h.t;
            }
        }
        SST_V(4, tmax[S - 1]);
        // hit records and the scatter (wgsl:205-218, 268-286)
        bool hit[S];
        bool any = false;
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) {
            hit[s] = live[s] && idx[s] >= 0;
            any = any || hit[s];
        }
        uint64_t hm[S], any_m = 0;
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) {
            hm[s] = mask_sge(idx[s], 0) & live_m[s];
            any_m |= hm[s];
        }
        if (any_m != 0ull) {
            float4 pr[S], mat[S];
#pragma unroll
            for (uint32_t s = 0; s < S; ++s) {
                const uint32_t j = hit[s] ? (uint32_t)idx[s] : 0u;
                if (kSingleLds<S> && ncand[s] != kCandNone) {
                    pr[s] = lblk[s * kCandStride + kCandSphOff + 2u * j];
                    mat[s] = lblk[s * kCandStride + kCandSphOff + 2u * j + 1u];
                } else {
                    // the wave-uniform record array as a buffer, the lane's 32-bit byte offset
                    // (j < 2^20 spheres, rt_abi.cpp kMaxSpheres): no 64-bit address arithmetic
                    // per lane
                    const float4* hs = ncand[s] != kCandNone ? blk[s] + kCandSphOff : p.sph;
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        (void*)hs, 0, (int)0x7FFFFFFF, 0x00020000);
                    pr[s] = buf_f4(rs, j * 32u);
                    mat[s] = buf_f4(rs, j * 32u + 16u);
                }
            }
#pragma unroll
            for (uint32_t s = 0; s < S; ++s) {
                float r_sb;
                v3 ruv;
                if (kUniRs) {
                    r_sb = p.rs.x;
                    ruv = mk(p.rs.y, p.rs.z, p.rs.w);
                } else {
                    const uint32_t sb = hash(seed[s] + 1u);       // wgsl:268, 355 (i = 0)
                    r_sb = rf(sb);
                    ruv = random_unit_vector(r_sb, sb);
                }
                v3 nd, att;
                bool blk_s, other_s;
                float ndd;
                shade_hit(pr[s], mat[s], tmax[s], o[s], d[s], r_sb, ruv, hit[s], hm[s],
                          p.normal_rn != 0u, nd, att, blk_s, other_s, ndd);
                any_other[s] = other_s;
                if (hm[s] == live_m[s]) {
                    // every live lane hit (a tile inside a sphere's image): no selects
                    asm volatile("");
                    cf[s] = att;
                    dsky[s] = nd;
                    ddsky[s] = ndd;
                    black[s] = blk_s;
                } else if (hit[s]) {                              // wgsl:285-286
                    cf[s] = att;
                    dsky[s] = nd;
                    ddsky[s] = ndd;
                    black[s] = blk_s;
                }
            }
        }
    }
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {
        const v3 c = sky_w(cf[s], dsky[s], ddsky[s]);             // wgsl:293-296
        // (black: only metal hits absorb, so only a wave that shaded one selects)
        if (!any_other[s]) {
            asm volatile("");
            col[s] = c;
        } else {
            col[s] = black[s] ? mk(0.0f, 0.0f, 0.0f) : c;         // wgsl:277-279
        }
    }
    SST_V(5, col[S - 1].x);
}

// kReset: the frame resets the accumulator (camera_has_moved > 0.5, wgsl:345-350) — a
// separate kernel (rt_single_reset_kernel), so that the steady-state kernel carries no
// per-pixel selects between the loaded and the zero accumulator, and the reset kernel no
// accumulator load at all.
template <int kPix, bool kReset, bool kChain>
__device__ __forceinline__ void single_body(
    const float4* __restrict__ a_cand, const uint32_t* __restrict__ a_hx,
    const float4* __restrict__ a_in, uint32_t a_width, uint32_t a_height, uint32_t a_bands,
    const uint32_t* __restrict__ a_order, const SingleParams& p) {
    static_assert(kPix >= 1 && kPix <= 4, "1 to 4 tiles per wave");
    constexpr uint32_t S = kPix;
    WAVE_TRACE(0);
#if RT_SSTAMPS
    sst_put(8, __builtin_amdgcn_s_memrealtime());
    sst_put(0, __builtin_amdgcn_s_memtime());
#endif
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tiles_x = (a_width + 7u) >> 3;
    // frame chains: a segment whose go wait gave up drops its image stores (the frames must
    // not run before the caller's stream reached them; rt_chain_go_kernel)
    // (a system-scope load: no cache between it and the go kernel's store; waited for only
    // at the stores)
    const uint32_t aborted =
        kChain ? __builtin_amdgcn_readfirstlane(
                     __hip_atomic_load(p.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
               : 0u;
    // workgroups by decreasing candidate-list load (wg_order, launch_wg_order): the
    // costliest are dispatched first and the cheap ones fill the tail
    uint32_t gx = blockIdx.x, lband = (p.lbands & 0xFFFFu) + blockIdx.y * (p.lbands >> 16);
    if (a_order) {   // (a leading, preloadable argument: one scalar load to the entry)
        const uint32_t pos = blockIdx.y * (kChain ? p.grid_x : gridDim.x) + blockIdx.x;
        const uint32_t e = __builtin_amdgcn_readfirstlane(a_order[pos]);
        gx = e & 0xFFFFu;
        lband = e >> 16;
    }
    SST_S(1, lband);
    const uint32_t tx0 = (gx * kSingleWg + wave) * S;
    const uint32_t band_first = a_bands & 0xFFFFu, band_step = (a_bands >> 16) & 0x7FFFu;
    TileCoord tc[S];
    uint32_t ncand[S], hxy[S];
    const float4* blk[S];
    float4 acc[S], bv[S];
    __shared__ float4 s_blk[kSingleWg * kPix * kCandStride];
    float4* lblk = s_blk + wave * S * kCandStride;
    constexpr bool kHash = (RT_SINGLE_HASH >> (kPix - 1)) & 1;
    uint32_t hy = 0u, hv = 0u;
    if (kHash) {
        // (all 64 lanes active here: ds_bpermute reads every lane)
        const uint32_t row = (band_first + lband * band_step) * RT_STRIPE_ROWS + lane - 8u * S;
        const bool col = lane < 8u * S;                           // (selects, no branch)
        hv = hash((col ? tx0 * 8u + lane : row) * (col ? 73u : 51u));    // wgsl:309-310
        hy = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((8u * S + (lane >> 3)) * 4u), (int)hv);
    } else {
        hy = a_hx[p.hy_off + min(band_first * RT_STRIPE_ROWS +
                                     lband * band_step * RT_STRIPE_ROWS + (lane >> 3),
                                 a_height - 1u)];
    }
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {
        const uint32_t tx = tx0 + s;
        const bool in = tx < tiles_x;
        const uint32_t tile = lband * tiles_x + (in ? tx : tx0);
        tc[s] = tile_coord(a_width, a_height, band_first, band_step, tx, lband, lane);
        blk[s] = a_cand + (size_t)tile * kCandStride;
        ncand[s] = in ? load_cnt(a_cand, tile) : 0u;
        const uint32_t hx =
            kHash ? (uint32_t)__builtin_amdgcn_ds_bpermute((int)((8u * s + (lane & 7u)) * 4u),
                                                           (int)hv)
                  : a_hx[min(tc[s].x, a_width - 1u)];
        hxy[s] = hx ^ hy;                                         // wgsl:309-310
    }
    uint64_t valid_m[S];        // (tc[s].valid as a lane mask)
#pragma unroll
    for (uint32_t s = 0; s < S; ++s)
        valid_m[s] = mask_ult(tc[s].x, a_width) & mask_ult(tc[s].y, a_height);
    // (issued after the seed-table loads: vmcnt waits in issue order, and the camera rays
    // need the seeds long before the scan and the accumulation need these)
#pragma unroll
    for (uint32_t s = 0; s < S; ++s)
        bv[s] = (kSingleLds<S> && tx0 + s < tiles_x) ? blk[s][lane]
                                                      : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    // Frame chains (rt_chain.cpp): consecutive frames of a part are AQL packets with no
    // cache acquire between them, so the accumulator the previous frame stored (write-
    // through, sc1) is read with sc1 loads: this CU's L1 may hold lines of an older frame.
    if (kChain && !kReset) {
        const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
            (void*)a_in, 0, (int)0x7FFFFFFF, 0x00020000);
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                rin, (int)((tc[s].valid ? tc[s].idx : 0) * 16u), 0, 16);   // sc1, wgsl:339
            acc[s] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y),
                                 __uint_as_float(v.z), __uint_as_float(v.w));
        }
    } else {
#pragma unroll
        for (uint32_t s = 0; s < S; ++s)
            acc[s] = kReset ? make_float4(0.0f, 0.0f, 0.0f, 0.0f)   // (discarded: no load)
                            : a_in[tc[s].valid ? tc[s].idx : 0];            // wgsl:339
    }
    if (tx0 >= tiles_x) return;
    SST_V(2, hxy[S - 1]);
    SST_S(2, ncand[S - 1]);

    Cam cam;
    cam.center = mk(p.center[0], p.center[1], p.center[2]);
    cam.vul = mk(p.vul[0], p.vul[1], p.vul[2]);
    cam.pdu = mk(p.pdu[0], p.pdu[1], p.pdu[2]);
    cam.pdv = mk(p.pdv[0], p.pdv[1], p.pdv[2]);
    cam.ddu = mk(p.ddu[0], p.ddu[1], p.ddu[2]);
    cam.ddv = mk(p.ddv[0], p.ddv[1], p.ddv[2]);
    cam.defocus_angle = p.defocus_angle;
    const uint32_t spp = p.spp;                                   // wgsl:343

    v3 c[S];
    uint32_t n[S];
    bool pending[S];
    bool any_pending = true;
    uint64_t pend_m = 0;        // (the lanes with pending pixels)
    if (p.hinted) {
        // Every pixel is expected to hold n_hint (the host's count bookkeeping): trace with
        // it while the accumulator loads are in flight, then verify.
        const uint32_t ng = p.n_hint;
        v3 col[S];
        if (ng < spp) {                                           // wgsl:352
            uint32_t seed[S];
            bool live[S];
#pragma unroll
            for (uint32_t s = 0; s < S; ++s) {
                seed[s] = 1u + ng + p.seed_b;                     // wgsl:353
                live[s] = tc[s].valid;
            }
            single_sample<S, true>(p, cam, tc, hxy, seed, blk, ncand, live, valid_m, bv, lblk,
                                   col);
        }
        any_pending = false;
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) {
            c[s] = kReset ? mk(0.0f, 0.0f, 0.0f) : mk(acc[s].x, acc[s].y, acc[s].z);
            n[s] = kReset ? 0u : f2u(acc[s].w);                   // wgsl:339-350
            pending[s] = tc[s].valid && n[s] != ng;               // a foreign count
            if (!kReset) pend_m |= mask_ne(n[s], ng) & valid_m[s];
            any_pending = any_pending || pending[s];
            if (ng < spp) {                                       // wgsl:352-357
                const v3 num = sub(col[s], c[s]);
                if (ng < kAccRnMax &&
                    (mask_ult(acc_min_bits(num), kAccOkDbl) & valid_m[s]) == 0ull) {
                    c[s] = acc_rn(c[s], num, (float)(ng + 1u), p.rcp_hint);
                } else {
                    const float k = (float)(ng + 1u);             // wgsl:356
                    c[s] = mk(c[s].x + num.x / k, c[s].y + num.y / k, c[s].z + num.z / k);
                }
                n[s] = ng + 1u;
            }
        }
    } else {
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) {
            pending[s] = tc[s].valid;
            pend_m |= valid_m[s];
        }
    }
    const bool wave_pending = pend_m != 0ull;
    if (wave_pending) {
        // pixels whose count is not the hinted one (or no hint): traced with their own
        // count and per-pixel random numbers
        uint32_t seed[S];
        bool live[S];
        v3 col[S];
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) {
            if (pending[s]) {
                c[s] = kReset ? mk(0.0f, 0.0f, 0.0f) : mk(acc[s].x, acc[s].y, acc[s].z);
                n[s] = kReset ? 0u : f2u(acc[s].w);
            }
            live[s] = pending[s] && n[s] < spp;                   // wgsl:352
            seed[s] = 1u + n[s] + p.seed_b;                       // wgsl:353
        }
        uint64_t live_m[S];
#pragma unroll
        for (uint32_t s = 0; s < S; ++s) live_m[s] = rt_ballot(live[s]);
        single_sample<S, false>(p, cam, tc, hxy, seed, blk, ncand, live, live_m, bv, lblk, col);
#pragma unroll
        for (uint32_t s = 0; s < S; ++s)
            if (live[s]) {                                        // wgsl:356-357
                const float k = (float)(n[s] + 1u);
                c[s] = mk(c[s].x + (col[s].x - c[s].x) / k, c[s].y + (col[s].y - c[s].y) / k,
                          c[s].z + (col[s].z - c[s].z) / k);
                n[s] += 1u;
            }
    }
    SST_V(6, c[S - 1].x);
    // write-through (sc1) stores: the lines leave the XCD's L2 as they are written, so the
    // launch ends with no dirty image lines to write back at the kernel boundary
    float4* band = p.out + (size_t)lband * RT_STRIPE_ROWS * a_width;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        band, 0, (int)(RT_STRIPE_ROWS * 16u * a_width), 0x00020000);
#pragma unroll
    for (uint32_t s = 0; s < S; ++s)
    {                                                             // wgsl:362-363
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = {__float_as_uint(c[s].x), __float_as_uint(c[s].y),
                             __float_as_uint(c[s].z), __float_as_uint((float)n[s])};
            // no branch: a pixel past the image edge stores to an offset past the band's
            // buffer record, which the buffer unit drops
            const uint32_t off = ((lane >> 3) * a_width + tc[s].x) * 16u;
            const bool drop = !tc[s].valid || (kChain && aborted != 0u);
            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, (int)(drop ? 0x7FFFFFF0u : off), 0,
                                                   16);
        }
#if RT_SSTAMPS
    sst_put(7, __builtin_amdgcn_s_memtime());
    sst_put(9, __builtin_amdgcn_s_memrealtime());
    sst_put(10, __builtin_amdgcn_s_getreg((31 << 11) | 4));    // HW_ID
    sst_put(11, __builtin_amdgcn_s_getreg((31 << 11) | 20));   // XCC_ID
#endif
    WAVE_TRACE(1);
}

template <int kPix>
__global__ __launch_bounds__(64 * kSingleWg, RT_SINGLE_MIN_WAVES) void rt_single_kernel(
    const float4* __restrict__ a_cand, const uint32_t* __restrict__ a_hx,
    const float4* __restrict__ a_in, uint32_t a_width, uint32_t a_height, uint32_t a_bands,
    const uint32_t* __restrict__ a_order, const SingleParams p) {
    single_body<kPix, false, false>(a_cand, a_hx, a_in, a_width, a_height, a_bands, a_order, p);
}
template <int kPix>
__global__ __launch_bounds__(64 * kSingleWg, RT_SINGLE_MIN_WAVES) void rt_single_reset_kernel(
    const float4* __restrict__ a_cand, const uint32_t* __restrict__ a_hx,
    const float4* __restrict__ a_in, uint32_t a_width, uint32_t a_height, uint32_t a_bands,
    const uint32_t* __restrict__ a_order, const SingleParams p) {
    single_body<kPix, true, false>(a_cand, a_hx, a_in, a_width, a_height, a_bands, a_order, p);
}
// The same kernels for frame chains (rt_chain.cpp: one AQL packet per frame and part on
// context-owned HSA queues; accumulator loads sc1, see single_body).
template <int kPix>
__global__ __launch_bounds__(64 * kSingleWg, RT_SINGLE_MIN_WAVES) void rt_chain_kernel(
    const float4* __restrict__ a_cand, const uint32_t* __restrict__ a_hx,
    const float4* __restrict__ a_in, uint32_t a_width, uint32_t a_height, uint32_t a_bands,
    const uint32_t* __restrict__ a_order, const SingleParams p) {
    single_body<kPix, false, true>(a_cand, a_hx, a_in, a_width, a_height, a_bands, a_order, p);
}
template <int kPix>
__global__ __launch_bounds__(64 * kSingleWg, RT_SINGLE_MIN_WAVES) void rt_chain_reset_kernel(
    const float4* __restrict__ a_cand, const uint32_t* __restrict__ a_hx,
    const float4* __restrict__ a_in, uint32_t a_width, uint32_t a_height, uint32_t a_bands,
    const uint32_t* __restrict__ a_order, const SingleParams p) {
    single_body<kPix, true, true>(a_cand, a_hx, a_in, a_width, a_height, a_bands, a_order, p);
}
// A chain's first packet: wait until the caller's stream has reached the chain (its
// hipStreamWriteValue32 of `want` into *go, signal memory).  Bounded by `ticks` of
// s_memrealtime (100 MHz; rt_chain.cpp, default 10 s): a wait that gives up sets *abort
// (device memory: every later chain frame drops its image stores, so no frame runs before
// the caller's stream has reached it) and *gave_up (coherent host memory: the host fails the
// chain on its next call, rt_abi.cpp, and runs HIP launches from then on).  Vector stores.
__global__ __launch_bounds__(64) void rt_chain_go_kernel(const uint32_t* go, uint32_t want,
                                                         uint32_t* abort, uint32_t* gave_up,
                                                         uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        if ((int32_t)(v - want) >= 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            if (threadIdx.x == 0u) {
                __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(gave_up, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}
// A chain's last packet (barrier bit: after every frame): the caller's stream, waiting in
// hipStreamWaitValue32 for `value`, continues.  A release store at system scope: the frames'
// stores are written back before the stream (or a copy engine, or RCCL over xGMI) reads on.
__global__ __launch_bounds__(64) void rt_chain_done_kernel(uint32_t* done, uint32_t value) {
    if (threadIdx.x == 0u)
        __hip_atomic_store(done, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- Frame groups over tile pairs (kTraceListPair2, kTraceListQuad2) -----------------
//
// The frame-group schedule of trace_pair (kFrameGroup waves, wave w traces frames f + w of
// each group, wave 0 accumulates through LDS) with the one-frame kernel's sample: each
// workgroup owns two horizontally adjacent tiles and each lane one pixel of each, the two
// tiles' candidate lists walked jointly (single_sample<2>) — two independent pixel chains per
// lane instead of one, and half the waves for the same work.  Called for launches whose
// every frame is hinted (rt_abi.cpp: the frame-group conditions); a workgroup whose loaded
// counts differ from the hint traces each tile with the general per-tile loop (waves 0 and
// 1).  Scheduling units (tile order, costs): tile pairs.  G: frames per group (2 or 4).
// Waves per SIMD the register plan targets: 7 (71 VGPRs, no scratch) — at 8 the compiler
// fits 64 VGPRs with 40 B of scratch per lane and 69 SGPR spills, and a whole-image 64-frame
// pair launch takes 14.94 against 14.27 us per frame (profiles/r05/r05af/ab_k3_fused.log).
#ifndef RT_TPAIR_MIN_WAVES
#define RT_TPAIR_MIN_WAVES 7
#endif
// single_sample's parameters for one frame of a frame group
struct FrameView {
    const float4* geom;
    const float4* sph;
    uint32_t count, depth, seed_b, normal_rn;
    float4 rs;
};
// (G an int: rocprofv3 lists the instances as rt_tpair_kernel<2> / <4>, rt_kernel_name's names)
template <int G>
__global__ __launch_bounds__(64 * G, RT_TPAIR_MIN_WAVES) void rt_tpair_kernel(
    const float4* __restrict__ a_cand, const uint32_t* __restrict__ a_hx,
    const float4* __restrict__ a_in, uint32_t a_width, uint32_t a_height, uint32_t a_bands,
    const TraceParams p) {
    WAVE_TRACE(0);
    constexpr uint32_t S = 2, Gu = (uint32_t)G;
    static_assert(!kSingleLds<S>, "the pair sample reads its records from the candidate blocks");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tiles_x = (a_width + 7u) >> 3;
    const uint32_t units_x = (tiles_x + S - 1u) / S;
    uint32_t ux = blockIdx.x, lband = blockIdx.y;
    const uint32_t band_first = a_bands & 0xFFFFu, band_step = (a_bands >> 16) & 0x7FFFu;
    if (a_bands >> 31) {                                 // costliest units first (tile_order)
        const uint32_t t =
            __builtin_amdgcn_readfirstlane(p.tile_order[blockIdx.y * gridDim.x + blockIdx.x]);
        ux = t & 0xFFFFu;
        lband = t >> 16;
    }
    const uint32_t unit = lband * units_x + ux;
    const uint32_t tx0 = ux * S;
    TileCoord tc[S];
    uint32_t ncand[S], hxy[S], tile[S];
    const float4* blk[S];
    float4 acc[S];
    uint64_t valid_m[S];
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {
        const uint32_t tx = tx0 + s;
        const bool in = tx < tiles_x;
        tile[s] = lband * tiles_x + (in ? tx : tx0);
        tc[s] = tile_coord(a_width, a_height, band_first, band_step, tx, lband, lane);
        blk[s] = a_cand + (size_t)tile[s] * kCandStride;
        ncand[s] = in ? load_cnt(a_cand, tile[s]) : 0u;
        acc[s] = a_in[tc[s].valid ? tc[s].idx : 0];               // wgsl:339
        hxy[s] = a_hx[min(tc[s].x, a_width - 1u)] ^                // wgsl:309-310
                 a_hx[hy_offset(a_width) + min(tc[s].y, a_height - 1u)];
        valid_m[s] = mask_ult(tc[s].x, a_width) & mask_ult(tc[s].y, a_height);
    }
    if (p.tile_cost && w == 0u && lane == 0u)
        p.tile_cost[unit] = (uint32_t)__builtin_amdgcn_s_memtime();
    const Cam cam = cam_params(p);
    const uint32_t n0 = p.hint_n[0];
    if (!p.reset_first &&
        rt_ballot((tc[0].valid && f2u(acc[0].w) != n0) || (tc[1].valid && f2u(acc[1].w) != n0)) !=
            0ull) {
        // a foreign count: wave s traces tile s frame after frame (stores every image itself)
        if (w < S && tx0 + w < tiles_x) {
            const float4 res = trace_pixel<kTraceListQuad, false>(
                p, cam, w ? tile[1] : tile[0], w ? ncand[1] : ncand[0], w ? tc[1] : tc[0],
                w ? hxy[1] : hxy[0], w ? acc[1] : acc[0]);
            const TileCoord& t = w ? tc[1] : tc[0];
            if (t.valid && !p.store_each) p.out[t.idx] = res;     // wgsl:363
        }
    } else {
        const uint32_t spp = p.spp;                               // wgsl:343
        // the tiles' accumulators stay in LDS between groups (no registers live across the
        // samples; the foreign-count fallback above sets the register peak)
        __shared__ float4 s_cols[2u * Gu * S * 64u];
        __shared__ float4 s_acc[S * 64u];
        if (w == 0u)
#pragma unroll
            for (uint32_t s = 0; s < S; ++s)
                s_acc[s * 64u + lane] = p.reset_first ? make_float4(0.0f, 0.0f, 0.0f, 0.0f)
                                                      : acc[s];
        const float4 zero4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        for (uint32_t f = 0; f < p.frames; f += Gu) {
            const uint32_t fw = f + w;
            // (single_sample writes every lane's colour; zeros only where nothing is traced)
            v3 col[S];
            const uint32_t ng = fw < p.frames ? p.hint_n[fw] : spp;  // count before frame fw
            if (ng >= spp) {
#pragma unroll
                for (uint32_t s = 0; s < S; ++s) col[s] = zero_v3_here();
            } else {                                              // wgsl:352
                {
                    FrameView v;
                    v.geom = p.geom;
                    v.sph = p.sph;
                    v.count = p.count;
                    v.depth = p.depth;
                    v.seed_b = p.seed_b[fw];
                    // (read from the kernarg segment every frame: as a loop invariant the
                    // flag was spilled and turned back into a lane mask per pixel, four VALU)
                    v.normal_rn = p.normal_rn;
                    v.rs = p.hint_rs[fw * p.depth];
                    uint32_t seed[S];
                    bool live[S];
                    const float4 bv[S] = {zero4, zero4};
#pragma unroll
                    for (uint32_t s = 0; s < S; ++s) {
                        seed[s] = 1u + ng + v.seed_b;             // wgsl:353
                        live[s] = tc[s].valid;
                    }
                    // the tiles' list pointers re-derived from the tile indices every frame
                    // (SALU) instead of staying live across the loop: 45 -> 28 SGPRs spilled
                    // to VGPR lanes, 30 -> 14 v_readlane in the loop; K3 13.60 -> 13.37 us per
                    // frame (tools/chain_ab.py, profiles/r06/r06ae/); re-reading the unit and
                    // the counts through the scalar cache every frame instead: 14.17 (r06af/)
                    const float4* blkf[S];
                    uint32_t ncf[S];
#pragma unroll
                    for (uint32_t s = 0; s < S; ++s) {
                        uint32_t t = tile[s], nc = ncand[s];
                        asm volatile("" : "+s"(t), "+s"(nc));
                        blkf[s] = a_cand + (size_t)t * kCandStride;
                        ncf[s] = nc;
                    }
                    single_sample<S, true>(v, cam, tc, hxy, seed, blkf, ncf, live, valid_m, bv,
                                           nullptr, col);
                }
            }
            // two LDS slots alternating by group (one barrier per group, as trace_pair): wave w
            // leaves its colour of tile t (frame f + w) in slot [w][t] unless it accumulates
            // that tile itself; wave t (< S) accumulates tile t's G frames in frame order —
            // the tiles' accumulation on two waves instead of all of it on wave 0.  The colours
            // as 12-B records (ds_write_b96: no register quad to fill with a zero).
            float4* slot = s_cols + ((f / Gu) & 1u) * Gu * S * 64u;
#pragma unroll
            for (uint32_t t = 0; t < S; ++t)
                if (w != t)
                    *reinterpret_cast<f3v*>(&slot[(w * S + t) * 64u + lane]) =
                        f3v{col[t].x, col[t].y, col[t].z};
            __syncthreads();
#pragma unroll
            for (uint32_t t = 0; t < S; ++t) {
                if (w != t) continue;                             // (wave-uniform)
#pragma unroll
                for (uint32_t j = 0; j < Gu; ++j) {
                    const uint32_t fj = f + j;
                    if (fj >= p.frames) break;
                    const uint32_t nb = p.hint_n[fj];             // count before frame fj
                    const bool acc_frame = nb < spp;              // wgsl:352-358
                    // f32(nb + 1) (the divisor k, wgsl:356) or f32(nb): the host's table
                    const float cnt = p.hint_cnt[fj];
                    float4* out = (fj & 1u) ? p.out2 : p.out;
                    const bool store = p.store_each == 2u || fj + 2u >= p.frames;
                    const float4 ca = s_acc[t * 64u + lane];
                    v3 cs = mk(ca.x, ca.y, ca.z);
                    v3 cj = col[t];
                    if (j != t) {
                        const float4 c4 = slot[(j * S + t) * 64u + lane];
                        cj = mk(c4.x, c4.y, c4.z);
                    }
                    if (acc_frame) {
                        const v3 num = sub(cj, cs);
                        // num / f32(nb + 1) (wgsl:356) as a Markstein division (acc_rn)
                        // (both conditions scalar, combined without a branch: a short-
                        // circuit && here kept nb's test in a VGPR)
                        const bool rn = (nb < kAccRnMax) &
                                        ((mask_ult(acc_min_bits(num), kAccOkDbl) &
                                          valid_m[t]) == 0ull);
                        if (rn) {
                            cs = acc_rn(cs, num, cnt, p.hint_rcp[fj]);
                        } else {
                            const float k = cnt;                     // wgsl:356
                            cs = mk(cs.x + num.x / k, cs.y + num.y / k, cs.z + num.z / k);
                        }
                    }
                    // (the alpha rides in the LDS copy: one register quad serves the LDS
                    // write and the image store)
                    const float4 v = make_float4(cs.x, cs.y, cs.z, cnt);
                    s_acc[t * 64u + lane] = v;
                    // wgsl:362-363: the images that survive (or every frame's)
                    if (store && tc[t].valid) out[tc[t].idx] = v;
                }
            }
        }
    }
    if (p.tile_cost && w == 0u && lane == 0u)
        p.tile_cost[unit] = (uint32_t)__builtin_amdgcn_s_memtime() - p.tile_cost[unit];
    WAVE_TRACE(1);
}

// ---- Bounce paths with workgroup-wide compaction (kTraceBounce) -----------------------
//
// rt_update_frames with bounce rays (max_depth >= 2), several frames per launch.  One
// workgroup = kBounceWaves waves = kBounceWaves consecutive 8x8 tiles of a stripe band; each
// lane owns one pixel and keeps its accumulator in registers across the launch's frames.
// Per frame the camera rays of a wave are its own tile's (candidate list or cone scan, as
// in the culled instance).  After every bounce the paths still alive in the workgroup are
// compacted: a ballot per wave, the popcounts combined through LDS into wave offsets, and
// mbcnt gives each live lane its slot; the path state (origin, direction, throughput, seed,
// owner) goes to LDS slot `prefix`, and the next bounce is traced by the first
// ceil(live / 64) waves only — the others wait at the barrier, their SIMD time free for
// other workgroups.  A path that ends (sky, absorbed, depth exhausted) writes its colour to
// its owner's LDS result slot; the owner accumulates it after the frame (wgsl:352-363).
// Every path runs exactly the reference's per-pixel arithmetic (ray_color, wgsl:261-297):
// only which lane executes it changes.  kBounceWaves = 4: a bounce's live paths of four
// tiles fill one wave where they filled four (K5: path lengths fall off geometrically, the
// longest of 64 lanes sets a wave's bounce count without compaction).
constexpr uint32_t kBounceLanes = 64 * kBounceWaves;
struct BounceLds {
    float4 po[kBounceLanes];   // origin, seed + 1 (bits) of the path in slot k
    float4 pd[kBounceLanes];   // direction, owner lane (bits)
    float4 pc[kBounceLanes];   // throughput
    float4 res[kBounceLanes];  // colour of the path owned by lane k
    uint32_t cnt[kBounceWaves];
};
__shared__ BounceLds s_bounce;


// One bounce of a path after its hit (wgsl:205-218 record, wgsl:268-286 scatter): the new
// direction and attenuation, or false when the metal scatter absorbs it.
struct Scatter {
    v3 hp, nd, att;
    bool ok;   // false: the metal scatter absorbed the path
};
// The divisions and square roots run on the exact fast cores where a wave-wide check of
// their operands allows (the camera-ray instances' checks, same bits): the normal's
// (p - C) / R by normal_div when every hit lane has |R| in [2^-20, 2^20] and its three
// numerators in [2^-100, 2^60] (div_core's domain; normal_rn: the scene's radii passed the
// one-step check), the metal / dielectric normalisations by normalize_w<true>.  (The
// dielectric's 1 / ir, reflectance division and square roots on the cores too measured
// neutral, K5 21.53 against 21.56 ms, and stay IEEE: profiles/r06/r06p/.)
__device__ __forceinline__ Scatter scatter_path(float4 pr, float4 mat, float t, v3 o, v3 d,
                                                float r_sb, v3 ruv, bool normal_rn) {
    // (results returned by value: out-parameters through references stayed in scratch)
    const v3 hp = fmas(t, d, o);
    v3 nd, att;
    const v3 rel = sub(hp, mk(pr.x, pr.y, pr.z));
    const uint32_t rel_lo = min(min(abs_bits(rel.x), abs_bits(rel.y)), abs_bits(rel.z));
    const uint32_t rel_hi = max(max(abs_bits(rel.x), abs_bits(rel.y)), abs_bits(rel.z));
    const bool nfast = rel_lo >= kBits2m100 && rel_hi <= 0x5D800000u &&            // 2^60
                       abs_bits(pr.w) - kBits2m20 <= 0x49800000u - kBits2m20;      // 2^20
    v3 outward;                                                                    // wgsl:209
    if (rt_ballot(!nfast) == 0ull)
        outward = normal_div(rel, pr.w, rcp_refined(pr.w), normal_rn);
    else
        outward = divs(rel, pr.w);
    const bool front = dot(d, outward) < 0.0f;
    // (component selects: a select of whole v3 values made the compiler keep them in
    // scratch memory)
    const v3 n = sel3(front, outward, neg(outward));
    if (mat.w < -1.0f) {                                      // lambertian wgsl:84-93
        const v3 dir = add(n, ruv);
        nd = sel3(dot(dir, dir) < 0x1.0c6f7ap-20f, n, dir);
        att = mk(mat.x, mat.y, mat.z);
    } else if (mat.w <= 1.0f) {                               // metal wgsl:95-100
        const v3 refl = fmas(mat.w, ruv, normalize_w<true>(reflect(d, n)));
        if (!(dot(refl, n) > 0.0f)) return Scatter{hp, d, d, false};   // wgsl:277-279
        nd = normalize_w<true>(refl);
        att = mk(mat.x, mat.y, mat.z);
    } else {                                                  // dielectric wgsl:102-135
        att = mk(1.0f, 1.0f, 1.0f);
        const float ratio = front ? 1.0f / mat.x : mat.x;
        const v3 u = normalize_w<true>(d);
        const float cos_t = fminf(dot(neg(u), n), 1.0f);
        const float sin_t = sqrtf(fmaf(-cos_t, cos_t, 1.0f));
        const bool cannot = ratio * sin_t > 1.0f;
        const bool refl = cannot || reflectance(cos_t, ratio) > r_sb;
        nd = normalize_w<true>(sel3(refl, reflect(u, n), refract(u, n, ratio)));
    }
    return Scatter{hp, nd, att, true};
}

// Sky colour of the final direction times the throughput (wgsl:293-296).
__device__ __forceinline__ v3 sky(v3 cf, v3 d) {
    const float uy = d.y / sqrtf(dot(d, d));
    const float a = 0.5f * (uy + 1.0f);
    const float om = 1.0f - a;
    return mul(cf, mk(fmaf(a, 0.5f, om), fmaf(a, 0x1.666666p-1f, om), fmaf(a, 1.0f, om)));
}

// Workgroup-wide prefix of `live` over the kBounceWaves waves: returns this lane's slot
// (valid when live) and the total.  Two barriers (counts written, counts read).
__device__ __forceinline__ uint32_t compact_slot(bool live, uint32_t wave, uint32_t& total) {
    const unsigned long long m = rt_ballot(live);
    if ((threadIdx.x & 63u) == 0u) s_bounce.cnt[wave] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    uint32_t before = 0, sum = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBounceWaves; ++w) {
        const uint32_t c = s_bounce.cnt[w];
        before += w < wave ? c : 0u;
        sum += c;
    }
    total = sum;
    return before + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Register plan of the bounce instance.  The camera (per frame) and the grid parameters (per bounce scan) are re-read from the kernarg segment through a pointer
// the compiler cannot see through (scalar-cache hits), instead of staying live in SGPRs for
// the whole launch; with it a 7-wave plan fits 94 SGPRs (106 and 6 waves before).  K5 per
// 64-spp step (profiles/r03/r03f_ab_k5.log, two rounds): 31.3 ms as before, 29.7 reloading at 6
// waves, 28.8 reloading at 7 (the default), 30.2 at 8 (78 SGPRs, 53 spilled to VGPR lanes),
// 30.5 at 7 without reloading (81 spilled).
#ifndef RT_BOUNCE_MIN_WAVES
#define RT_BOUNCE_MIN_WAVES 7
#endif
// RT_BOUNCE_PRIO: the first RT_BOUNCE_PRIO workgroups of the cost order run at raised wave
// priority (s_setprio), 0 = off.  K5 per-rank prediction (profiles/r03/r03m_rank_sim_k5_*: two
// rounds of five 64-frame launches each, the same frames for every build): 8-rank share
// 74.7 µs per spp off, 72.6 with 512 (efficiency 0.745 -> 0.769), 73.5 with 2048; the
// whole image unchanged (445 µs per spp).
#ifndef RT_BOUNCE_PRIO
#define RT_BOUNCE_PRIO 512
#endif
__device__ __forceinline__ const kconst TraceParams* karg_bounce_params() {
    // rt_bounce_kernel's only argument: the TraceParams block at kernarg offset 0
    const kconst TraceParams* q =
        (const kconst TraceParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));
    return q;
}
// Modes: kBounceWave — one-wave workgroups (one tile each: the finest unit for the
// cost-ordered schedule) whose paths stay in their lanes, colours in registers, no
// barriers; kBounceCompact — four-wave workgroups exchanging paths through LDS (above);
// kBouncePair — two waves per tile on alternate frames, wave 1 handing its colours to wave
// 0 through LDS, which accumulates both in order (the frame groups of the camera-ray
// instance, trace_pair): half as long a chain per wave, for small per-rank shares;
// kBounceSplit — one-wave workgroups, each tile's frames split into p.split consecutive
// chunks traced by separate waves (units (tile, chunk), the costliest tiles' chunks first):
// a chunk stores its frames' colours write-through, the wave whose arrival is the tile's
// last accumulates all of them in frame order (wgsl:352-363) and stores the images.  Small
// rank shares (a few waves per SIMD in per-wave mode) then run S times as many, S times
// shorter waves, so the launch no longer ends with SIMDs idle behind the costliest tiles'
// 64-frame chains.
constexpr int kBounceWave = 0, kBounceCompact = 1, kBouncePair = 2, kBounceSplit = 3;
template <int kMode>
constexpr uint32_t bounce_waves() {
    return kMode == kBounceCompact ? kBounceWaves : kMode == kBouncePair ? 2u : 1u;
}
__shared__ float4 s_pair_col[64];   // kBouncePair: wave 1's colours of the current pair
template <int kMode>
__global__ __launch_bounds__(64 * bounce_waves<kMode>(), RT_BOUNCE_MIN_WAVES) void
rt_bounce_kernel(const TraceParams p) {
    WAVE_TRACE(0);
    constexpr bool kCompact = kMode == kBounceCompact, kPair = kMode == kBouncePair;
    constexpr bool kSplit = kMode == kBounceSplit;
    constexpr uint32_t kW = bounce_waves<kMode>();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = kW == 1u ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t me = threadIdx.x;                    // lane in the workgroup
    const uint32_t tiles_x = (p.width + 7u) >> 3;
    uint32_t gx = blockIdx.x, lband = blockIdx.y;       // group of kW tiles
    // kSplit: workgroup u = unit; the first p.split_tiles slots of the order (the costliest
    // tiles) run as p.split chunks each (slot u / S, chunk u % S), every later slot as one
    // unit (S = 1: the per-wave schedule); a one-dimensional grid of tiles + split_tiles *
    // (S - 1) units
    const uint32_t unit = blockIdx.y * gridDim.x + blockIdx.x;
    uint32_t S = 1u, chunk = 0u, slot = unit;
    bool ordered_units = false;
    if (kSplit && p.unit_order) {
        // the measured unit order (launch_unit_order): the costliest tiles split, every unit
        // placed by its own cost; the grid's units past the count exit at once
        if (unit >= __builtin_amdgcn_readfirstlane(*p.unit_count)) return;
        const uint32_t e = __builtin_amdgcn_readfirstlane(p.unit_order[unit]);
        gx = e & 0xFFFFu;
        lband = (e >> 16) & 0xFFFu;
        chunk = (e >> 28) & 7u;
        S = (e >> 31) ? p.split : 1u;
        ordered_units = true;
    } else if (kSplit) {
        const uint32_t su = p.split_tiles * p.split;
        if (unit < su) {
            S = p.split;
            slot = unit / S;
            chunk = unit % S;
        } else {
            slot = unit - su + p.split_tiles;
        }
        gx = slot % tiles_x;
        lband = slot / tiles_x;
    }
    const bool sp = kSplit && S > 1u;                   // (wave-uniform)
    if (p.tile_order && !ordered_units) {               // costliest groups first
        const uint32_t pos = slot;
        const uint32_t t = __builtin_amdgcn_readfirstlane(p.tile_order[pos]);
        gx = t & 0xFFFFu;
        lband = t >> 16;
#if RT_BOUNCE_PRIO
        // the costliest tiles' waves carry the launch's critical path (a small rank
        // share's launch lasts as long as its heaviest tile's frames): they win the
        // SIMD's instruction arbitration over the cheap waves that fill around them
        if (pos < RT_BOUNCE_PRIO) __builtin_amdgcn_s_setprio(2);
#endif
    }
    const uint32_t tx = kPair ? gx : gx * kW + wave;   // (pairs: both waves, one tile)
    const bool wave_in = tx < tiles_x;
    const TileCoord tc = tile_coord(p, wave_in ? tx : 0u, lband, lane);
    const bool valid = wave_in && tc.valid;
    if (p.lds_records) {                                // records for the cone culling
        for (uint32_t j = threadIdx.x; j < p.lds_records; j += 64u * kW) lds_recs[j] = p.geom[j];
    }
    constexpr uint32_t kTiles = kPair ? 1u : kW;        // tiles per workgroup
    const uint32_t group = lband * ((tiles_x + kTiles - 1u) / kTiles) + gx;
    if (p.tile_cost && threadIdx.x == 0u && chunk == 0u)
        p.tile_cost[group] = (uint32_t)__builtin_amdgcn_s_memtime();
    if (p.lds_records || kW > 1u) __syncthreads();
    const uint32_t tile = lband * tiles_x + (wave_in ? tx : 0u);
    const uint32_t ncand = (p.cand_k && wave_in) ? load_cnt(p.cand, tile) : kCandNone;
    const float4* blk = p.cand + (size_t)tile * kCandStride;
    const uint32_t hxy = p.hx[min(tc.x, p.width - 1u)] ^ p.hy[min(tc.y, p.height - 1u)];
    const uint32_t spp = p.spp, depth = p.depth;        // wgsl:343, 264
    // the pixel's accumulator (wgsl:339-341; a frame-0 reset discards it)
    v3 c = mk(0.0f, 0.0f, 0.0f);
    uint32_t n = 0u;
    if (!p.reset_first && valid) {
        const float4 acc = p.in[tc.idx];
        c = mk(acc.x, acc.y, acc.z);
        n = f2u(acc.w);
    }
    constexpr uint32_t kStep = kPair ? 2u : 1u;               // frames per iteration
    // kSplit: this chunk's frames [f_lo, f_hi), and the pixel's count before f_lo (the
    // count arithmetic of wgsl:345-362 over the frames before it, f32 round trip included)
    uint32_t f_lo = 0u, f_hi = p.frames;
    // kSplit: chunk 0 accumulates its frames in registers when none of them stores an image
    // (an image store of an early frame may go to the input buffer, p.out2, which the later
    // chunks read at their start); otherwise it stores colours like the others
    const uint32_t cs = sp ? (p.frames + S - 1u) / S : p.frames;
    const bool c0_regs = sp && cs < p.frames && p.store_each != 2u &&
                         !(p.store_each && p.frames - 2u < cs);
    if (sp) {
        f_lo = min(chunk * cs, p.frames);
        f_hi = min(f_lo + cs, p.frames);
        for (uint32_t f = 0; f < f_lo; ++f) {
            if (f == 0u && p.reset_first) n = 0u;
            n = f2u((float)(n < spp ? n + 1u : n));
        }
    }
    // (kSplit: this tile's colour rows, one 1-KB row per frame)
    const __amdgpu_buffer_rsrc_t col_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        p.split_col + ((size_t)lband * tiles_x + (wave_in ? tx : 0u)) * p.frames * 64u, 0,
        (int)(p.frames * 1024u), 0x00020000);
    for (uint32_t f0 = f_lo; f0 < f_hi; f0 += kStep) {
        if (f0 == 0 && p.reset_first) {                           // wgsl:345-350
            c = mk(0.0f, 0.0f, 0.0f);
            n = 0u;
        }
        // this wave's frame and the pixel's count before it (pairs: wave 1 takes the next
        // frame, whose count follows from wgsl:352-362 with the f32 round trip)
        const uint32_t f = f0 + (kPair ? wave : 0u);
        const uint32_t n_next = f2u((float)(n < spp ? n + 1u : n));
        const uint32_t nf = (kPair && wave == 1u) ? n_next : n;
        const bool frame_in = f < p.frames;
        const uint32_t B = p.seed_b[frame_in ? f : f0];           // wgsl:311, 353
        const bool sampling = valid && frame_in && nf < spp;      // wgsl:352
        const uint32_t seed = 1u + nf + B;                        // wgsl:353
        // every sampling pixel of the wave at the hinted count of frame f: the scatter's
        // random numbers (pixel-independent given the count) come from hint_rs_dev
        // (compaction moves paths between waves: it keeps computing them)
        const bool uni_rs = !kCompact && f < p.hint_rs_dev_frames &&
                            rt_ballot(sampling && nf != p.hint_n[f]) == 0ull;
        BCOUNT(uni_rs ? 12 : 16);
        v3 res = mk(0.0f, 0.0f, 0.0f);                            // this pixel's colour
        if (kCompact) s_bounce.res[me] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        // bounce 0: this wave's own camera rays (wgsl:305-325), its tile's scan
        v3 o, d, cf = mk(1.0f, 1.0f, 1.0f);
        const Cam cam = cam_params(*karg_bounce_params());
        get_ray<kSingleDisk>(cam, tc.x, tc.y, hxy, seed * 25u + B, o, d);
        uint32_t pseed = seed + 1u;                               // ray_color's seed
        bool live = sampling;
        uint32_t owner = me;
        if (depth == 0u && live) {                                // no bounce: the sky
            res = sky(cf, d);
            if (kCompact) s_bounce.res[me] = make_float4(res.x, res.y, res.z, 0.0f);
        }
        for (uint32_t i = 0; i < depth; ++i) {
            // this wave's paths of bounce i (slot = lane for i == 0)
            Hit hit{-1, 0.0f};
            const float4* hs = p.sph;
            if (rt_ballot(live) != 0ull) {
                const bool listed = i == 0u && ncand != kCandNone;
                BCOUNT(i == 0u ? 6 : 8);
                const GridP gp = grid_params(*karg_bounce_params());
                if (listed) {
                    // the tile's camera rays: consider_fast's roots where the wave is in
                    // their domain (roots_fast_wave), the IEEE ones otherwise
                    if (roots_fast_wave(p.roots_fast, o, dot(d, d), live))
                        hit = scan_exhaustive<RT_BOUNCE_LIST_CHUNK, true, true>(blk + kCandRecOff,
                                                                         ncand, o, d);
                    else
                        hit = scan_exhaustive<RT_BOUNCE_LIST_CHUNK, false, true>(blk + kCandRecOff,
                                                                          ncand, o, d);
                } else {
                    hit = p.lds_records
                              ? scan_culled<true>(gp, p.geom, p.count, o, d, live, i > 0)
                              : scan_culled<false>(gp, p.geom, p.count, o, d, live, i > 0);
                }
                if (listed) hs = blk + kCandSphOff;
            }
            bool done = false, keep = false;
            v3 col = mk(0.0f, 0.0f, 0.0f);
            if (live) {
                if (hit.idx < 0) {                                // wgsl:288-290: sky
                    done = true;
                    col = sky_w(cf, d);
                } else {
                    const float4 pr = hs[2 * hit.idx], mat = hs[2 * hit.idx + 1];
                    // the scatter's random numbers (wgsl:268, 234-243): from the device
                    // table when every path of the wave is at the hinted count
                    float r_sb;
                    v3 ruv;
                    if (uni_rs) {
                        const float4 hr =
                            ((const kconst float4*)p.hint_rs_dev)[f * depth + i];
                        r_sb = hr.x;
                        ruv = mk(hr.y, hr.z, hr.w);
                    } else {
                        const uint32_t sb = hash(pseed + i * 1000u);
                        r_sb = rf(sb);
                        ruv = random_unit_vector(r_sb, sb);
                    }
                    BCOUNT(10);
                    const Scatter sc = scatter_path(pr, mat, hit.t, o, d, r_sb, ruv,
                                                    p.normal_rn != 0u);
                    const v3 hp = sc.hp, nd = sc.nd, att = sc.att;
                    if (!sc.ok) {
                        done = true;                              // absorbed: black
                    } else {
                        cf = mul(cf, att);                        // wgsl:285-286
                        o = hp;
                        d = nd;
                        if (i + 1u == depth) {                    // depth exhausted: sky
                            done = true;
                            col = sky_w(cf, d);
                        } else {
                            keep = true;
                        }
                    }
                }
                if (done) {
                    if (kCompact)
                        s_bounce.res[owner] = make_float4(col.x, col.y, col.z, 0.0f);
                    else
                        res = col;
                }
            }
            if (!kCompact) {                                      // paths stay in their lane
                live = keep;
                if (rt_ballot(keep) == 0ull) break;
                continue;
            }
            // compact the surviving paths into the first slots (uniform trip count)
            uint32_t total;
            const uint32_t slot = compact_slot(keep, wave, total);
            if (keep) {
                s_bounce.po[slot] = make_float4(o.x, o.y, o.z, __uint_as_float(pseed));
                s_bounce.pd[slot] = make_float4(d.x, d.y, d.z, __uint_as_float(owner));
                s_bounce.pc[slot] = make_float4(cf.x, cf.y, cf.z, 0.0f);
            }
            __syncthreads();
            if (total == 0u) break;                               // workgroup-uniform
            live = me < total;
            if (live) {
                const float4 a = s_bounce.po[me], b = s_bounce.pd[me], e = s_bounce.pc[me];
                o = mk(a.x, a.y, a.z);
                pseed = __float_as_uint(a.w);
                d = mk(b.x, b.y, b.z);
                owner = __float_as_uint(b.w);
                cf = mk(e.x, e.y, e.z);
            }
            __syncthreads();                                      // slots read
        }
        if (kCompact) {
            __syncthreads();                                      // results written
            const float4 r = s_bounce.res[me];
            res = mk(r.x, r.y, r.z);
        }
        if (kPair) {                                              // wave 1's colour to wave 0
            if (wave == 1u) s_pair_col[lane] = make_float4(res.x, res.y, res.z, 0.0f);
            __syncthreads();
        }
        if (sp && (chunk != 0u || !c0_regs)) {
            // the frame's colour, write-through (sc1): the tile's last arriver reads it
            // (chunk 0 accumulates its frames in registers, as the per-wave mode does)
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = {__float_as_uint(res.x), __float_as_uint(res.y),
                             __float_as_uint(res.z), 0u};
            __builtin_amdgcn_raw_buffer_store_b128(v, col_rsrc, (int)((f0 * 64u + lane) * 16u),
                                                   0, 16);
            n = f2u((float)(n < spp ? n + 1u : n));
            continue;
        }
        // accumulate this iteration's frames in order (pairs: wave 0 does both; wave 1 only
        // follows the count)
        for (uint32_t j = 0; j < kStep; ++j) {
            const uint32_t fj = f0 + j;
            if (fj >= p.frames) break;
            if (!kPair || wave == 0u) {
                v3 col = res;
                if (kPair && j == 1u) {
                    const float4 r = s_pair_col[lane];
                    col = mk(r.x, r.y, r.z);
                }
                // wgsl:352, 356-357; num / f32(n + 1) as the Markstein step from the host's
                // RN32(1 / f32(n + 1)) (acc_rn) when every accumulating pixel of the wave holds
                // the hinted count (a reset launch's pixels all do), else the IEEE division
                const bool acc = valid && n < spp;
                const v3 num = sub(col, c);
                if (fj < p.hint_acc_frames && p.hint_n[fj] < kAccRnMax &&
                    rt_ballot(acc && (n != p.hint_n[fj] || !acc_ok(num))) == 0ull) {
                    if (acc) c = acc_rn(c, num, (float)(n + 1u), p.hint_rcp[fj]);
                } else if (acc) {
                    const float k = (float)(n + 1u);
                    c = mk(c.x + num.x / k, c.y + num.y / k, c.z + num.z / k);
                }
                // the images of the launch's last two frames survive (wgsl:362-363): frame
                // fj's image belongs to out for even fj, out2 (the input buffer) for odd fj
                // (store_each; 2: every frame's image is stored); otherwise only the last
                // frame's, to out
                if (valid && (fj + 1u == p.frames ||
                              (p.store_each && (p.store_each == 2u || fj + 2u == p.frames)))) {
                    float4* dst = (p.store_each && (fj & 1u)) ? p.out2 : p.out;
                    dst[tc.idx] = make_float4(c.x, c.y, c.z, (float)(n < spp ? n + 1u : n));
                }
            }
            n = f2u((float)(n < spp ? n + 1u : n));
        }
        if (kCompact || kPair) __syncthreads();                   // LDS reused next frame
    }
    if (sp) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        // chunk 0 leaves its accumulator after its frames (colour and count: the state every
        // later frame starts from) in row 0, which holds no colour of its own
        if (chunk == 0u && c0_regs) {
            const u32x4 v = {__float_as_uint(c.x), __float_as_uint(c.y), __float_as_uint(c.z), n};
            __builtin_amdgcn_raw_buffer_store_b128(v, col_rsrc, (int)(lane * 16u), 0, 16);
        }
        // arrival: every colour of this chunk has left the CU (sc1 stores, drained), then one
        // agent-scope add; the tile's last arriver (told by the add's value) reads the other
        // chunks' colours with sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility,
        // first row of the hand-off table) and accumulates their frames in order after chunk
        // 0's state
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t* cnt = p.split_cnt + (size_t)lband * tiles_x + (wave_in ? tx : 0u);
        uint32_t old = 0u;
        if (lane == 0u) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        old = __builtin_amdgcn_readlane(old, 0);
        if (old + 1u == S) {
            if (lane == 0u)    // (the next launch starts after this one ends)
                __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!c0_regs) {      // every frame's colour is in the buffer
                c = mk(0.0f, 0.0f, 0.0f);
                n = 0u;
                if (!p.reset_first && valid) {
                    const float4 acc = p.in[tc.idx];
                    c = mk(acc.x, acc.y, acc.z);
                    n = f2u(acc.w);
                }
            } else if (chunk != 0u) {   // (chunk 0 arriving last holds its state in registers)
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(col_rsrc, (int)(lane * 16u),
                                                                      0, 16);
                c = mk(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z));
                n = v.w;
            }
            // the colours of the frames after chunk 0's state in batches of kMergeBatch
            // frames, all of a batch's loads in flight before its accumulation (one dependent
            // load per frame made the merge as long as 64 load latencies)
            constexpr uint32_t kMergeBatch = 8;
            for (uint32_t f0 = c0_regs ? cs : 0u; f0 < p.frames; f0 += kMergeBatch) {
                u32x4 v[kMergeBatch];
#pragma unroll
                for (uint32_t j = 0; j < kMergeBatch; ++j)   // (rows past the last frame:
                    v[j] = __builtin_amdgcn_raw_buffer_load_b128(   // dropped by the buffer)
                        col_rsrc, (int)(((f0 + j) * 64u + lane) * 16u), 0, 16);
#pragma unroll
                for (uint32_t j = 0; j < kMergeBatch; ++j) {
                    const uint32_t fj = f0 + j;
                    if (fj >= p.frames) break;
                    if (fj == 0u && p.reset_first) {              // wgsl:345-350
                        c = mk(0.0f, 0.0f, 0.0f);
                        n = 0u;
                    }
                    const v3 col = mk(__uint_as_float(v[j].x), __uint_as_float(v[j].y),
                                      __uint_as_float(v[j].z));
                    if (valid && n < spp) {                       // wgsl:352, 356-357
                        const float k = (float)(n + 1u);
                        c = mk(c.x + (col.x - c.x) / k, c.y + (col.y - c.y) / k,
                               c.z + (col.z - c.z) / k);
                    }
                    // wgsl:362-363, the same images as the per-wave mode
                    if (valid && (fj + 1u == p.frames ||
                                  (p.store_each && (p.store_each == 2u || fj + 2u == p.frames)))) {
                        float4* dst = (p.store_each && (fj & 1u)) ? p.out2 : p.out;
                        dst[tc.idx] = make_float4(c.x, c.y, c.z, (float)(n < spp ? n + 1u : n));
                    }
                    n = f2u((float)(n < spp ? n + 1u : n));
                }
            }
        }
    }
    // (a split tile's cost: its chunk 0's duration times S, the chunks carrying equal frames,
    // so that the next launch's order ranks it with the unsplit tiles)
    if (p.tile_cost && threadIdx.x == 0u && chunk == 0u)
        p.tile_cost[group] =
            ((uint32_t)__builtin_amdgcn_s_memtime() - p.tile_cost[group]) * S;
    WAVE_TRACE(1);
}

// launch_tile_order: one 1024-thread workgroup; bucket = quantised log2 of the cost (four
// buckets per octave).  Each wave counts its tiles into its own LDS histogram (atomics only
// contend inside a wave), one block-wide scan over the [bucket][wave] counts turns them
// into offsets, costliest bucket first, and each tile is placed at its wave's next slot of
// its bucket (order inside a bucket is arbitrary: tiles are independent).
// parts > 1: the sorted list is dealt round-robin into `parts` contiguous sub-lists (entry
// pos to part pos % parts), one per concurrent part of a one-frame update (launch_single):
// every part gets the same mix of costly and cheap workgroups, costliest first.
__device__ __forceinline__ uint32_t part_pos(uint32_t pos, uint32_t n, uint32_t parts) {
    if (parts <= 1u) return pos;
    const uint32_t k = pos % parts, j = pos / parts;
    return k * (n / parts) + min(k, n % parts) + j;
}
__global__ __launch_bounds__(1024) void rt_tile_order_kernel(const uint32_t* __restrict__ cost,
                                                             uint32_t* __restrict__ order,
                                                             uint32_t tiles, uint32_t tiles_x,
                                                             uint32_t parts) {
    constexpr uint32_t kBuckets = 128, kWaves = 16, kSlots = kBuckets * kWaves;
    __shared__ uint32_t hist[kSlots];          // [bucket][wave]
    __shared__ uint32_t scan[1024];
    auto bucket = [](uint32_t c) -> uint32_t {
        if (c == 0u) return kBuckets - 1u;
        const uint32_t lz = (uint32_t)__builtin_clz(c);
        const uint32_t e = 31u - lz;
        const uint32_t m = e >= 2u ? (c >> (e - 2u)) & 3u : (c << (2u - e)) & 3u;
        return kBuckets - 1u - (e * 4u + m);          // descending cost
    };
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    hist[2 * tid] = 0u;
    hist[2 * tid + 1] = 0u;
    __syncthreads();
    // (loads in batches of 8 per thread: one memory latency per batch, not per tile)
    constexpr uint32_t kBatch = 8;
    for (uint32_t t0 = tid; t0 < tiles; t0 += 1024u * kBatch) {
        uint32_t c[kBatch];
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            const uint32_t t = t0 + k * 1024u;
            c[k] = t < tiles ? cost[t] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k)
            if (t0 + k * 1024u < tiles) atomicAdd(&hist[bucket(c[k]) * kWaves + wave], 1u);
    }
    __syncthreads();
    // exclusive scan of the 2048 counts: pairs per thread, Hillis-Steele over the threads
    const uint32_t a0 = hist[2 * tid], a1 = hist[2 * tid + 1];
    uint32_t v = a0 + a1;
    scan[tid] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 1024u; d <<= 1) {
        const uint32_t add = tid >= d ? scan[tid - d] : 0u;
        __syncthreads();
        v += add;
        scan[tid] = v;
        __syncthreads();
    }
    const uint32_t before = v - a0 - a1;               // exclusive prefix of the pair
    hist[2 * tid] = before;
    hist[2 * tid + 1] = before + a0;
    __syncthreads();
    for (uint32_t t0 = tid; t0 < tiles; t0 += 1024u * kBatch) {
        uint32_t c[kBatch];
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            const uint32_t t = t0 + k * 1024u;
            c[k] = t < tiles ? cost[t] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            const uint32_t t = t0 + k * 1024u;
            if (t < tiles) {
                const uint32_t pos = atomicAdd(&hist[bucket(c[k]) * kWaves + wave], 1u);
                order[part_pos(pos, tiles, parts)] =
                    ((t / tiles_x) << 16) | (t % tiles_x);
            }
        }
    }
}

hipError_t launch_tile_order(const uint32_t* tile_cost, uint32_t* tile_order, uint32_t tiles,
                             uint32_t tiles_x, hipStream_t stream, uint32_t parts) {
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_tile_order_kernel, dim3(1), dim3(1024), 0, stream, tile_cost,
                       tile_order, tiles, tiles_x, parts);
    return hipGetLastError();
}

// launch_unit_order: the split bounce schedule's units by their own recorded cost (one
// 1024-thread workgroup, the buckets of rt_tile_order_kernel).  A tile whose cost exceeds
// thr = k_thr * (sum of all costs) — k_thr = alpha / (resident waves of the launch), i.e. alpha
// times the launch's ideal span — becomes S chunk units of cost / S (its bucket moves 4 * log2 S
// places: four per octave), every other tile one unit; the units are then placed costliest
// first, a split tile's chunks side by side, so the tail after the last dispatch is bounded by
// the costliest unit rather than by the costliest tile (longest-processing-time-first on the
// units).  *count = the number of units.
__global__ __launch_bounds__(1024) void rt_unit_order_kernel(const uint32_t* __restrict__ cost,
                                                             uint32_t* __restrict__ order,
                                                             uint32_t* __restrict__ count,
                                                             uint32_t tiles, uint32_t tiles_x,
                                                             uint32_t S, float k_thr) {
    constexpr uint32_t kBuckets = 128, kWaves = 16;
    __shared__ uint32_t hist[kBuckets * kWaves];       // [bucket][wave]
    __shared__ uint32_t scan[1024];
    __shared__ unsigned long long total;
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    const uint32_t shift = 4u * (31u - (uint32_t)__builtin_clz(S));   // 4 * log2 S (S = 2^k)
    auto bucket = [](uint32_t c) -> uint32_t {
        if (c == 0u) return kBuckets - 1u;
        const uint32_t lz = (uint32_t)__builtin_clz(c);
        const uint32_t e = 31u - lz;
        const uint32_t m = e >= 2u ? (c >> (e - 2u)) & 3u : (c << (2u - e)) & 3u;
        return kBuckets - 1u - (e * 4u + m);          // descending cost
    };
    hist[2 * tid] = 0u;
    hist[2 * tid + 1] = 0u;
    if (tid == 0u) total = 0ull;
    __syncthreads();
    unsigned long long mine = 0ull;
    for (uint32_t t = tid; t < tiles; t += 1024u) mine += cost[t];
    atomicAdd(&total, mine);
    __syncthreads();
    const double thr_d = (double)total * (double)k_thr;
    const uint32_t thr = thr_d >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)thr_d;
    auto unit_bucket = [&](uint32_t c, bool& split) -> uint32_t {
        split = S > 1u && c > thr;
        const uint32_t b = bucket(c);
        return split ? min(b + shift, kBuckets - 1u) : b;
    };
    for (uint32_t t = tid; t < tiles; t += 1024u) {
        bool split;
        const uint32_t b = unit_bucket(cost[t], split);
        atomicAdd(&hist[b * kWaves + wave], split ? S : 1u);
    }
    __syncthreads();
    const uint32_t a0 = hist[2 * tid], a1 = hist[2 * tid + 1];
    uint32_t v = a0 + a1;
    scan[tid] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 1024u; d <<= 1) {
        const uint32_t add = tid >= d ? scan[tid - d] : 0u;
        __syncthreads();
        v += add;
        scan[tid] = v;
        __syncthreads();
    }
    const uint32_t before = v - a0 - a1;
    hist[2 * tid] = before;
    hist[2 * tid + 1] = before + a0;
    if (tid == 1023u) *count = v;                      // (the inclusive total)
    __syncthreads();
    for (uint32_t t = tid; t < tiles; t += 1024u) {
        bool split;
        const uint32_t b = unit_bucket(cost[t], split);
        const uint32_t n = split ? S : 1u;
        const uint32_t pos = atomicAdd(&hist[b * kWaves + wave], n);
        const uint32_t e = (split ? 0x80000000u : 0u) | ((t / tiles_x) << 16) | (t % tiles_x);
        for (uint32_t k = 0; k < n; ++k) order[pos + k] = e | (k << 28);
    }
}

hipError_t launch_unit_order(const uint32_t* tile_cost, uint32_t* unit_order,
                             uint32_t* unit_count, uint32_t tiles, uint32_t tiles_x,
                             uint32_t split, float k_thr, hipStream_t stream) {
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_unit_order_kernel, dim3(1), dim3(1024), 0, stream, tile_cost,
                       unit_order, unit_count, tiles, tiles_x, split, k_thr);
    return hipGetLastError();
}

// Per-workgroup candidate-list load of one-frame launches (wg_order's sort key): the sum of
// its `per` tiles' loads (4 + count for a tile with a list, 64 for a tile without one).
__global__ __launch_bounds__(256) void rt_wg_cost_kernel(const float4* __restrict__ cand,
                                                         uint32_t tiles_x, uint32_t cols,
                                                         uint32_t per, uint32_t units,
                                                         uint32_t* __restrict__ cost) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    if (u >= units) return;
    const uint32_t b = u / cols, g = u % cols;
    uint32_t sum = 1u;                                  // (cost 0 sorts last)
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t tx = g * per + k;
        if (tx >= tiles_x) break;
        const uint32_t c = load_cnt(cand, b * tiles_x + tx);
        sum += c == kCandNone ? 64u : (c ? 4u + c : 0u);
    }
    cost[u] = sum;
}

// List the spheres the camera rays of each tile can hit (see footprint_cone).
// One wave per block of 8 x 8 tiles (8 columns of tiles x 8 local bands), one lane per
// tile.  The wave first tests the spheres, 64 at a time, against the cone of the whole
// block's footprint and stages the survivors (scan + sphere records, index order) in LDS,
// kCandStage spheres per pass with all their loads in flight together; then every lane
// tests the staged spheres against its own
// tile's cone, one sphere per step (an LDS broadcast), appending hits to its tile's list.
// A sphere the block cone rejects provably misses every camera ray of the block (the same
// exact margins as the tile test), so the lists hold every sphere a camera ray of the tile
// can hit, in index order, and the scans over them return the full scan's bits.  (A block
// whose cone is degenerate stages every sphere.)  Per tile the cone setup is done once per
// lane and a sphere costs one cone test, instead of 64 lanes repeating the setup and
// testing all spheres per tile.
#ifndef RT_CAND_BX
#define RT_CAND_BX 8
#endif
#ifndef RT_CAND_BY
#define RT_CAND_BY 8
#endif
constexpr uint32_t kCandBX = RT_CAND_BX;   // block width in tiles
constexpr uint32_t kCandBY = RT_CAND_BY;   // block height in local bands (kCandBX * kCandBY <= 64)
static_assert(kCandBX * kCandBY <= 64, "one lane per tile");
constexpr uint32_t kCandGroup = 8;                 // blocks of 64 spheres per pass
constexpr uint32_t kCandStage = 64 * kCandGroup;   // spheres per pass
__global__ __launch_bounds__(64) void rt_candidates_kernel(const TraceParams p,
                                                           float4* __restrict__ cand) {
    __shared__ float4 s_rec[kCandStage];
    __shared__ float4 s_sph[2 * kCandStage];
    __shared__ uint32_t s_idx[kCandStage];
    const float4* __restrict__ geom = p.geom;
    const float4* __restrict__ gsph = p.sph;
    const uint32_t count = p.count;
    const uint32_t lane = threadIdx.x;
    const uint32_t tiles_x = (p.width + 7u) >> 3;
    const uint32_t tx0 = blockIdx.x * kCandBX, lb0 = blockIdx.y * kCandBY;
    const uint32_t tx1 = min(tx0 + kCandBX, tiles_x);
    const uint32_t lb1 = min(lb0 + kCandBY, p.local_bands);
    const auto row0 = [&](uint32_t lb) {
        return (float)((p.band_first + lb * p.band_step) * RT_STRIPE_ROWS);
    };
    Cone kb;
    const bool in_blk = footprint_cone(p, (float)(tx0 * 8u), (float)(tx1 * 8u), row0(lb0),
                                    row0(lb1 - 1u) + 8.0f, kb);
    // this lane's tile and its cone
    const uint32_t tx = tx0 + lane % kCandBX, lb = lb0 + lane / kCandBX;
    const bool mine = tx < tx1 && lb < lb1;
    Cone k;
    const bool ok = mine && footprint_cone(p, (float)(tx * 8u), (float)(tx * 8u + 8u), row0(lb),
                                           row0(lb) + 8.0f, k);
    const uint32_t tile = lb * tiles_x + tx;
    const uint32_t K = p.cand_k;
    float4* const own = cand + (size_t)tile * kCandStride;
    float4* const rec = own + kCandRecOff;
    float4* const sph = own + kCandSphOff;
    uint32_t n = 0;
    for (uint32_t gbase = 0; gbase < count; gbase += kCandStage) {   // (uniform)
        // the group's scan records, all loads in flight together
        float4 gv[kCandGroup];
#pragma unroll
        for (uint32_t b = 0; b < kCandGroup; ++b) {
            const uint32_t i = gbase + b * 64u + lane;
            gv[b] = geom[i < count ? i : 0u];
        }
        uint32_t m = 0;
#pragma unroll
        for (uint32_t b = 0; b < kCandGroup; ++b) {             // block-cone survivors
            const uint32_t i = gbase + b * 64u + lane;
            const bool keep = i < count && (!in_blk || !cone_misses(kb, gv[b]));
            const unsigned long long mask = rt_ballot(keep);
            if (keep) {
                const uint32_t pos = m + __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
                s_rec[pos] = gv[b];
                s_idx[pos] = i;
            }
            m += (uint32_t)__builtin_popcountll(mask);
        }
        __syncthreads();
        for (uint32_t j = lane; j < m; j += 64u) {              // their sphere records
            const uint32_t i = s_idx[j];
            s_sph[2u * j] = gsph[2u * i];
            s_sph[2u * j + 1u] = gsph[2u * i + 1u];
        }
        __syncthreads();
        for (uint32_t j = 0; j < m; ++j) {                      // this lane's tile test
            const float4 gj = s_rec[j];
            if (ok && !cone_misses(k, gj)) {
                if (n < K) {
                    rec[n] = gj;
                    sph[2u * n] = s_sph[2u * j];
                    sph[2u * n + 1u] = s_sph[2u * j + 1u];
                }
                ++n;
            }
        }
        __syncthreads();                                        // (the next group restages)
    }
    if (!mine) return;
    const uint32_t c = ok && n <= K ? n : kCandNone;
    // zero the chunk padding after the last record
    if (c != kCandNone)
        for (uint32_t q = n; q < ((n + 3u) & ~3u); ++q)
            rec[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    own[0] = make_float4(__uint_as_float(c), 0.0f, 0.0f, 0.0f);
}

__global__ __launch_bounds__(256) void rt_init_kernel(float4* __restrict__ out, uint64_t n) {
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = z;
}

// gathered = nranks x max_local_rows x width texels; band b of the full image is local
// band b / nranks of rank b % nranks.
__global__ __launch_bounds__(256) void rt_deinterleave_kernel(const float4* __restrict__ g,
                                                              float4* __restrict__ out,
                                                              uint32_t width, uint32_t height,
                                                              uint32_t nranks,
                                                              uint32_t max_local_rows) {
    const uint64_t total = (uint64_t)width * height;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t y = (uint32_t)(i / width);
        const uint32_t x = (uint32_t)(i - (uint64_t)y * width);
        const uint32_t band = y / RT_STRIPE_ROWS;
        const uint32_t rank = band % nranks;
        const uint32_t lrow = (band / nranks) * RT_STRIPE_ROWS + (y % RT_STRIPE_ROWS);
        out[i] = g[((uint64_t)rank * max_local_rows + lrow) * width + x];
    }
}

// Band-set partitions (rt_deinterleave_bands): band_src[b] = the gathered row holding band
// b's first row (rank * rows_per_rank + local band * 8), built and checked on the host.
__global__ __launch_bounds__(256) void rt_deinterleave_bands_kernel(
    const float4* __restrict__ g, float4* __restrict__ out, uint32_t width, uint32_t height,
    const uint32_t* __restrict__ band_src) {
    const uint64_t texels = (uint64_t)width * height;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < texels;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t y = (uint32_t)(i / width), x = (uint32_t)(i % width);
        const uint32_t row = band_src[y / RT_STRIPE_ROWS] + y % RT_STRIPE_ROWS;
        out[i] = g[(uint64_t)row * width + x];
    }
}

// rt_present_rgba8: one texel per lane per step, 16 B in / 4 B out.  The sRGB boundary
// table (1 KB) is staged in LDS; each channel is a branch-free 8-step binary search.
template <bool kSrgb>
__global__ __launch_bounds__(256) void rt_present_kernel(const float4* __restrict__ in,
                                                         uchar4* __restrict__ out,
                                                         uint64_t texels,
                                                         const float* __restrict__ srgb_t) {
    __shared__ float T[256];
    if (kSrgb) {
        T[threadIdx.x] = srgb_t[threadIdx.x];
        __syncthreads();
    }
    auto enc = [&](float c) -> uint32_t {
        if (kSrgb) {
            uint32_t k = 0;
#pragma unroll
            for (uint32_t s = 128; s >= 1; s >>= 1)
                k += (c >= T[k + s]) ? s : 0u;   // NaN compares false -> 0
            return k;
        }
        const float v = fminf(fmaxf(c, 0.0f), 1.0f);  // fmaxf(NaN, 0) = 0
        return (uint32_t)(v * 255.0f + 0.5f);
    };
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < texels;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        out[i] = make_uchar4((uint8_t)enc(v.x), (uint8_t)enc(v.y), (uint8_t)enc(v.z), 255);
    }
}

// ---- Self-test of the exact fast paths (rt_selftest_fastmath) ------------------------
// cnt[0]: defocus normalisation, all 2^32 values of hash(seed + 1): both disk_unit forms vs
//         sqrtf and the IEEE divisions (also the eight-value range of len2 disk_unit<3> needs).
// cnt[1]: div_core_signed vs a / b on random a, b over div_core's domain (rt_device.h:
//         |b| in [2^-20, 2^33), |a| in [2^-100, 2^91), exponent gap in [-120, 88]; a also
//         +-0, b also the accumulator's n + 1 up to 2^32) and over [2^-40, 2^40]^2;
//         div_rn (y = RN32(1 / b)) vs a / b beyond integer denominators (|b| in
//         [2^-20, 2^20], |a| in [2^-100, 2^43], where |b y - 1| <= 2^-25; half of them with
//         both significands near 2); and acc_rn vs c + num / k for numerators acc_ok accepts
//         (finite f32 bits or NaN, many near the subnormal range) and k in [1, 2^22).
// cnt[2]: sqrt_core vs sqrtf on every finite x >= 2^-96 (exhaustive).
// cnt[3]: consider_fast vs consider (root selection, tmax and index) on random rays and
//         spheres of the camera-ray domain (|d|^2 in [2^-11, 2^20], |O|, |C| + |R| <= 2^39),
//         half of them grazing (D near 0), with random incoming tmax.
// cnt[4]: cases run.
__device__ __forceinline__ uint32_t mix32(uint64_t i, uint32_t salt) {
    return hash((uint32_t)i ^ hash((uint32_t)(i >> 32) + salt));
}
// sign from r's top bit, mantissa from r, exponent e (unbiased)
__device__ __forceinline__ float with_exp(uint32_t r, int e) {
    return __uint_as_float((r & 0x807FFFFFu) | ((uint32_t)(127 + e) << 23));
}
__device__ __forceinline__ float unit_rand(uint32_t r) {   // [-1, 1)
    return (float)(int32_t)r * 0x1p-31f;
}
__device__ __forceinline__ bool same_bits(float x, float y) {   // NaN == NaN
    return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
}
__device__ __forceinline__ bool root_case(uint64_t i) {
    const uint32_t r0 = mix32(i, 11u), r1 = mix32(i, 12u), r2 = mix32(i, 13u),
                   r3 = mix32(i, 14u), r4 = mix32(i, 15u), r5 = mix32(i, 16u);
    const float ds = with_exp(0u, -5 + (int)(r0 % 15u));          // |d| up to ~2^10
    const v3 d = mk(unit_rand(r1) * ds, unit_rand(r2) * ds, unit_rand(r3) * ds);
    const float os = with_exp(0u, -10 + (int)((r0 >> 8) % 48u));  // |O| up to ~2^38
    const v3 o = mk(unit_rand(r4) * os, unit_rand(r5) * os, unit_rand(r1 ^ r5) * os);
    const float R = with_exp(r2 & 0x7FFFFFu, -20 + (int)((r0 >> 16) % 40u));
    // a point on the ray at parameter t0, then sideways by ~R (grazing) or anywhere
    const float t0 = unit_rand(r3 ^ r4) * with_exp(0u, -12 + (int)((r0 >> 24) % 30u));
    v3 side = mk(unit_rand(r4 ^ r2), unit_rand(r5 ^ r3), unit_rand(r1 ^ r4));
    const float sd = dot(side, d) / dot(d, d);
    side = sub(side, mk(sd * d.x, sd * d.y, sd * d.z));           // ~perpendicular to d
    const float sl = sqrtf(dot(side, side));
    const float jitter = 1.0f + unit_rand(r5) * with_exp(0u, -(int)(r1 % 31u));
    const float k = (r2 & 1u) ? R * jitter / sl : unit_rand(r3) * os / sl;
    const v3 C = mk(fmaf(t0, d.x, o.x) + k * side.x, fmaf(t0, d.y, o.y) + k * side.y,
                    fmaf(t0, d.z, o.z) + k * side.z);
    const float a = dot(d, d);
    if (!(a >= 0x1p-11f && a <= 0x1p20f) || !(sqrtf(dot(o, o)) <= 0x1p39f) ||
        !(sqrtf(dot(C, C)) + R <= 0x1p39f) || !(sl > 0.0f))
        return true;                                  // outside the domain: not a case
    float h;
    const float disc = discriminant(make_float4(C.x, C.y, C.z, R * R), o, d, a, h);
    const uint32_t tk = r4 % 3u;
    const float t_in = tk == 0 ? 0x1.05ed2ep+118f : tk == 1 ? fabsf(t0) : fabsf(t0) * 0.5f;
    float t1 = t_in, t2 = t_in;
    int i1 = 7, i2 = 7;
    consider(disc, h, a, 3u, t1, i1);
    consider_fast(disc, h, a, rcp_refined(a), 3u, t2, i2);
    return same_bits(t1, t2) && i1 == i2;
}
__global__ __launch_bounds__(256) void rt_selftest_kernel(unsigned long long* cnt, uint64_t n_rand) {
    unsigned long long bad0 = 0, bad1 = 0, bad2 = 0, bad3 = 0, runs = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32);
         i += stride) {
        const float ang = 0x1.921fb4p+2f * rf((uint32_t)i);
        float sa, ca;
        sincos_c(ang, sa, ca);
        const float len_ref = sqrtf(fmaf(sa, sa, ca * ca));
        const float ux_ref = ca / len_ref, uy_ref = sa / len_ref;
        float ux, uy, fx, fy;
        disk_unit<0>(sa, ca, ux, uy);
        disk_unit<3>(sa, ca, fx, fy);
        bad0 += (__float_as_uint(fx) != __float_as_uint(ux_ref)) ||
                (__float_as_uint(fy) != __float_as_uint(uy_ref)) ||
                (__float_as_uint(ux) != __float_as_uint(ux_ref)) ||
                (__float_as_uint(uy) != __float_as_uint(uy_ref));
        const float x = __uint_as_float((uint32_t)i);
        if ((uint32_t)i >= 0x0F800000u && (uint32_t)i < 0x7F800000u)   // [2^-96, +inf)
            bad2 += __float_as_uint(sqrt_core(x)) != __float_as_uint(sqrtf(x));
        ++runs;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_rand; i += stride) {
        const uint32_t r0 = mix32(i, 1u), r1 = mix32(i, 2u), r2 = mix32(i, 3u);
        float a, b;
        if (r2 & 0x40000000u) {                       // the general domain
            const int eb = -20 + (int)(r2 % 53u);
            int ea = -100 + (int)((r2 >> 8) % 191u);
            ea = max(eb - 120, min(eb + 88, ea));
            a = with_exp(r0, ea);
            b = with_exp(r1, eb);
        } else {                                      // [2^-40, 2^40]^2
            a = with_exp(r0, -40 + (int)(r2 % 80u));
            b = with_exp(r1, -40 + (int)((r2 >> 8) % 80u));
        }
        if ((r2 & 0x70000u) == 0) a = (r0 & 1u) ? -0.0f : 0.0f;
        if ((r2 & 0x380000u) == 0)                    // n + 1 counts, n < 2^32 - 1
            b = (float)((r2 & 0x400000u) ? 1u + (r1 & 0xFFFFFFu) : max(r1, 1u));
        bad1 += !same_bits(div_core_signed(a, b, rcp_refined(b)), a / b);
        {   // the sky's d.y / |d| with |d| and its reciprocal from one rsq (sqrt_core_rcp):
            // |d|^2 in [2^-20, 2^40], |d.y| <= |d| (and >= 2^-100 or zero)
            const float dd = with_exp(r1 & 0x7FFFFFu, -20 + (int)(r2 % 60u));
            float y;
            const float len = sqrt_core_rcp(dd, y);
            const float dy = (r0 & 0x1000u) ? 0.0f : unit_rand(r0) * len;
            if (dd <= 0x1p40f && (dy == 0.0f || fabsf(dy) >= 0x1p-100f))
                bad1 += !same_bits(div_core(dy, len, y), dy / sqrtf(dd));
        }
        {   // div_rn with real denominators where Markstein's hypothesis holds: y = RN32(1 / b)
            // and |b y - 1| <= 2^-25, so q = RN(a y) is within an ulp of a / b; every other
            // case the kernels' callers rule out (the radii are checked exhaustively at
            // upload, rt_rcp_check_kernel; the accumulator's k is an integer < 2^22).  Half
            // the cases in the corner where |b y - 1| approaches 2^-24: divisor significands
            // in [1.99, 2), numerator significands within 2^-11 of 2.
            const bool corner = (r2 >> 20) & 1u;
            const uint32_t mb = corner ? 0x7EB852u + r1 % (0x800000u - 0x7EB852u) : r1;
            const uint32_t ma = corner ? 0x7FFFFFu - (r0 % 4096u) : (r0 ^ r2);
            const float rb = with_exp((r1 & 0x80000000u) | (mb & 0x7FFFFFu), -20 + (int)(r2 % 41u));
            const float ra = with_exp((r0 & 0x80000000u) | (ma & 0x7FFFFFu),
                                      -100 + (int)((r2 >> 8) % 144u));
            const float yb = 1.0f / rb;
            if (fabsf(fmaf(rb, yb, -1.0f)) <= 0x1p-25f)
                bad1 += !same_bits(div_rn(ra, rb, yb), ra / rb);
        }
        // the accumulator's Markstein division: any finite f32 numerator or NaN (r0's bits:
        // zeros and subnormals included; the kernels' num = col - c is never +-inf against a
        // finite c, see acc_ok), k = f32(n + 1) for n + 1 in [1, 2^22) (kAccRnMax)
        const uint32_t kk = (r2 & 0x800000u) ? 1u + (r1 % (kAccRnMax - 1u))
                                             : 1u + (r1 % 4096u);   // small counts too
        const v3 num = mk(__uint_as_float(r0), __uint_as_float(r0 ^ r1),
                          __uint_as_float(r2 & 0x83FFFFFFu));       // (many tiny ones)
        if (acc_ok(num) && !isinf(num.x) && !isinf(num.y) && !isinf(num.z)) {
            const float kf = (float)kk;
            const v3 c0 = mk(0.0f, 0.0f, 0.0f);
            const v3 q = acc_rn(c0, num, kf, 1.0f / kf);
            bad1 += !same_bits(q.x, 0.0f + num.x / kf) || !same_bits(q.y, 0.0f + num.y / kf) ||
                    !same_bits(q.z, 0.0f + num.z / kf);
        }
        ++runs;
    }
    atomicAdd(&cnt[0], bad0);
    atomicAdd(&cnt[1], bad1);
    atomicAdd(&cnt[2], bad2);
    atomicAdd(&cnt[3], bad3);
    atomicAdd(&cnt[4], runs);
}

// TraceParams::normal_rn: is one Markstein step from y = rcp_refined(R) the IEEE quotient
// a / R for every numerator the kernels divide, for every distinct radius R of the scene?
// Markstein's theorem needs y within half an ulp of 1 / R AND q = RN(a y) within one ulp of
// a / R; a correctly rounded y alone gives |R y - 1| <= 2^-24, and with a divisor's and a
// quotient's significands both near 2 q can then be 1.5 ulp off (round-5 ADVICE).  So the
// check is exhaustive instead of sufficient: for each radius every numerator significand
// (2^23 of them) in two binades, [1, 2) and [2^-100, 2^-99) (the kernels' smallest
// numerators), against the IEEE division.  A step and its operands scale exactly by powers of
// two while q, the residual and the result stay normal (numerators in [2^-100, 2^43], R in
// [2^-20, 2^20]: the callers' domain), so these two binades cover every numerator; the sign
// is symmetric.  One thread per (radius, significand, binade), a vector atomic OR on a miss.
constexpr uint32_t kRcpCheckPerRadius = 2u << 23;
__global__ __launch_bounds__(256) void rt_rcp_check_kernel(const float* radii, uint32_t n,
                                                           uint32_t* bad) {
    const uint64_t total = (uint64_t)n * kRcpCheckPerRadius;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t miss = 0u;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const float r = radii[i / kRcpCheckPerRadius];
        const uint32_t j = (uint32_t)(i % kRcpCheckPerRadius);
        // significand j & 0x7FFFFF; binade 2^0 or 2^-100
        const float a = __uint_as_float(((j >> 23) ? 0x0D800000u : 0x3F800000u) | (j & 0x7FFFFFu));
        const float y = rcp_refined(r);
        miss |= __float_as_uint(div_rn(a, r, y)) != __float_as_uint(a / r);
    }
    if (miss) atomicOr(bad, 1u);
}
hipError_t launch_rcp_check(const float* radii, uint32_t n, uint32_t* bad, hipStream_t stream) {
    if (n == 0u) return hipSuccess;
    hipLaunchKernelGGL(rt_rcp_check_kernel, dim3(2048), dim3(256), 0, stream, radii, n, bad);
    return hipGetLastError();
}

hipError_t launch_selftest(unsigned long long* cnt, uint64_t n_rand, hipStream_t stream) {
    hipLaunchKernelGGL(rt_selftest_kernel, dim3(8192), dim3(256), 0, stream, cnt, n_rand);
    return hipGetLastError();
}

// 256-thread workgroups: 4 waves = 4 tiles along a stripe band; grid (columns/4, bands).
static dim3 tile_grid(const TraceParams& p, uint32_t waves = 4) {
    const uint32_t tiles_x = (p.width + 7u) >> 3;
    return dim3((tiles_x + waves - 1u) / waves, p.local_bands);
}

// Launches through hipModuleLaunchKernel with the arguments packed in the kernel's layout and
// a function handle cached per device and kernel (the launch_single path below): no
// per-launch symbol lookup or per-argument marshalling of the 2.6-KB TraceParams block.
// Slots: 0-4 rt_trace_kernel<k>, 5-8 rt_bounce_kernel<m>, 9-10 rt_tpair_kernel<4 / 2>.
constexpr int kLaunchSlots = 12;
// Launch timing (rt_set_launch_timing): while armed, launch_packed goes through
// hipExtModuleLaunchKernel with the armed events — the start event on the first launch
// after arming, the stop event on every launch — so the dispatch packets themselves carry
// the timestamps (no marker packets on the stream, which cost an idle GPU's short region
// ≈ 2.5 µs).  Per host thread, like the calls that arm it.
static thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;
static thread_local uint32_t g_ev_launches = 0;
void arm_launch_events(hipEvent_t start, hipEvent_t stop) {
    g_ev_start = start;
    g_ev_stop = stop;
    g_ev_launches = 0;
}
uint32_t disarm_launch_events() {
    g_ev_start = g_ev_stop = nullptr;
    return g_ev_launches;
}
static hipError_t launch_packed(int slot, const void* sym, dim3 grid, dim3 block, size_t lds,
                                hipStream_t stream, void* args, size_t bytes) {
    constexpr int kMaxDevices = 64;
    static hipFunction_t fn[kMaxDevices][kLaunchSlots] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices || slot < 0 || slot >= kLaunchSlots)
        return hipErrorInvalidValue;
    if (!fn[dev][slot]) {
        e = hipGetFuncBySymbol(&fn[dev][slot], sym);
        if (e != hipSuccess) {
            fn[dev][slot] = nullptr;
            return e;
        }
    }
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &bytes,
                     HIP_LAUNCH_PARAM_END};
    if (g_ev_stop) {
        // (global work sizes in work-items)
        e = hipExtModuleLaunchKernel(fn[dev][slot], grid.x * block.x, grid.y * block.y,
                                     grid.z * block.z, block.x, block.y, block.z, lds, stream,
                                     nullptr, extra, g_ev_start, g_ev_stop, 0);
        if (e == hipSuccess) {
            g_ev_start = nullptr;
            ++g_ev_launches;
        }
        return e;
    }
    return hipModuleLaunchKernel(fn[dev][slot], grid.x, grid.y, grid.z, block.x, block.y,
                                 block.z, (unsigned)lds, stream, nullptr, extra);
}

// rt_trace_kernel's explicit arguments in its layout (the preloaded leading dwords, then
// TraceParams at kParamsOff)
struct TraceArgs {
    const float4* cand;
    const uint32_t* hx;
    const float4* in;
    uint32_t width, height, bands;
    TraceParams p;
};
static_assert(offsetof(TraceArgs, p) == kParamsOff, "rt_trace_kernel's argument layout");

template <int kScan>
static hipError_t launch_trace_as(const TraceParams& p, size_t lds, hipStream_t stream) {
    constexpr uint32_t w = wg_waves<kScan>();
    const dim3 grid = tile_grid(p, is_group_kernel(kScan) ? 1u : w);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    TraceArgs args;
    std::memset(&args, 0, offsetof(TraceArgs, p));
    args.cand = p.cand;
    args.hx = p.hx;
    args.in = p.in;
    args.width = p.width;
    args.height = p.height;
    args.bands = pack_bands(p.band_first, p.band_step, p.tile_order != nullptr);
    args.p = p;
    return launch_packed(kScan, reinterpret_cast<const void*>(&rt_trace_kernel<kScan>), grid,
                         dim3(64 * w), lds, stream, &args, sizeof(args));
}

// rt_tpair_kernel<G>: one workgroup of G waves per pair of tiles along a stripe band, grid
// (tile pairs, bands) — or the tile order's units in that shape.
template <int G>
static hipError_t launch_tpair(const TraceParams& p, hipStream_t stream) {
    const dim3 grid((((p.width + 7u) >> 3) + 1u) >> 1, p.local_bands);
    if (grid.x == 0 || grid.y == 0 || !p.cand) return grid.x && grid.y ? hipErrorInvalidValue
                                                                      : hipSuccess;
    TraceArgs args;
    std::memset(&args, 0, offsetof(TraceArgs, p));
    args.cand = p.cand;
    args.hx = p.hx;
    args.in = p.in;
    args.width = p.width;
    args.height = p.height;
    args.bands = pack_bands(p.band_first, p.band_step, p.tile_order != nullptr);
    args.p = p;
    return launch_packed(G == 4 ? 9 : 10, reinterpret_cast<const void*>(&rt_tpair_kernel<G>),
                         grid, dim3(64 * G), 0, stream, &args, sizeof(args));
}

// TraceParams::hint_rs_dev: row f * depth + i = (rf(sb), random_unit_vector(sb)) with
// sb = hash(hint_n[f] + seed_b[f] + 2 + 1000 i) (wgsl:268, 353) — the values a pixel at the
// hinted count computes itself, by the same device functions.
__global__ __launch_bounds__(256) void rt_hint_rs_kernel(const TraceParams p) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= p.hint_rs_dev_frames * p.depth) return;
    const uint32_t f = t / p.depth, i = t % p.depth;
    const uint32_t sb = hash(p.hint_n[f] + p.seed_b[f] + 2u + i * 1000u);
    const float r_sb = rf(sb);
    const v3 u = random_unit_vector(r_sb, sb);
    p.hint_rs_dev[t] = make_float4(r_sb, u.x, u.y, u.z);
}

// Workgroups of kBounceWaves tiles along a stripe band: grid (column groups, bands).
static hipError_t launch_bounce(const TraceParams& p, hipStream_t stream) {
    const uint32_t tiles_x = (p.width + 7u) >> 3;
    if (p.hint_rs_dev && p.hint_rs_dev_frames) {
        if (p.hint_rs_dev_frames > kHintFrames || p.depth > kHintRsDepth)
            return hipErrorInvalidValue;
        const uint32_t n = p.hint_rs_dev_frames * p.depth;
        rt_hint_rs_kernel<<<dim3((n + 255u) / 256u), dim3(256), 0, stream>>>(p);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const uint32_t w = p.compact == 1u ? kBounceWaves : 1u;   // tiles per workgroup
    dim3 grid((tiles_x + w - 1u) / w, p.local_bands);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    const size_t lds = (size_t)p.lds_records * sizeof(float4);
    TraceParams args = p;
    const void* sym = reinterpret_cast<const void*>(&rt_bounce_kernel<kBounceWave>);
    uint32_t threads = 64;
    if (p.compact == 3u) {                                    // (tile, chunk) units
        grid = dim3(p.unit_order ? tiles_x * p.local_bands * p.split
                                 : tiles_x * p.local_bands + p.split_tiles * (p.split - 1u), 1);
        sym = reinterpret_cast<const void*>(&rt_bounce_kernel<kBounceSplit>);
    } else if (p.compact == 1u) {
        sym = reinterpret_cast<const void*>(&rt_bounce_kernel<kBounceCompact>);
        threads = 64 * kBounceWaves;
    } else if (p.compact == 2u) {
        sym = reinterpret_cast<const void*>(&rt_bounce_kernel<kBouncePair>);
        threads = 128;
    }
    return launch_packed(5 + (int)p.compact, sym, grid, dim3(threads), lds, stream, &args,
                         sizeof(args));
}

// The explicit arguments of rt_single_kernel / rt_chain_kernel, in the kernels' layout.
struct SingleArgs {
    const float4* cand;
    const uint32_t* hx;
    const float4* in;
    uint32_t width, height, bands;
    const uint32_t* order;
    SingleParams q;
};
static_assert(offsetof(SingleArgs, q) == 48, "rt_single_kernel's argument layout");

// One part of a one-frame launch (kSingleWg waves of kPix tiles each per workgroup along a
// stripe band): its arguments and grid; false when the part has no workgroup.
template <int kPix>
static bool single_args(const TraceParams& p, SingleArgs& args, dim3& grid) {
    const uint32_t tiles_x = (p.width + 7u) >> 3;
    const uint32_t per = kSingleWg * kPix;
    const uint32_t cols = (tiles_x + per - 1u) / per;
    const uint32_t parts = p.parts > 1u ? p.parts : 1u, part = parts > 1u ? p.part : 0u;
    // this part's workgroups: its sub-list of the order, or every parts-th local band
    grid = dim3(cols, p.local_bands);
    const uint32_t* order = p.wg_order;
    uint32_t lbands = 1u << 16;
    if (parts > 1u) {
        if (order) {
            uint32_t first = 0, len = 0;
            part_range(cols * p.local_bands, parts, part, first, len);
            grid = dim3(len, 1);
            order += first;
        } else {
            grid.y = p.local_bands > part ? (p.local_bands - part + parts - 1u) / parts : 0u;
            lbands = part | (parts << 16);
        }
    }
    if (grid.x == 0 || grid.y == 0) return false;
    SingleParams& q = args.q;
    std::memset(&args, 0, sizeof(args));
    args.cand = p.cand;
    args.hx = p.hx;
    args.in = p.in;
    args.width = p.width;
    args.height = p.height;
    args.bands = pack_bands(p.band_first, p.band_step, false);
    args.order = order;
    q.lbands = lbands;
    q.out = p.out;
    q.geom = p.geom;
    q.sph = p.sph;
    q.count = p.count;
    q.depth = p.depth;
    q.spp = p.spp;
    q.hinted = p.hint_frames != 0u;
    q.n_hint = p.hint_n[0];
    q.seed_b = p.seed_b[0];
    q.hy_off = (uint32_t)(p.hy - p.hx);
    q.rcp_hint = p.hint_rcp[0];
    q.normal_rn = p.normal_rn;
    q.rs = p.hint_rs[0];
    for (int i = 0; i < 3; ++i) {
        q.center[i] = p.center[i];
        q.vul[i] = p.vul[i];
        q.pdu[i] = p.pdu[i];
        q.pdv[i] = p.pdv[i];
        q.ddu[i] = p.ddu[i];
        q.ddv[i] = p.ddv[i];
    }
    q.defocus_angle = p.defocus_angle;
    q.grid_x = grid.x;
    return true;
}

template <int kPix>
static hipError_t launch_single(const TraceParams& p, hipStream_t stream) {
    SingleArgs args;
    dim3 grid;
    if (!single_args<kPix>(p, args, grid)) return hipSuccess;
    // hipModuleLaunchKernel with the arguments packed in the kernel's layout and a cached
    // function handle: no per-launch symbol lookup or per-argument marshalling (320-byte
    // arguments: 4.2-4.4 against 5.0-6.0 µs of host time per launch through the
    // hipLaunchKernelGGL path, profiles/r03/r03j_launch_rate.jsonl) — the host's issue rate
    // bounds small rank shares and the concurrent parts
    size_t bytes = sizeof(args);
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &bytes,
                     HIP_LAUNCH_PARAM_END};
    // (function handles are per device: the caller's DeviceGuard has made it current)
    constexpr int kMaxDevices = 64;
    static hipFunction_t fn[kMaxDevices][2] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    const int r = p.reset_first ? 1 : 0;
    if (!fn[dev][r]) {
        e = hipGetFuncBySymbol(&fn[dev][r],
                               r ? reinterpret_cast<const void*>(&rt_single_reset_kernel<kPix>)
                                 : reinterpret_cast<const void*>(&rt_single_kernel<kPix>));
        if (e != hipSuccess) {
            fn[dev][r] = nullptr;
            return e;
        }
    }
    return hipModuleLaunchKernel(fn[dev][r], grid.x, grid.y, 1, 64 * kSingleWg, 1, 1, 0, stream,
                                 nullptr, extra);
}

// ---- Frame chains (rt_chain.cpp) ----------------------------------------------------------
// The code object's chain kernels: [pix == 1 ? 0 : 1][reset], the go and the done kernel.
// hipGetFuncBySymbol makes HIP load the code object on the current device, so that the
// HSA loader lists their symbols (rt_chain.cpp looks them up by these mangled-name parts).
hipError_t chain_load_kernels() {
    const void* k[] = {reinterpret_cast<const void*>(&rt_chain_kernel<1>),
                       reinterpret_cast<const void*>(&rt_chain_reset_kernel<1>),
                       reinterpret_cast<const void*>(&rt_chain_kernel<(int)kSinglePix>),
                       reinterpret_cast<const void*>(&rt_chain_reset_kernel<(int)kSinglePix>),
                       reinterpret_cast<const void*>(&rt_chain_go_kernel),
                       reinterpret_cast<const void*>(&rt_chain_done_kernel)};
    for (const void* f : k) {
        hipFunction_t h = nullptr;
        hipError_t e = hipGetFuncBySymbol(&h, f);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
const char* chain_kernel_symbol(int which) {
    // (Itanium mangling of rtk::rt_chain_kernel<N> etc.: "ILi<N>E" is the template argument)
    static const char* const pix1[2] = {"15rt_chain_kernelILi1EE", "21rt_chain_reset_kernelILi1EE"};
    static const char* const pix2[2] = {"15rt_chain_kernelILi2EE", "21rt_chain_reset_kernelILi2EE"};
    static const char* const pix3[2] = {"15rt_chain_kernelILi3EE", "21rt_chain_reset_kernelILi3EE"};
    static const char* const pix4[2] = {"15rt_chain_kernelILi4EE", "21rt_chain_reset_kernelILi4EE"};
    const char* const* big = kSinglePix == 2 ? pix2 : kSinglePix == 3 ? pix3 : kSinglePix == 4 ? pix4 : pix1;
    switch (which) {
        case kChainPix1: return pix1[0];
        case kChainPix1Reset: return pix1[1];
        case kChainPix: return big[0];
        case kChainPixReset: return big[1];
        case kChainGo: return "18rt_chain_go_kernel";
        default: return "20rt_chain_done_kernel";
    }
}
// The kernel arguments of one part of a one-frame launch of `kernel` (kTraceSingle /
// kTraceSingleOne) for an AQL packet: the explicit arguments, then the hidden ones of code
// object v5 at the next 8-byte boundary (block counts, group sizes, grid dimensions; the
// chain kernels read none of them — the workgroups per row come in SingleParams::grid_x).
// Returns the bytes written (0: the part has no workgroup), the grid in workgroups and the
// chain kernel (kChain*).
uint32_t chain_args(const TraceParams& p, int kernel, const uint32_t* abort, unsigned char* out,
                    uint32_t cap, uint32_t grid[2], uint32_t* group_threads, int* which) {
    SingleArgs args;
    dim3 g;
    const bool one = kernel == kTraceSingleOne;
    const bool any = one ? single_args<1>(p, args, g) : single_args<(int)kSinglePix>(p, args, g);
    if (!any) return 0;
    args.q.abort = abort;
    const uint32_t hb = (uint32_t)((sizeof(args) + 7u) & ~(size_t)7u);
    const uint32_t total = hb + kHiddenArgsBytes;
    if (total > cap) return 0;
    std::memset(out, 0, total);
    std::memcpy(out, &args, sizeof(args));
    const uint32_t bc[3] = {g.x, g.y, 1u};
    const uint16_t gs[3] = {(uint16_t)(64u * kSingleWg), 1u, 1u};
    const uint16_t dims = 2;
    std::memcpy(out + hb, bc, sizeof(bc));                 // hidden_block_count_x/y/z
    std::memcpy(out + hb + 12, gs, sizeof(gs));            // hidden_group_size_x/y/z
    std::memcpy(out + hb + 64, &dims, sizeof(dims));       // hidden_grid_dims
    grid[0] = g.x;
    grid[1] = g.y;
    *group_threads = 64u * kSingleWg;
    *which = (one ? kChainPix1 : kChainPix) + (p.reset_first ? 1 : 0);
    return total;
}

hipError_t launch_trace(const TraceParams& p, int kernel, hipStream_t stream) {
    if (kernel == kTraceSingle) return launch_single<(int)kSinglePix>(p, stream);
    if (kernel == kTraceSingleOne) return launch_single<1>(p, stream);
    if (kernel == kTraceCulled)
        return launch_trace_as<kTraceCulled>(p, (size_t)p.lds_records * sizeof(float4), stream);
    if (kernel == kTraceList) return launch_trace_as<kTraceList>(p, 0, stream);
    if (kernel == kTraceListPair)
        return launch_trace_as<kTraceListPair>(p, group_lds_bytes<kTraceListPair>(), stream);
    if (kernel == kTraceBounce) return launch_bounce(p, stream);
    if (kernel == kTraceListQuad)
        return launch_trace_as<kTraceListQuad>(p, group_lds_bytes<kTraceListQuad>(), stream);
    if (kernel == kTraceListQuad2) return launch_tpair<4>(p, stream);
    if (kernel == kTraceListPair2) return launch_tpair<2>(p, stream);
    return launch_trace_as<kTraceExhaustive>(p, 0, stream);
}

hipError_t launch_candidates(const TraceParams& p, float4* cand, hipStream_t stream) {
    const uint32_t tiles_x = (p.width + 7u) >> 3;
    const dim3 grid((tiles_x + kCandBX - 1u) / kCandBX,
                    (p.local_bands + kCandBY - 1u) / kCandBY);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_candidates_kernel, grid, dim3(64), 0, stream, p, cand);
    return hipGetLastError();
}

uint32_t single_wg_tiles(uint32_t pix) { return kSingleWg * pix; }
uint32_t single_pix() { return kSinglePix; }

hipError_t launch_wg_order(const float4* cand, uint32_t tiles_x, uint32_t bands, uint32_t pix,
                           uint32_t* wg_cost, uint32_t* wg_order, hipStream_t stream,
                           uint32_t parts) {
    const uint32_t per = kSingleWg * pix;
    const uint32_t cols = (tiles_x + per - 1u) / per;
    const uint32_t units = cols * bands;
    if (units == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_wg_cost_kernel, dim3((units + 255u) / 256u), dim3(256), 0, stream, cand,
                       tiles_x, cols, per, units, wg_cost);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_tile_order(wg_cost, wg_order, units, cols, stream, parts);
}

hipError_t launch_init(float4* out, uint64_t texels, hipStream_t stream) {
    if (texels == 0) return hipSuccess;
    uint64_t blocks = (texels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(rt_init_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, out,
                       texels);
    return hipGetLastError();
}

hipError_t launch_deinterleave(const float4* gathered, float4* out, uint32_t width,
                               uint32_t height, uint32_t nranks, uint32_t max_local_rows,
                               hipStream_t stream) {
    const uint64_t texels = (uint64_t)width * height;
    if (texels == 0) return hipSuccess;
    uint64_t blocks = (texels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(rt_deinterleave_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream,
                       gathered, out, width, height, nranks, max_local_rows);
    return hipGetLastError();
}

hipError_t launch_deinterleave_bands(const float4* gathered, float4* out, uint32_t width,
                                     uint32_t height, const uint32_t* band_src,
                                     hipStream_t stream) {
    const uint64_t texels = (uint64_t)width * height;
    if (texels == 0) return hipSuccess;
    uint64_t blocks = (texels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(rt_deinterleave_bands_kernel, dim3((uint32_t)blocks), dim3(256), 0,
                       stream, gathered, out, width, height, band_src);
    return hipGetLastError();
}

hipError_t launch_present(const float4* in, uchar4* out, uint64_t texels,
                          const float* srgb_t, hipStream_t stream) {
    if (texels == 0) return hipSuccess;
    uint64_t blocks = (texels + 255u) / 256u;
    if (blocks > 16384u) blocks = 16384u;
    if (srgb_t)
        hipLaunchKernelGGL(rt_present_kernel<true>, dim3((uint32_t)blocks), dim3(256), 0,
                           stream, in, out, texels, srgb_t);
    else
        hipLaunchKernelGGL(rt_present_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0,
                           stream, in, out, texels, srgb_t);
    return hipGetLastError();
}

const char* trace_kernel_name() { return "rt_trace_kernel"; }
const char* single_kernel_name(uint32_t pix) {
    static const char* const names[] = {"rt_single_kernel<1>", "rt_single_kernel<2>",
                                        "rt_single_kernel<3>", "rt_single_kernel<4>"};
    return names[(pix ? pix : kSinglePix) - 1];
}

}  // namespace rtk


#if RT_SSTAMPS
// Diagnostic builds: copies the one-frame kernel's per-wave stamps (12 words each, see
// RT_SSTAMPS) of the first n waves of the last launch to out[12 n] and clears them.
extern "C" __attribute__((visibility("default"))) int rt_diag_single_stamps(
    unsigned long long* out, unsigned n) {
    if (n > rtk::kSStampWaves) n = rtk::kSStampWaves;
    static unsigned long long t[rtk::kSStampWaves][12];
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpyFromSymbol(t, HIP_SYMBOL(rtk::g_sst), sizeof(t)) != hipSuccess) return 1;
    std::memcpy(out, t, (size_t)n * 12 * sizeof(unsigned long long));
    std::memset(t, 0, sizeof(t));
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_sst), t, sizeof(t)) != hipSuccess) return 1;
    return 0;
}
#endif

#if RT_BOUNCE_COUNTS
// Diagnostic builds: copies the bounce counters (n <= 32) to out and clears them.
extern "C" __attribute__((visibility("default"))) int rt_diag_bounce_counts(unsigned long long* out,
                                                                            unsigned n) {
    if (n > 32) n = 32;
    static unsigned long long c[32];
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpyFromSymbol(c, HIP_SYMBOL(rtk::g_bcount), sizeof(c)) != hipSuccess) return 1;
    for (unsigned i = 0; i < n; ++i) out[i] = c[i];
    static const unsigned long long zero[32] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_bcount), zero, sizeof(zero)) == hipSuccess ? 0 : 1;
}
#endif
#if RT_WAVE_TRACE
// Diagnostic builds: copies (start, end, hw_id, xcc_id) of the first n waves of the last
// traced launch to out[4 n] and clears them.
extern "C" __attribute__((visibility("default"))) int rt_diag_wave_trace(unsigned long long* out,
                                                                         unsigned n) {
    if (n > rtk::kTraceWaves) n = rtk::kTraceWaves;
    static unsigned long long t[rtk::kTraceWaves][2];
    static unsigned id[rtk::kTraceWaves][2];
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpyFromSymbol(t, HIP_SYMBOL(rtk::g_wave_t), sizeof(t)) != hipSuccess) return 1;
    if (hipMemcpyFromSymbol(id, HIP_SYMBOL(rtk::g_wave_id), sizeof(id)) != hipSuccess) return 1;
    for (unsigned i = 0; i < n; ++i) {
        out[4 * i] = t[i][0];
        out[4 * i + 1] = t[i][1];
        out[4 * i + 2] = id[i][0];
        out[4 * i + 3] = id[i][1];
    }
    std::memset(t, 0, sizeof(t));
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_wave_t), t, sizeof(t)) != hipSuccess) return 1;
    return 0;
}
#endif
