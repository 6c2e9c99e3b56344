// rt_device.h — restatement of the reference shader's per-pixel math
// (assets/compute_shader.wgsl) for gfx950, under the canonical float semantics of
// DESIGN.md §3 (explicit fmaf, IEEE sqrt/div, fixed sin/cos polynomial).  Compiled with
// -ffp-contract=off so that no other fusion happens: the image is bit-identical to the
// CPU oracle's.  The RT_HD functions are also compiled for the host (csrc/rt_abi.cpp
// precomputes per-frame random numbers with them), where they give the same bits.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#define RT_HD __host__ __device__ __forceinline__

// sincos_c's quadrant swap as bit selects (1, default) or selects (0); identical bits
// (with the closed-form disk reciprocal, K2 15.74 against 16.0 us per update,
// profiles/r03/r03a_ab_single.log)
#ifndef RT_SINCOS_BITS
#define RT_SINCOS_BITS 1
#endif

namespace rtd {

struct v3 {
    float x, y, z;
};

RT_HD v3 mk(float x, float y, float z) { return v3{x, y, z}; }
RT_HD v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
RT_HD v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
// p + s*q (contracted)
RT_HD v3 fmas(float s, v3 q, v3 p) {
    return mk(fmaf(s, q.x, p.x), fmaf(s, q.y, p.y), fmaf(s, q.z, p.z));
}
RT_HD float dot(v3 a, v3 b) {
    return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x));
}
RT_HD v3 normalize(v3 v) { return divs(v, sqrtf(dot(v, v))); }

// wgsl:50-59.  Three v_mul_lo_u32 (quarter rate) — the RNG's cost per call.
RT_HD uint32_t hash(uint32_t s) {
    s ^= 2747636419u;
    s *= 2654435769u;
    s ^= s >> 16;
    s *= 2654435769u;
    s ^= s >> 16;
    s *= 2654435769u;
    return s;
}
// wgsl:61-63: f32(hash) / 4294967295.0 where the literal rounds to 2^32 in f32.
RT_HD float rf(uint32_t v) { return (float)hash(v) * 0x1p-32f; }

// WGSL u32(f32): truncate, saturate, NaN -> 0 (what v_cvt_u32_f32 does).
// Branch-free (selects only): NaN and negatives go through fmaxf to 0.
RT_HD uint32_t f2u(float f) {
    const uint32_t t = (uint32_t)fminf(fmaxf(f, 0.0f), 4294967040.0f);  // largest f32 < 2^32
    return f >= 4294967296.0f ? 0xFFFFFFFFu : t;
}

// x with its sign bit xor-ed with m (0 or 0x80000000): the bits of x or -x
RT_HD float flip_sign(float x, uint32_t m) {
    uint32_t u;
    memcpy(&u, &x, 4);
    u ^= m;
    memcpy(&x, &u, 4);
    return x;
}

// Canonical sin/cos: Cody-Waite by pi/2 in three parts, Cephes minimax.
// k1s / k1c: the leading coefficients of the two polynomials, -0x1.9943f2p-13f and
// 0x1.99eb9cp-16f, passed in so that a kernel can keep them in registers (sincos_c below
// passes the literals; the arithmetic is the same either way).
// finite: x is known finite (no NaN guard on the quadrant; the same bits for finite x)
RT_HD void sincos_k(float x, float& s, float& c, float k1s, float k1c, bool finite = false) {
    const float q = rintf(x * 0x1.45f306p-1f);
    const int k = (finite || q == q) ? (int)q : 0;
    float r = fmaf(q, -0x1.921fb6p+0f, x);
    r = fmaf(q, 0x1.777a5cp-25f, r);
    r = fmaf(q, 0x1p-49f, r);
    const float r2 = r * r;
    const float ps = fmaf(fmaf(k1s, r2, 0x1.11073cp-7f), r2, -0x1.555546p-3f);
    const float sr = fmaf(r * r2, ps, r);
    const float pc = fmaf(fmaf(k1c, r2, -0x1.6c0c34p-10f), r2, 0x1.55554ap-5f);
    const float cr = fmaf(r2 * r2, pc, fmaf(-0.5f, r2, 1.0f));
#if RT_SINCOS_BITS
    // the odd-quadrant swap as bit selects under an all-ones mask: on gfx950 one v_bfe_i32
    // and one v_bitop3 per select (no compare writing VCC, no hazard nops); the same bits
    // as the selects below
    float s0, c0;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t sw = (uint32_t)__builtin_amdgcn_sbfe(k, 0, 1);   // 0 or all ones
    uint32_t s0b, c0b;
    // bitop3:0xCA = S0 ? S1 : S2 bitwise (truth table over 0xF0, 0xCC, 0xAA)
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(s0b) : "v"(sw), "v"(cr), "v"(sr));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(c0b) : "v"(sw), "v"(sr), "v"(cr));
    s0 = __uint_as_float(s0b);
    c0 = __uint_as_float(c0b);
#else
    const uint32_t sw = 0u - ((uint32_t)k & 1u);
    uint32_t sb, cb;
    memcpy(&sb, &sr, 4);
    memcpy(&cb, &cr, 4);
    const uint32_t s0b = (cb & sw) | (sb & ~sw), c0b = (sb & sw) | (cb & ~sw);
    memcpy(&s0, &s0b, 4);
    memcpy(&c0, &c0b, 4);
#endif
#else
    const bool swap = (k & 1) != 0;
    const float s0 = swap ? cr : sr;
    const float c0 = swap ? sr : cr;
#endif
    // the quadrant's signs as sign-bit flips (the bits of -x; no compare + select)
    s = flip_sign(s0, ((uint32_t)k << 30) & 0x80000000u);
    c = flip_sign(c0, ((uint32_t)(k + 1) << 30) & 0x80000000u);
}

RT_HD void sincos_c(float x, float& s, float& c) {
    sincos_k(x, s, c, -0x1.9943f2p-13f, 0x1.99eb9cp-16f);
}

// wgsl:234-243; rf_seed = rf(seed)
RT_HD v3 random_unit_vector(float rf_seed, uint32_t seed) {
    const float z = fmaf(2.0f, rf_seed, -1.0f);
    // rf(seed + 1) * 6.283185307f in one rounding (the 2^-32 scale of rf is exact)
    const float a = (float)hash(seed + 1u) * 0x1.921fb6p-30f;
    const float r = sqrtf(fmaf(-z, z, 1.0f));
    float sa, ca;
    sincos_c(a, sa, ca);
    return mk(r * ca, r * sa, z);
}

// WGSL reflect(e1,e2) = e1 - 2*dot(e2,e1)*e2
RT_HD v3 reflect(v3 e1, v3 e2) {
    const float k = 2.0f * dot(e2, e1);
    return fmas(-k, e2, e1);
}

// WGSL refract(e1,e2,eta)
RT_HD v3 refract(v3 e1, v3 e2, float eta) {
    const float d = dot(e2, e1);
    const float k = fmaf(-(eta * eta), fmaf(-d, d, 1.0f), 1.0f);
    if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
    const float m = fmaf(eta, d, sqrtf(k));
    return mk(fmaf(eta, e1.x, -(m * e2.x)), fmaf(eta, e1.y, -(m * e2.y)),
              fmaf(eta, e1.z, -(m * e2.z)));
}

// wgsl:137-141, pow(x, 5.0) = ((x*x)*(x*x))*x
RT_HD float reflectance(float cos_t, float ri) {
    float r0 = (1.0f - ri) / (1.0f + ri);
    r0 = r0 * r0;
    const float x = 1.0f - cos_t;
    const float x2 = x * x;
    return fmaf(1.0f - r0, (x2 * x2) * x, r0);
}

// ---- Exact fast paths of the IEEE f32 division and square root ---------------------
//
// The compiler's correctly rounded a / b (the parity contract) on gfx950 is
//   b' = v_div_scale(b), a' = v_div_scale(a), r = v_rcp(b'), y = fma(fma(-b', r, 1), r, r),
//   q0 = a'*y, q1 = fma(fma(-b', q0, a'), y, q0), q2 = v_div_fmas(fma(-b', q1, a'), y, q1),
//   result = v_div_fixup(q2, b, a).
// div_scale rescales only when b or 1/b is subnormal, |a| < 2^-103, or the exponent gap
// e(a) - e(b) reaches 96 or -126.  On the domain
//     |b| in [2^-20, 2^33),  |a| in [2^-100, 2^91),  e(a) - e(b) in [-120, 88]
// (and for a == +-0, b in that range) it returns its operand unchanged and asks for no
// rescaling, div_fmas is then a plain fma, and div_fixup only restores the sign of a zero
// quotient.  div_core is that unscaled arithmetic, so on this domain it returns exactly the
// bits of a / b — and y, which depends on b only, is shared by every division by the same
// b.  sqrt_core is one residual correction of x * rsq(x), g + (x - g^2) * rsq(x) / 2: five
// VALU operations against the compiler's sixteen (rescaling of x < 2^-96, v_sqrt, a
// two-sided +-1 ulp residual test, the +-0 / +inf fix-up).  It returns the bits of sqrtf
// for every finite x >= 2^-96 — all 1.88e9 of them are compared on the device by the
// self-test — and NaN for +0 and +inf, which are outside its domain.
// Used where the operands are in the domain by construction or by a wave-wide check
// (rt_kernels.hip: defocus disk, roots, normal, sky, metal / dielectric normalisations);
// tests/test_gpu_parity.py::test_fastmath_selftest checks both against the IEEE operations
// on the GPU over that domain, and the root selection built on them against consider().
__device__ __forceinline__ float rcp_refined(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    return fmaf(fmaf(-b, r, 1.0f), r, r);
}
// a / b except for a == -0 with b > 0 (the one case where the unscaled core gets the sign
// of a zero quotient wrong); div_core_signed below covers every sign.
__device__ __forceinline__ float div_core(float a, float b, float y) {
    const float q0 = a * y;
    const float q1 = fmaf(fmaf(-b, q0, a), y, q0);
    return fmaf(fmaf(-b, q1, a), y, q1);
}
// a / b from y = RN32(1 / b), correctly rounded (Markstein): q = RN(a y), the exact residual
// a - b q (one fma), RN(q + residual y).  Exactly the IEEE quotient whenever a, b and the
// quotient are normal and finite (Markstein's theorem: y within half an ulp of 1 / b and q
// within one ulp of a / b); checked by the device self-test (rt_selftest_fastmath) and on the
// host over 10^9 random operands plus every normal numerator for 24 integer divisors
// ("Correctly rounded reciprocals").  For a = -0 it returns +0.
RT_HD float div_rn(float a, float b, float y) {
    const float q = a * y;
    return fmaf(fmaf(-b, q, a), y, q);
}
__device__ __forceinline__ float div_core_signed(float a, float b, float y) {
    const float q0 = a * y;                       // carries sign(a) ^ sign(b), also for a == 0
    return copysignf(div_core(a, b, y), q0);
}
__device__ __forceinline__ float sqrt_core(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float g = x * y, h = 0.5f * y;
    return fmaf(fmaf(-g, g, x), h, g);
}
// sqrt_core(x) and, from the same rsq(x), a refined reciprocal of the result (one Newton
// step, no v_rcp): y is within the accuracy rcp_refined gives (rsq(x) is within ~1.5 ulp of
// 1 / sqrt_core(x), the step squares that), so div_core(a, len, y) is the IEEE a / len on
// div_core's domain (rt_selftest_fastmath replays it: out[1]).
__device__ __forceinline__ float sqrt_core_rcp(float x, float& y) {
    const float r = __builtin_amdgcn_rsqf(x);
    const float g = x * r, h = 0.5f * r;
    const float len = fmaf(fmaf(-g, g, x), h, g);
    y = fmaf(fmaf(-len, r, 1.0f), r, r);
    return len;
}
// |x| as its bit pattern (domain checks on the integer view)
__device__ __forceinline__ uint32_t abs_bits(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }
constexpr uint32_t kBits2m100 = 0x0D800000u;   // 2^-100
constexpr uint32_t kBits2m20 = 0x35800000u;    // 2^-20
constexpr uint32_t kBits2p40 = 0x53800000u;    // 2^40

}  // namespace rtd
