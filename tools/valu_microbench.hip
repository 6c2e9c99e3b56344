// VALU issue-rate microbenchmark for gfx950 (diagnostic tool, not product code).
// Measures cycles per wave64 VALU instruction per SIMD for a few instruction forms, with
// 8 waves per SIMD (2048 blocks of 256 threads on 256 CUs), independent chains.
// Clock: s_memtime (shader clock) vs s_memrealtime (100 MHz) stamped in block 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;


__global__ __launch_bounds__(256) void k0(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k1(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, %3, %2" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k2(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_add_f32 %0, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k3(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k4(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sub_f32 %0, %3, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k5(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_subrev_f32 %0, %3, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k6(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_add_f32 %0, %3, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %3, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %3, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %3, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %3, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %3, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %3, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_f32 %0, %3, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k7(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32 %0, %3, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k8(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k9(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k10(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_f32_e64 %0, %1, -%0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k11(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_max_f32 %0, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_f32 %0, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_f32 %0, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_f32 %0, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_f32 %0, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_f32 %0, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_f32 %0, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_f32 %0, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k12(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_max_i32 %0, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_i32 %0, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_i32 %0, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_i32 %0, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_i32 %0, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_i32 %0, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_i32 %0, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max_i32 %0, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k13(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k14(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k15(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_add_u32 %0, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_u32 %0, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_u32 %0, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_u32 %0, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_u32 %0, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_u32 %0, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_u32 %0, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_add_u32 %0, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k16(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k17(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_mov_b32 %0, %1" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mov_b32 %0, %1" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mov_b32 %0, %1" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mov_b32 %0, %1" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mov_b32 %0, %1" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mov_b32 %0, %1" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mov_b32 %0, %1" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_mov_b32 %0, %1" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k18(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k19(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cmp_lt_f32 vcc, %1, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k20(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_fmac_f32 %0, 0x3f800001, %2" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k21(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p0) : "v"(px)); asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p1) : "v"(px)); asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p2) : "v"(px)); asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p3) : "v"(px));asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p0) : "v"(px)); asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p1) : "v"(px)); asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p2) : "v"(px)); asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p3) : "v"(px)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k22(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_sqrt_f32 %0, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sqrt_f32 %0, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sqrt_f32 %0, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sqrt_f32 %0, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sqrt_f32 %0, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sqrt_f32 %0, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sqrt_f32 %0, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_sqrt_f32 %0, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k23(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_rcp_f32 %0, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_rcp_f32 %0, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_rcp_f32 %0, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_rcp_f32 %0, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_rcp_f32 %0, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_rcp_f32 %0, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_rcp_f32 %0, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_rcp_f32 %0, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

__global__ __launch_bounds__(256) void k24(float* out, unsigned long long* clk, float s0) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = a0 * 0.5f, y = a0 * 0.25f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; const f2 px = {x, y};
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < ITERS; ++i) { asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a0) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a1) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a2) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a3) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a4) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a5) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a6) : "v"(x), "v"(y), "s"(s0));asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a7) : "v"(x), "v"(y), "s"(s0)); }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    f2 q = p0 + p1 + p2 + p3;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + q.x + q.y;
}

template <typename F>
int run(const char* name, F launch, float* d_out, unsigned long long* d_clk, int blocks) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    unsigned long long clk[2];
    CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
    const double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;
    const double waves = blocks * 4.0;
    const double instr = waves * ITERS * 8;              // per kernel, wave-instructions
    const double simd_cycles = ms * 1e-3 * ghz * 1e9 * 1024;  // 256 CUs x 4 SIMDs
    printf("%-22s %8.3f ms  clk %.2f GHz  %.2f cycles/wave-instr/SIMD\n", name, ms, ghz,
           simd_cycles / instr);
    return 0;
}

int main() {
    const int blocks = 2048;
    float* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, blocks * 256 * sizeof(float)));
    CHECK(hipMalloc(&d_clk, 16));
    run("v_fmac_f32 v,v", [&] { hipLaunchKernelGGL(k0, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_fmac_f32 s,v", [&] { hipLaunchKernelGGL(k1, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_add_f32 v,v", [&] { hipLaunchKernelGGL(k2, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_sub_f32 v,v", [&] { hipLaunchKernelGGL(k3, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_sub_f32 s,v", [&] { hipLaunchKernelGGL(k4, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_subrev_f32 s,v", [&] { hipLaunchKernelGGL(k5, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_add_f32 s,v", [&] { hipLaunchKernelGGL(k6, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_mul_f32 s,v", [&] { hipLaunchKernelGGL(k7, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_fma_f32 v,v,v", [&] { hipLaunchKernelGGL(k8, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_fma_f32 -v,v,v", [&] { hipLaunchKernelGGL(k9, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_mul_f32_e64 v,-v", [&] { hipLaunchKernelGGL(k10, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_max_f32 v,v", [&] { hipLaunchKernelGGL(k11, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_max_i32 v,v", [&] { hipLaunchKernelGGL(k12, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_max3_i32 v,v,v", [&] { hipLaunchKernelGGL(k13, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_xor_b32 v,v", [&] { hipLaunchKernelGGL(k14, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_add_u32 v,v", [&] { hipLaunchKernelGGL(k15, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_mul_lo_u32 v,v", [&] { hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_mov_b32 v", [&] { hipLaunchKernelGGL(k17, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_cndmask_b32 (vcc)", [&] { hipLaunchKernelGGL(k18, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_cmp_lt_f32 -> vcc", [&] { hipLaunchKernelGGL(k19, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_fmac_f32 lit", [&] { hipLaunchKernelGGL(k20, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_pk_add_f32", [&] { hipLaunchKernelGGL(k21, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_sqrt_f32", [&] { hipLaunchKernelGGL(k22, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_rcp_f32", [&] { hipLaunchKernelGGL(k23, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    run("v_cvt_f32_u32", [&] { hipLaunchKernelGGL(k24, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 1.f); }, d_out, d_clk, blocks);
    return 0;
}
