// Practical HBM floor of the progressive update's memory pattern on MI355X: one launch per
// frame reads a 1920x1080 RGBA32F image and writes the other (ping-pong, 16 B + 16 B per
// pixel = 66.4 MB per launch), with no ray tracing at all.  Variants: plain stores,
// write-through (sc1) stores as rt_single_kernel uses, non-temporal loads + stores; one
// float4 per thread or two per thread.  Chains of 200 dependent launches timed with HIP
// events (what bench.py's per-dispatch step sees).
// Build: hipcc --offload-arch=gfx950 -O3 tools/rmw_floor.hip -o tools/rmw_floor
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int kMode, int kPer>
__global__ __launch_bounds__(256) void rmw(const float4* __restrict__ in, float4* __restrict__ out,
                                           uint32_t n) {
    const uint32_t base = (blockIdx.x * 256u * kPer) + threadIdx.x;
    float4 v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = base + k * 256u;
        if (i < n) {
            if (kMode == 2) {
                const u32x4 u = __builtin_nontemporal_load((const u32x4*)in + i);
                v[k] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y),
                                   __uint_as_float(u.z), __uint_as_float(u.w));
            } else {
                v[k] = in[i];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = base + k * 256u;
        if (i >= n) continue;
        const float4 r = make_float4(v[k].x * 0.5f + 1.0f, v[k].y * 0.5f + 1.0f,
                                     v[k].z * 0.5f + 1.0f, v[k].w + 1.0f);
        if (kMode == 1) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                out, 0, (int)(n * 16u), 0x00020000);
            const u32x4 u = {__float_as_uint(r.x), __float_as_uint(r.y), __float_as_uint(r.z),
                             __float_as_uint(r.w)};
            __builtin_amdgcn_raw_buffer_store_b128(u, rs, (int)(i * 16u), 0, 16);
        } else if (kMode == 2) {
            const u32x4 u = {__float_as_uint(r.x), __float_as_uint(r.y), __float_as_uint(r.z),
                             __float_as_uint(r.w)};
            __builtin_nontemporal_store(u, (u32x4*)out + i);
        } else {
            out[i] = r;
        }
    }
}

template <int kMode, int kPer>
static int run(const char* name, float4* a, float4* b, uint32_t n, hipStream_t s) {
    const dim3 grid((n + 256u * kPer - 1u) / (256u * kPer));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 4; ++rep) {
        for (int k = 0; k < 20; ++k) {
            hipLaunchKernelGGL((rmw<kMode, kPer>), grid, dim3(256), 0, s, a, b, n);
            float4* t = a; a = b; b = t;
        }
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < 200; ++k) {
            hipLaunchKernelGGL((rmw<kMode, kPer>), grid, dim3(256), 0, s, a, b, n);
            float4* t = a; a = b; b = t;
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / 200;
        printf("{\"variant\": \"%s\", \"rep\": %d, \"us_per_launch\": %.2f, \"GB_s\": %.0f, "
               "\"frac_of_8TBs\": %.3f}\n", name, rep, us, n * 32.0 / us / 1e3,
               n * 32.0 / us / 1e3 / 8000.0);
    }
    return 0;
}

int main() {
    const uint32_t n = 1920u * 1080u;
    float4 *a, *b;
    CK(hipMalloc(&a, n * 16ull));
    CK(hipMalloc(&b, n * 16ull));
    CK(hipMemset(a, 0, n * 16ull));
    CK(hipMemset(b, 0, n * 16ull));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    if (run<0, 1>("plain, 1 px/thread", a, b, n, s)) return 1;
    if (run<1, 1>("write-through sc1 store, 1 px/thread", a, b, n, s)) return 1;
    if (run<2, 1>("nt load + nt store, 1 px/thread", a, b, n, s)) return 1;
    if (run<0, 2>("plain, 2 px/thread", a, b, n, s)) return 1;
    if (run<1, 2>("write-through sc1 store, 2 px/thread", a, b, n, s)) return 1;
    if (run<1, 4>("write-through sc1 store, 4 px/thread", a, b, n, s)) return 1;
    return 0;
}
