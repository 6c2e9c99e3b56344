// Exhaustive check of cheaper f32 square-root sequences against the correctly rounded
// sqrtf over every positive finite x >= 2^-96 (diagnostic for rt_device.h::sqrt_core).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/sqrt_search.hip -o tools/sqrt_search
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void search(unsigned long long* bad, unsigned lo, unsigned hi) {
    unsigned long long b[6] = {0, 0, 0, 0, 0, 0};
    for (unsigned long long u = lo + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
         u < hi; u += (unsigned long long)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((unsigned)u);
        const unsigned want = __float_as_uint(sqrtf(x));
        // E: the raw v_sqrt_f32
        const float s0 = __builtin_amdgcn_sqrtf(x);
        b[0] += __float_as_uint(s0) != want;
        // A: rsq-based one-step correction
        const float y = __builtin_amdgcn_rsqf(x);
        const float g = x * y, h = 0.5f * y;
        const float ra = fmaf(-g, g, x);
        b[1] += __float_as_uint(fmaf(ra, h, g)) != want;
        // B: v_sqrt + residual * 0.5 rsq
        const float rb = fmaf(-s0, s0, x);
        b[2] += __float_as_uint(fmaf(rb, h, s0)) != want;
        // C: v_sqrt + residual * 0.5 rcp(s0)
        const float yc = 0.5f * __builtin_amdgcn_rcpf(s0);
        b[3] += __float_as_uint(fmaf(rb, yc, s0)) != want;
        // D: A with a refined half-reciprocal h' = h + h * (0.5 - g h)
        const float e = fmaf(-g, h, 0.5f);
        const float h2 = fmaf(h, e, h), g2 = fmaf(g, e, g);
        const float rd = fmaf(-g2, g2, x);
        b[4] += __float_as_uint(fmaf(rd, h2, g2)) != want;
        // F: B with the refined h2
        b[5] += __float_as_uint(fmaf(rb, h2, s0)) != want;
    }
    for (int i = 0; i < 6; ++i) atomicAdd(&bad[i], b[i]);
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 6 * sizeof(unsigned long long));
    hipMemset(d, 0, 6 * sizeof(unsigned long long));
    // [2^-96, +inf): biased exponent 31 .. 254
    search<<<8192, 256>>>(d, 0x0F800000u, 0x7F800000u);
    unsigned long long h[6];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[6] = {"E raw v_sqrt", "A rsq one-step", "B sqrt+rsq fix",
                            "C sqrt+rcp fix", "D rsq refined", "F sqrt+refined h"};
    for (int i = 0; i < 6; ++i) printf("%-20s mismatches %llu of %u\n", names[i], h[i],
                                       0x7F800000u - 0x0F800000u);
    return 0;
}
