// Probe: does hipExtLaunchKernel(..., hipExtAnyOrderLaunch) let a kernel start before its
// predecessor on the same stream has finished (no AQL barrier bit) on gfx950?
// Kernel A: one workgroup that runs ~40 us (s_memrealtime loop) and records start/end.
// Kernel B: records its start.  Printed: B.start - A.end (negative = overlap), both flags.
// Also times chains of 200 short trace-like launches (64 x 256-thread WGs of busy work)
// with and without the flag.
// Build: hipcc --offload-arch=gfx950 -O3 tools/anyorder_probe.hip -o tools/anyorder_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void kA(unsigned long long* t, uint64_t ticks) {
    const uint64_t t0 = now();
    uint64_t t1 = t0;
    while (t1 - t0 < ticks) { __builtin_amdgcn_s_sleep(2); t1 = now(); }
    if (threadIdx.x == 0) { t[0] = t0; t[1] = t1; }
}
__global__ void kB(unsigned long long* t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t[2] = now();
}
__global__ void kWork(float* out, int iters) {
    float v = threadIdx.x * 1e-3f;
    for (int i = 0; i < iters; ++i) v = fmaf(v, 0.999f, 0.5f);
    if (v == 12345.f) out[blockIdx.x] = v;
}

int main() {
    unsigned long long* t;
    float* o;
    CK(hipMalloc(&t, 64));
    CK(hipMalloc(&o, 1 << 20));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const uint64_t ticks = 4000;   // s_memrealtime is 100 MHz: 40 us
    for (int flag = 0; flag <= 1; ++flag) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemsetAsync(t, 0, 64, s));
            CK(hipStreamSynchronize(s));
            void* aa[] = {&t, (void*)&ticks};
            CK(hipExtLaunchKernel((const void*)kA, dim3(1), dim3(64), aa, 0, s, nullptr, nullptr, 0));
            void* ab[] = {&t};
            CK(hipExtLaunchKernel((const void*)kB, dim3(1), dim3(64), ab, 0, s, nullptr, nullptr, flag));
            CK(hipStreamSynchronize(s));
            unsigned long long h[3];
            CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
            printf("flag=%d rep=%d A %.2f us, B.start - A.end = %.2f us\n", flag, rep,
                   (h[1] - h[0]) * 0.01, ((double)h[2] - (double)h[1]) * 0.01);
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 2000;
    for (int flag = 0; flag <= 1; ++flag) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < 200; ++k) {
                void* aw[] = {&o, (void*)&iters};
                CK(hipExtLaunchKernel((const void*)kWork, dim3(2048), dim3(256), aw, 0, s, nullptr,
                                      nullptr, flag));
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("flag=%d chain of 200 x 2048 WGs: %.2f us per launch\n", flag, ms * 1e3f / 200);
        }
    }
    return 0;
}
