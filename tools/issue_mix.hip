// Issue-mix microbenchmark (diagnostic tool, not product code): does scalar / branch work
// in a wave's stream cost SIMD issue cycles beside its VALU work?  8 waves per SIMD
// (2048 x 256 threads); per loop iteration: 8 independent v_fma_f32 plus the extra
// instructions named by the kernel.  Prints cycles per iteration per wave-slot.
//   hipcc --offload-arch=gfx950 -O3 tools/issue_mix.hip -o tools/issue_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int ITERS = 2048;
#define FMA8 asm volatile("v_fma_f32 %0, %8, %9, %0\n v_fma_f32 %1, %8, %9, %1\n v_fma_f32 %2, %8, %9, %2\n v_fma_f32 %3, %8, %9, %3\n v_fma_f32 %4, %8, %9, %4\n v_fma_f32 %5, %8, %9, %5\n v_fma_f32 %6, %8, %9, %6\n v_fma_f32 %7, %8, %9, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));
#define KER(NAME, EXTRA)                                                                   \
    __global__ __launch_bounds__(256) void NAME(float* out, unsigned long long* clk) {      \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,         \
              a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                        \
        const float x = a0 * 0.5f, y = a0 * 0.25f;                                          \
        unsigned s0 = blockIdx.x, s1 = blockIdx.x * 3;                                      \
        unsigned long long t0 = 0, r0 = 0;                                                  \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                          \
            t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }     \
        for (int i = 0; i < ITERS; ++i) { FMA8 EXTRA }                                      \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                          \
            clk[0] = __builtin_amdgcn_s_memtime() - t0;                                     \
            clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }                               \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s0 + s1; \
    }
KER(k_fma8, )
KER(k_salu4, asm volatile("s_mov_b32 %0, %1\n s_mov_b32 %1, %0\n s_mov_b32 %0, %1\n s_mov_b32 %1, %0" : "+s"(s0), "+s"(s1));)
KER(k_salu8, asm volatile("s_mov_b32 %0, %1\n s_mov_b32 %1, %0\n s_mov_b32 %0, %1\n s_mov_b32 %1, %0\n s_mov_b32 %0, %1\n s_mov_b32 %1, %0\n s_mov_b32 %0, %1\n s_mov_b32 %1, %0" : "+s"(s0), "+s"(s1));)
KER(k_nop4, asm volatile("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0");)
KER(k_cmp2, asm volatile("v_cmp_lt_f32 vcc, %0, %1\n v_cmp_gt_f32 vcc, %0, %1" :: "v"(a0), "v"(x) : "vcc");)
#define VMOV4 { float t0_; asm volatile("v_mov_b32 %0, %1\n v_mov_b32 %0, %1\n v_mov_b32 %0, %1\n v_mov_b32 %0, %1" : "=v"(t0_) : "v"(x)); s1 += (unsigned)t0_; }
KER(k_vmov4, VMOV4)
#define RL2 { unsigned r; asm volatile("v_readlane_b32 %0, %1, 3\n v_readlane_b32 %0, %1, 5" : "=s"(r) : "v"(a1)); s0 += r; }
KER(k_readlane2, RL2)
template <typename F>
int run(const char* name, F launch, unsigned long long* d_clk, int blocks) {
    hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    launch(); CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) launch(); CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1)); float ms = 0; CHECK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    unsigned long long clk[2]; CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
    const double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;
    const double iters = blocks * 4.0 * ITERS;                   // wave-iterations
    printf("%-12s %8.3f ms  clk %.2f GHz  %.2f cycles/iteration/SIMD (8 fma = %.1f at 2.4)\n",
           name, ms, ghz, ms * 1e-3 * ghz * 1e9 * 1024 / iters, 8 * 2.4);
    return 0;
}
#define RUN(K) run(#K, [&] { hipLaunchKernelGGL(K, dim3(blocks), dim3(256), 0, 0, d_out, d_clk); }, d_clk, blocks)
int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int blocks = 2048; float* d_out; unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, blocks * 256 * sizeof(float))); CHECK(hipMalloc(&d_clk, 16));
    RUN(k_fma8); RUN(k_salu4); RUN(k_salu8); RUN(k_nop4); RUN(k_cmp2); RUN(k_vmov4); RUN(k_readlane2);
    return 0;
}
