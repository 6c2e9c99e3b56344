// Host cost of one kernel launch against the size of its by-value argument block (diagnostic):
// an empty kernel taking a struct of B bytes, launched L times back to back on one stream
// (hipLaunchKernelGGL), host µs per launch; then one launch after the stream drained, host µs
// to return and µs until the stream is idle again (hipStreamSynchronize).  Question it answers:
// how much of rt_update_frames' host time before a frame chain reaches the GPU is the
// 2.5-KB TraceParams block (rt_kernels.h) rather than the launch itself.
// Build: hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o build/launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

template <int B>
struct Blob {
    unsigned char b[B];
};

template <int B>
__global__ void k_empty(Blob<B> a, unsigned* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[B - 1] == 0x5Au) out[0] = a.b[0];
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

template <int B>
static void run(hipStream_t s, unsigned* d) {
    Blob<B> a;
    std::memset(a.b, 1, sizeof(a.b));
    const int L = 2000;
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, s, a, d);
    (void)hipStreamSynchronize(s);
    auto t0 = clk::now();
    for (int i = 0; i < L; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, s, a, d);
    auto t1 = clk::now();
    (void)hipStreamSynchronize(s);
    auto t2 = clk::now();
    // one launch on an idle stream, as a timed call issues it
    double one = 0, rt = 0;
    const int R = 200;
    for (int i = 0; i < R; ++i) {
        auto u0 = clk::now();
        hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, s, a, d);
        auto u1 = clk::now();
        (void)hipStreamSynchronize(s);
        auto u2 = clk::now();
        one += us(u0, u1);
        rt += us(u0, u2);
    }
    std::printf("{\"arg_bytes\": %d, \"host_us_per_launch_back_to_back\": %.2f, "
                "\"gpu_us_per_launch_back_to_back\": %.2f, \"host_us_idle_launch\": %.2f, "
                "\"launch_to_idle_us\": %.2f}\n",
                B, us(t0, t1) / L, us(t0, t2) / L, one / R, rt / R);
}

int main() {
    hipStream_t s;
    unsigned* d;
    if (hipStreamCreate(&s) != hipSuccess || hipMalloc(&d, 64) != hipSuccess) return 1;
    run<64>(s, d);
    run<320>(s, d);
    run<1024>(s, d);
    run<2048>(s, d);
    run<2560>(s, d);
    run<3584>(s, d);
    run<64>(s, d);
    run<2560>(s, d);
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    return 0;
}
