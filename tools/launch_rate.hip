// Host cost of issuing kernels (diagnostic): an empty kernel with a small and with a
// 320-byte argument block, launched N times back to back on one stream and round-robin over
// 2 / 4 streams; prints the host time per launch (the issuing loop alone) and the GPU time
// per launch (until all have run).  Build: hipcc --offload-arch=gfx950 -O2 tools/launch_rate.hip
// -o tools/launch_rate
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

struct Big {
    float v[80];
};

__global__ void k_small(float* out, uint32_t n) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && n == 0xFFFFFFFFu) out[0] = 1.0f;
}
__global__ void k_big(float* out, const Big b) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[79] == -1.0f) out[0] = 1.0f;
}

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main() {
    float* out = nullptr;
    CHECK(hipMalloc(&out, 4));
    hipStream_t s[4];
    for (auto& x : s) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    Big b{};
    const int n = 4000;
    for (int big = 0; big < 2; ++big)
        for (int ns : {1, 2, 4}) {
            for (int rep = 0; rep < 2; ++rep) {   // (first repetition warms up)
                CHECK(hipDeviceSynchronize());
                const auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < n; ++i) {
                    hipStream_t st = s[i % ns];
                    if (big)
                        hipLaunchKernelGGL(k_big, dim3(1024), dim3(256), 0, st, out, b);
                    else
                        hipLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, st, out, (uint32_t)i);
                }
                const auto t1 = std::chrono::steady_clock::now();
                CHECK(hipDeviceSynchronize());
                const auto t2 = std::chrono::steady_clock::now();
                if (rep)
                    std::printf("{\"args\": \"%s\", \"streams\": %d, \"host_us_per_launch\": %.3f, "
                                "\"gpu_us_per_launch\": %.3f}\n",
                                big ? "320 B" : "12 B", ns,
                                std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                                std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
            }
        }
    // the 320-byte kernel through hipModuleLaunchKernel with a cached function handle and a
    // pre-packed argument buffer (HIP_LAUNCH_PARAM_BUFFER_POINTER): no per-launch symbol
    // lookup or per-argument marshalling
    {
        hipFunction_t fn = nullptr;
        CHECK(hipGetFuncBySymbol(&fn, reinterpret_cast<const void*>(&k_big)));
        struct {
            float* out;
            Big b;
        } packed{out, b};
        size_t sz = sizeof(packed);
        void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &packed, HIP_LAUNCH_PARAM_BUFFER_SIZE,
                         &sz, HIP_LAUNCH_PARAM_END};
        for (int ns : {1, 2}) {
            for (int rep = 0; rep < 2; ++rep) {
                CHECK(hipDeviceSynchronize());
                const auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < n; ++i)
                    CHECK(hipModuleLaunchKernel(fn, 1024, 1, 1, 256, 1, 1, 0, s[i % ns], nullptr,
                                                extra));
                const auto t1 = std::chrono::steady_clock::now();
                CHECK(hipDeviceSynchronize());
                const auto t2 = std::chrono::steady_clock::now();
                if (rep)
                    std::printf("{\"args\": \"320 B packed\", \"api\": \"hipModuleLaunchKernel\", "
                                "\"streams\": %d, \"host_us_per_launch\": %.3f, "
                                "\"gpu_us_per_launch\": %.3f}\n", ns,
                                std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                                std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
            }
        }
    }
    // a captured graph of `per` launches (the 320-byte kernel) replayed: host cost of one
    // hipGraphLaunch per `per` kernels
    for (int per : {20, 100}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < per; ++i)
            hipLaunchKernelGGL(k_big, dim3(1024), dim3(256), 0, s[0], out, b);
        CHECK(hipStreamEndCapture(s[0], &g));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const int reps = n / per;
        for (int rep = 0; rep < 2; ++rep) {
            CHECK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < reps; ++i) CHECK(hipGraphLaunch(ge, s[0]));
            const auto t1 = std::chrono::steady_clock::now();
            CHECK(hipDeviceSynchronize());
            const auto t2 = std::chrono::steady_clock::now();
            if (rep)
                std::printf("{\"graph_kernels\": %d, \"host_us_per_kernel\": %.3f, "
                            "\"gpu_us_per_kernel\": %.3f}\n", per,
                            std::chrono::duration<double, std::micro>(t1 - t0).count() / (reps * per),
                            std::chrono::duration<double, std::micro>(t2 - t0).count() / (reps * per));
        }
        CHECK(hipGraphExecDestroy(ge));
        CHECK(hipGraphDestroy(g));
    }
    // instantiation of a captured graph of `per` kernels, and updating every kernel node's
    // arguments of the instantiated graph (hipGraphExecKernelNodeSetParams)
    for (int per : {8, 32, 128}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < per; ++i)
            hipLaunchKernelGGL(k_big, dim3(1024), dim3(256), 0, s[0], out, b);
        CHECK(hipStreamEndCapture(s[0], &g));
        const auto t0 = std::chrono::steady_clock::now();
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const auto t1 = std::chrono::steady_clock::now();
        size_t nn = 0;
        CHECK(hipGraphGetNodes(g, nullptr, &nn));
        hipGraphNode_t nodes[128];
        CHECK(hipGraphGetNodes(g, nodes, &nn));
        float* argp = out;
        Big bb = b;
        void* args[] = {&argp, &bb};
        hipKernelNodeParams kp{};
        CHECK(hipGraphKernelNodeGetParams(nodes[0], &kp));
        kp.kernelParams = args;
        const auto t2 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < nn; ++i) {
            bb.v[0] = (float)i;
            CHECK(hipGraphExecKernelNodeSetParams(ge, nodes[i], &kp));
        }
        const auto t3 = std::chrono::steady_clock::now();
        CHECK(hipGraphLaunch(ge, s[0]));
        CHECK(hipDeviceSynchronize());
        std::printf("{\"graph_kernels\": %d, \"instantiate_us\": %.1f, "
                    "\"set_params_us_per_node\": %.3f}\n", per,
                    std::chrono::duration<double, std::micro>(t1 - t0).count(),
                    std::chrono::duration<double, std::micro>(t3 - t2).count() / nn);
        CHECK(hipGraphExecDestroy(ge));
        CHECK(hipGraphDestroy(g));
    }
    // a small host-to-device copy on the stream: pageable and pinned source
    {
        float* dtab = nullptr;
        CHECK(hipMalloc(&dtab, 8192));
        static float pageable[2048];
        float* pinned = nullptr;
        CHECK(hipHostMalloc(&pinned, 8192, 0));
        for (int pin = 0; pin < 2; ++pin)
            for (int bytes : {1024, 8192}) {
                CHECK(hipDeviceSynchronize());
                const int reps = 500;
                const auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < reps; ++i)
                    CHECK(hipMemcpyAsync(dtab, pin ? pinned : pageable, bytes,
                                         hipMemcpyHostToDevice, s[0]));
                const auto t1 = std::chrono::steady_clock::now();
                CHECK(hipDeviceSynchronize());
                const auto t2 = std::chrono::steady_clock::now();
                std::printf("{\"h2d_bytes\": %d, \"pinned\": %d, \"host_us\": %.3f, "
                            "\"gpu_us\": %.3f}\n", bytes, pin,
                            std::chrono::duration<double, std::micro>(t1 - t0).count() / reps,
                            std::chrono::duration<double, std::micro>(t2 - t0).count() / reps);
            }
        CHECK(hipHostFree(pinned));
        CHECK(hipFree(dtab));
    }
    for (auto& x : s) CHECK(hipStreamDestroy(x));
    CHECK(hipFree(out));
    return 0;
}
