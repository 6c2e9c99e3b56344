// Dispatch-rate microbenchmark (diagnostic, not the product): how long a grid of small
// workgroups takes when each wave does (a) nothing, (b) one 16-B load + store per lane
// (the accumulator traffic of one `update`), (c) a fixed VALU loop, (d) both — for
// 1-wave and 4-wave workgroups and a persistent grid that walks the same tiles.
// hipcc --offload-arch=gfx950 -O3 tools/dispatch_rate.hip -o tools/dispatch_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <bool kMem, int kSpin>
__device__ __forceinline__ void body(const float4* in, float4* out, unsigned tile) {
    const unsigned i = tile * 64u + (threadIdx.x & 63u);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (kMem) v = in[i];
    float a = (float)i;
#pragma unroll 1
    for (int k = 0; k < kSpin; ++k) a = fmaf(a, 1.0001f, 0.5f);
    v.x += a;
    if (kMem || kSpin) out[i] = v;
}

template <bool kMem, int kSpin>
__global__ void per_tile(const float4* in, float4* out, unsigned tiles) {
    const unsigned tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (tile < tiles) body<kMem, kSpin>(in, out, tile);
}

template <bool kMem, int kSpin>
__global__ void persistent(const float4* in, float4* out, unsigned tiles) {
    const unsigned waves = gridDim.x * (blockDim.x >> 6);
    for (unsigned tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); tile < tiles;
         tile += waves)
        body<kMem, kSpin>(in, out, tile);
}

template <typename F>
float time_us(F launch, int iters = 50) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / iters;
}

template <bool kMem, int kSpin>
void run(const char* name, const float4* in, float4* out, unsigned tiles) {
    const float t1 = time_us([&] { per_tile<kMem, kSpin><<<tiles, 64>>>(in, out, tiles); });
    const float t4 = time_us([&] { per_tile<kMem, kSpin><<<(tiles + 3) / 4, 256>>>(in, out, tiles); });
    const float tp = time_us([&] { persistent<kMem, kSpin><<<2048, 256>>>(in, out, tiles); });
    const float tq = time_us([&] { persistent<kMem, kSpin><<<1024, 256>>>(in, out, tiles); });
    std::printf("{\"case\": \"%s\", \"tiles\": %u, \"wg1_us\": %.2f, \"wg4_us\": %.2f, "
                "\"persist2048x4_us\": %.2f, \"persist1024x4_us\": %.2f}\n",
                name, tiles, t1, t4, tp, tq);
}

int main() {
    const unsigned tiles = 240u * 135u;   // 1920x1080 in 8x8 tiles
    float4 *in = nullptr, *out = nullptr;
    CHECK(hipMalloc(&in, (size_t)tiles * 64 * sizeof(float4)));
    CHECK(hipMalloc(&out, (size_t)tiles * 64 * sizeof(float4)));
    CHECK(hipMemset(in, 0, (size_t)tiles * 64 * sizeof(float4)));
    run<false, 0>("empty", in, out, tiles);
    run<true, 0>("copy16B", in, out, tiles);
    run<false, 256>("spin256", in, out, tiles);
    run<true, 256>("copy16B+spin256", in, out, tiles);
    run<false, 1024>("spin1024", in, out, tiles);
    run<true, 1024>("copy16B+spin1024", in, out, tiles);
    CHECK(hipDeviceSynchronize());
    return 0;
}
