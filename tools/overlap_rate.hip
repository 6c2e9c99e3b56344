// Overlap microbenchmark (diagnostic, not the product): does one 16-B-per-lane
// accumulator read-modify-write per tile overlap with VALU work on MI355X?  Per tile: load
// (optional), N independent FMAs in four chains (issue-bound), store.  Three launch
// shapes: one-wave workgroups (one tile each), four-wave workgroups, and a persistent
// grid whose waves prefetch the next tile's texel before computing the current one.
// hipcc --offload-arch=gfx950 -O3 tools/overlap_rate.hip -o tools/overlap_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int kN>
__device__ __forceinline__ float4 work(float4 v) {
    float a = v.x, b = v.y, c = v.z, d = v.w;
#pragma unroll 8
    for (int k = 0; k < kN / 4; ++k) {
        a = fmaf(a, 1.0001f, 0.5f);
        b = fmaf(b, 0.9999f, 0.25f);
        c = fmaf(c, 1.0002f, 0.125f);
        d = fmaf(d, 0.9998f, 0.0625f);
    }
    return make_float4(a, b, c, d);
}

template <bool kMem, int kN>
__global__ void per_tile(const float4* in, float4* out, unsigned tiles) {
    const unsigned tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (tile >= tiles) return;
    const unsigned i = tile * 64u + (threadIdx.x & 63u);
    float4 v = kMem ? in[i] : make_float4((float)i, 1.f, 2.f, 3.f);
    out[i] = work<kN>(v);
}

template <bool kMem, int kN>
__global__ __launch_bounds__(256) void persistent(const float4* in, float4* out, unsigned tiles) {
    const unsigned waves = gridDim.x * (blockDim.x >> 6);
    unsigned tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (tile >= tiles) return;
    const unsigned lane = threadIdx.x & 63u;
    float4 next = kMem ? in[tile * 64u + lane] : make_float4((float)tile, 1.f, 2.f, 3.f);
    for (;;) {
        const unsigned cur = tile;
        const float4 v = next;
        tile += waves;
        const bool more = tile < tiles;
        if (more) next = kMem ? in[tile * 64u + lane] : make_float4((float)tile, 1.f, 2.f, 3.f);
        out[cur * 64u + lane] = work<kN>(v);
        if (!more) break;
    }
}

template <typename F>
float time_us(F launch, int iters = 40) {
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

template <bool kMem, int kN>
void run(const float4* in, float4* out, unsigned tiles, int resident_wgs) {
    const float t1 = time_us([&] { per_tile<kMem, kN><<<tiles, 64>>>(in, out, tiles); });
    const float t4 = time_us([&] { per_tile<kMem, kN><<<(tiles + 3) / 4, 256>>>(in, out, tiles); });
    const float tp = time_us([&] { persistent<kMem, kN><<<resident_wgs, 256>>>(in, out, tiles); });
    std::printf("{\"mem\": %d, \"fma_per_lane\": %d, \"wg1_us\": %.2f, \"wg4_us\": %.2f, "
                "\"persist_prefetch_us\": %.2f}\n", (int)kMem, kN, t1, t4, tp);
}

int main() {
    const unsigned tiles = 240u * 135u;   // 1920x1080 in 8x8 tiles
    float4 *in = nullptr, *out = nullptr;
    CHECK(hipMalloc(&in, (size_t)tiles * 64 * sizeof(float4)));
    CHECK(hipMalloc(&out, (size_t)tiles * 64 * sizeof(float4)));
    CHECK(hipMemset(in, 0, (size_t)tiles * 64 * sizeof(float4)));
    int per_cu = 0, cus = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent<true, 256>, 256, 0));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::printf("{\"resident_wgs\": %d}\n", per_cu * cus);
    const int r = per_cu * cus;
    run<false, 0>(in, out, tiles, r);
    run<true, 0>(in, out, tiles, r);
    run<false, 128>(in, out, tiles, r);
    run<true, 128>(in, out, tiles, r);
    run<false, 256>(in, out, tiles, r);
    run<true, 256>(in, out, tiles, r);
    run<false, 512>(in, out, tiles, r);
    run<true, 512>(in, out, tiles, r);
    run<false, 1024>(in, out, tiles, r);
    run<true, 1024>(in, out, tiles, r);
    CHECK(hipDeviceSynchronize());
    return 0;
}
