// Probe: can the host write kernel arguments straight into VRAM (large-BAR mapping of the
// GPU's coarse-grained pool) and have a kernel read them back exactly, and what does a write
// + HDP flush + read-back cost?  No AQL packets here: a HIP kernel copies the words.
// Build: hipcc --offload-arch=gfx950 -O3 tools/devkarg_probe.hip -o tools/devkarg_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void kCopy(const unsigned* src, unsigned* dst, unsigned n) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        dst[i] = src[i];
}

struct Agents { hsa_agent_t gpu{}, cpu{}; bool g = false, c = false; uint32_t bdf; };
static hsa_status_t agent_cb(hsa_agent_t a, void* d) {
    Agents* f = (Agents*)d;
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && !f->c) { f->cpu = a; f->c = true; }
    if (t == HSA_DEVICE_TYPE_GPU && !f->g) {
        uint32_t bdf = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        if ((bdf & ~7u) == f->bdf) { f->gpu = a; f->g = true; }
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t pool_cb(hsa_amd_memory_pool_t pool, void* d) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    bool alloc = false;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && alloc) {
        *(hsa_amd_memory_pool_t*)d = pool;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

int main() {
    CK(hipSetDevice(0));
    CK(hipFree(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    if (hsa_init() != HSA_STATUS_SUCCESS) { printf("hsa_init failed\n"); return 1; }
    Agents a;
    a.bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
    hsa_iterate_agents(agent_cb, &a);
    if (!a.g || !a.c) { printf("agents not found\n"); return 1; }
    hsa_amd_memory_pool_t pool{};
    if (hsa_amd_agent_iterate_memory_pools(a.gpu, pool_cb, &pool) != HSA_STATUS_INFO_BREAK) {
        printf("no coarse-grained GPU pool\n"); return 1;
    }
    const size_t bytes = 1 << 20;
    void* p = nullptr;
    hsa_status_t s = hsa_amd_memory_pool_allocate(pool, bytes, 0, &p);
    printf("allocate: %d p=%p\n", (int)s, p);
    if (s != HSA_STATUS_SUCCESS) return 1;
    s = hsa_amd_agents_allow_access(1, &a.cpu, nullptr, p);
    printf("allow_access(cpu): %d\n", (int)s);
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    s = hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr);
    printf("pointer_info: %d type=%d agentBase=%p hostBase=%p size=%zu\n", (int)s, (int)info.type,
           info.agentBaseAddress, info.hostBaseAddress, info.sizeInBytes);
    hsa_amd_hdp_flush_t hdp{};
    s = hsa_agent_get_info(a.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp);
    printf("hdp flush regs: %d mem=%p reg=%p\n", (int)s, (void*)hdp.HDP_MEM_FLUSH_CNTL,
           (void*)hdp.HDP_REG_FLUSH_CNTL);
    if (!info.hostBaseAddress) { printf("not host-accessible: stop\n"); return 0; }
    unsigned* h = (unsigned*)info.hostBaseAddress;
    unsigned* d = nullptr;
    CK(hipMalloc(&d, bytes));
    const unsigned n = bytes / 4;
    for (int rep = 0; rep < 5; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        for (unsigned i = 0; i < n; ++i) h[i] = i * 2654435761u + rep;
        _mm_sfence();
        if (hdp.HDP_MEM_FLUSH_CNTL) {
            *hdp.HDP_MEM_FLUSH_CNTL = 1u;
            (void)*(volatile uint32_t*)hdp.HDP_MEM_FLUSH_CNTL;
        }
        (void)*(volatile unsigned*)(h + n - 1);
        auto t1 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(kCopy, dim3(256), dim3(256), 0, 0, (const unsigned*)p, d, n);
        CK(hipDeviceSynchronize());
        std::vector<unsigned> back(n);
        CK(hipMemcpy(back.data(), d, bytes, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (unsigned i = 0; i < n; ++i) bad += back[i] != i * 2654435761u + rep;
        printf("rep %d: host write 1 MB + flush %.1f us, kernel saw %zu wrong words\n", rep,
               std::chrono::duration<double, std::micro>(t1 - t0).count(), bad);
    }
    // per-packet cost: 512 B writes + sfence + flush + one read-back
    for (int rep = 0; rep < 3; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < 1000; ++k) {
            unsigned* q = h + (k % 1024) * 128;
            for (int i = 0; i < 128; ++i) q[i] = k + i;
            _mm_sfence();
            if (hdp.HDP_MEM_FLUSH_CNTL) {
                *hdp.HDP_MEM_FLUSH_CNTL = 1u;
                (void)*(volatile uint32_t*)hdp.HDP_MEM_FLUSH_CNTL;
            }
            (void)*(volatile unsigned*)(q + 127);
        }
        auto t1 = std::chrono::steady_clock::now();
        printf("512-B slot write + flush + read-back: %.2f us each\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    }
    for (int rep = 0; rep < 3; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < 1000; ++k) {
            unsigned* q = h + (k % 1024) * 128;
            for (int i = 0; i < 128; ++i) q[i] = k + i;
        }
        _mm_sfence();
        auto t1 = std::chrono::steady_clock::now();
        printf("512-B slot write only: %.2f us each\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    }
    hsa_amd_memory_pool_free(p);
    printf("done\n");
    return 0;
}
