// Probe: one-dispatch-per-frame chains submitted as raw AQL packets on our own HSA queue.
//
// Questions (gfx950, ROCm 7.2):
//  P1  does a dispatch whose AQL barrier bit is 0 start before its predecessor on the same
//      queue has finished?
//  P2  are the workgroups of packet k+1 dispatched only after every workgroup of packet k
//      (in-order dispatch: a wave of frame k+1 that waits on a wave of frame k can never
//      block it)?
//  P3  a chain of "frames" (each wave reads its slot sc1, works an uneven time, writes the
//      slot sc1 write-through, drains, publishes a per-slot flag sc1): µs per frame for HIP
//      launches, AQL barrier=1 packets, AQL barrier=0 packets + per-slot flag waits; the
//      final data checked word for word (stale hand-offs would show).
//  P4  host cost per submitted packet.
//  P5  joining a HIP stream: hipStreamWriteValue32 -> a "go" kernel on our queue polls it;
//      our "done" kernel writes signal memory -> hipStreamWaitValue32 on the HIP stream.
// Every spin loop is bounded by s_memrealtime (50 ms) and counts a timeout in err[].
// Build: hipcc --offload-arch=gfx950 -O3 tools/aql_probe.hip -o tools/aql_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char* m_ = ""; \
    hsa_status_string(s_, &m_); printf("%s:%d hsa %d %s\n", __FILE__, __LINE__, (int)s_, m_); \
    return 1; } } while (0)

__device__ __forceinline__ uint64_t rtc() { return __builtin_amdgcn_s_memrealtime(); }
constexpr uint64_t kTimeout = 5000000;   // 50 ms at 100 MHz

extern "C" __global__ void kLong(unsigned long long* t, unsigned long long ticks) {
    const uint64_t t0 = rtc();
    uint64_t t1 = t0;
    while (t1 - t0 < ticks) { __builtin_amdgcn_s_sleep(2); t1 = rtc(); }
    if (threadIdx.x == 0) { t[0] = t0; t[1] = t1; }
}
extern "C" __global__ void kStamp(unsigned long long* t, unsigned slot) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t[slot] = rtc();
}
extern "C" __global__ void kStarts(unsigned long long* starts, unsigned ticks) {
    const uint64_t t0 = rtc();
    if (threadIdx.x == 0) starts[blockIdx.x] = t0;
    uint64_t t1 = t0;
    while (t1 - t0 < ticks) { __builtin_amdgcn_s_sleep(1); t1 = rtc(); }
}
// go: one wave polls *go >= want (sc1 loads), bounded
extern "C" __global__ void kGo(const unsigned* go, unsigned want, unsigned* err) {
    const uint64_t t0 = rtc();
    while (true) {
        unsigned v = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v = __builtin_amdgcn_readfirstlane(v);
        if ((int)(v - want) >= 0) break;
        if (rtc() - t0 > kTimeout) { if (threadIdx.x == 0) atomicAdd(err, 1u); break; }
        __builtin_amdgcn_s_sleep(2);
    }
}
extern "C" __global__ void kDone(unsigned* word, unsigned value) {
    if (threadIdx.x == 0) __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef float f4 __attribute__((ext_vector_type(4)));
// One frame: wave u of the grid owns slot (u * mapmul + mapadd) % nslots.
extern "C" __global__ __launch_bounds__(256) void kFrame(const float4* in, float4* out,
        unsigned* flags, unsigned wait_seq, unsigned pub_seq, const unsigned* cost,
        unsigned* err, unsigned nslots, unsigned mapmul, unsigned mapadd) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned u = blockIdx.x * 4u + wave;
    if (u >= nslots) return;
    const unsigned slot = (unsigned)(((unsigned long long)u * mapmul + mapadd) % nslots);
    if (wait_seq) {
        const uint64_t t0 = rtc();
        while (true) {
            unsigned v = __hip_atomic_load(&flags[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = __builtin_amdgcn_readfirstlane(v);
            if ((int)(v - wait_seq) >= 0) break;
            if (rtc() - t0 > kTimeout) { if (lane == 0) atomicAdd(err, 1u); break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(in + (size_t)slot * 64), 0, 1024, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(out + (size_t)slot * 64), 0, 1024, 0x00020000);
    f4 v = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rin, (int)(lane * 16u), 0, 16));
    float w = v.y;
    const unsigned n = cost[slot];
    for (unsigned i = 0; i < n; ++i) w = fmaf(w, 0.999f, 0.25f);
    v.x += 1.0f;
    v.y = w;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                           rout, (int)(lane * 16u), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
        __hip_atomic_store(&flags[slot], pub_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- HSA plumbing -----------------------------------------------------------------------
struct Sym { uint64_t obj = 0; uint32_t karg = 0, group = 0, priv = 0; };
struct Find { hsa_agent_t agent; const char* name; Sym* out; };
static hsa_ven_amd_loader_1_03_pfn_t g_ld;

static hsa_status_t sym_cb(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void* d) {
    Find* f = (Find*)d;
    hsa_symbol_kind_t kind;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind);
    if (kind != HSA_SYMBOL_KIND_KERNEL) return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    std::string nm(len, '\0');
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &nm[0]);
    const std::string want = f->name;
    if (nm == want || nm == want + ".kd") {
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &f->out->obj);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &f->out->karg);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &f->out->group);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &f->out->priv);
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t exec_cb(hsa_executable_t e, void* d) {
    Find* f = (Find*)d;
    hsa_executable_iterate_agent_symbols(e, f->agent, sym_cb, d);
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t agent_cb(hsa_agent_t a, void* d) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
    auto* v = (std::vector<hsa_agent_t>*)d;
    v->push_back(a);
    return HSA_STATUS_SUCCESS;
}

struct Queue {
    hsa_queue_t* q = nullptr;
    hsa_kernel_dispatch_packet_t* base = nullptr;
    unsigned char* karg_dev = nullptr;       // device kernarg ring
    std::vector<unsigned char> karg_host;
    uint32_t slot_bytes = 512, slots = 8192, next = 0;
};

static uint16_t hdr(bool barrier, int acq, int rel) {
    return (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                      ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                      (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                      (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
}

// kernarg block: explicit bytes, then the COv5 hidden block counts / group sizes at align8
static uint32_t stage_args(Queue& Q, const void* a, uint32_t n, uint32_t gx, uint32_t wg) {
    const uint32_t s = Q.next++ % Q.slots;
    unsigned char* h = Q.karg_host.data() + (size_t)s * Q.slot_bytes;
    std::memset(h, 0, Q.slot_bytes);
    std::memcpy(h, a, n);
    const uint32_t hb = (n + 7u) & ~7u;
    const uint32_t bc[3] = {gx, 1, 1};
    const uint16_t gs[3] = {(uint16_t)wg, 1, 1};
    std::memcpy(h + hb, bc, 12);
    std::memcpy(h + hb + 12, gs, 6);
    const uint16_t dims = 1;
    std::memcpy(h + hb + 64, &dims, 2);
    return s;
}

static void submit(Queue& Q, const Sym& k, uint32_t slot, uint32_t gx, uint32_t wg, bool barrier,
                   int acq, int rel, hsa_signal_t done) {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(Q.q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(Q.q) >= Q.q->size) {}
    hsa_kernel_dispatch_packet_t* p = Q.base + (idx % Q.q->size);
    p->workgroup_size_x = (uint16_t)wg;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = gx * wg;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = k.priv;
    p->group_segment_size = k.group;
    p->kernel_object = k.obj;
    p->kernarg_address = Q.karg_dev + (size_t)slot * Q.slot_bytes;
    p->reserved2 = 0;
    p->completion_signal = done;
    const uint32_t full = hdr(barrier, acq, rel) |
                          ((uint32_t)1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16;
    __atomic_store_n(&p->full_header, full, __ATOMIC_RELEASE);
    hsa_signal_store_relaxed(Q.q->doorbell_signal, (hsa_signal_value_t)idx);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int frames = argc > 1 ? atoi(argv[1]) : 200;
    CK(hipSetDevice(0));
    CK(hipFree(0));
    // make HIP load the code object (the kernels we dispatch ourselves live in it)
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, (const void*)kFrame));
    CK(hipFuncGetAttributes(&fa, (const void*)kLong));
    CK(hipFuncGetAttributes(&fa, (const void*)kStamp));
    CK(hipFuncGetAttributes(&fa, (const void*)kStarts));
    CK(hipFuncGetAttributes(&fa, (const void*)kGo));
    CK(hipFuncGetAttributes(&fa, (const void*)kDone));
    HK(hsa_init());
    std::vector<hsa_agent_t> gpus;
    HK(hsa_iterate_agents(agent_cb, &gpus));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    hsa_agent_t agent{};
    bool found = false;
    for (auto a : gpus) {
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        const uint32_t want = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
        printf("gpu agent bdf=%x dom=%u (hip bus %d dev %d dom %d)\n", bdf, dom, prop.pciBusID,
               prop.pciDeviceID, prop.pciDomainID);
        if ((bdf & ~7u) == want && (int)dom == prop.pciDomainID) { agent = a; found = true; }
    }
    if (!found) { printf("no matching agent\n"); return 1; }
    HK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(g_ld), &g_ld));
    Sym sFrame, sLong, sStamp, sStarts, sGo, sDone;
    const char* names[] = {"kFrame", "kLong", "kStamp", "kStarts", "kGo", "kDone"};
    Sym* syms[] = {&sFrame, &sLong, &sStamp, &sStarts, &sGo, &sDone};
    for (int i = 0; i < 6; ++i) {
        Find f{agent, names[i], syms[i]};
        HK(g_ld.hsa_ven_amd_loader_iterate_executables(exec_cb, &f));
        printf("symbol %s obj=%llx karg=%u group=%u priv=%u\n", names[i],
               (unsigned long long)syms[i]->obj, syms[i]->karg, syms[i]->group, syms[i]->priv);
        if (!syms[i]->obj) return 1;
    }
    Queue Q;
    HK(hsa_queue_create(agent, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX,
                        UINT32_MAX, &Q.q));
    Q.base = (hsa_kernel_dispatch_packet_t*)Q.q->base_address;
    CK(hipMalloc(&Q.karg_dev, (size_t)Q.slots * Q.slot_bytes));
    Q.karg_host.assign((size_t)Q.slots * Q.slot_bytes, 0);
    hsa_signal_t sig;
    HK(hsa_signal_create(1, 0, nullptr, &sig));
    const hsa_signal_t none{0};
    auto flush_args = [&]() -> int {   // stage every block written so far (synchronous copy)
        CK(hipMemcpy(Q.karg_dev, Q.karg_host.data(), Q.karg_host.size(), hipMemcpyHostToDevice));
        return 0;
    };
    auto wait_sig = [&]() -> bool {
        const hsa_signal_value_t v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1,
                                                               2000000000ull, HSA_WAIT_STATE_BLOCKED);
        if (v >= 1) { printf("signal wait timed out\n"); return false; }
        hsa_signal_store_relaxed(sig, 1);
        return true;
    };

    unsigned long long* t;
    unsigned* err;
    CK(hipMalloc(&t, 1 << 20));
    CK(hipMalloc(&err, 64));
    CK(hipMemset(t, 0, 1 << 20));
    CK(hipMemset(err, 0, 64));

    // ---- P1: overlap with the barrier bit clear ----
    for (int variant = 0; variant < 4; ++variant) {
        const int barrier = variant & 1, relA = variant & 2 ? 0 : HSA_FENCE_SCOPE_SYSTEM;
        for (int rep = 0; rep < 2; ++rep) {
            Q.next = 0;
            struct { unsigned long long* t; unsigned long long ticks; } a1{t, 4000};
            struct { unsigned long long* t; unsigned slot; } a2{t, 2};
            uint32_t s1 = stage_args(Q, &a1, sizeof(a1), 1, 64);
            uint32_t s2 = stage_args(Q, &a2, 12, 1, 64);
            if (flush_args()) return 1;
            submit(Q, sLong, s1, 1, 64, true, HSA_FENCE_SCOPE_SYSTEM, relA, none);
            submit(Q, sStamp, s2, 1, 64, barrier, relA ? HSA_FENCE_SCOPE_SYSTEM : 0, HSA_FENCE_SCOPE_SYSTEM, sig);
            if (!wait_sig()) return 1;
            // the stamp may finish first: wait for the long one too
            const uint32_t s3 = stage_args(Q, &a2, 12, 1, 64);
            if (flush_args()) return 1;
            submit(Q, sStamp, s3, 1, 64, true, 0, 0, sig);
            if (!wait_sig()) return 1;
            unsigned long long h[3];
            CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
            printf("P1 barrier=%d releaseA=%d rep=%d A %.2f us, B.start - A.end = %.2f us\n", barrier, relA, rep,
                   (h[1] - h[0]) * 0.01, ((double)h[2] - (double)h[1]) * 0.01);
        }
    }

    // ---- P2: in-order workgroup dispatch across barrier-free packets ----
    {
        const uint32_t G = 16384;
        unsigned long long *sa, *sb;
        CK(hipMalloc(&sa, G * 8));
        CK(hipMalloc(&sb, G * 8));
        for (int rep = 0; rep < 3; ++rep) {
            Q.next = 0;
            struct { unsigned long long* s; unsigned ticks; } a1{sa, 100}, a2{sb, 100};
            uint32_t s1 = stage_args(Q, &a1, 12, G, 256), s2 = stage_args(Q, &a2, 12, G, 256);
            struct { unsigned long long* t; unsigned slot; } a3{t, 3};
            const uint32_t s3 = stage_args(Q, &a3, 12, 1, 64);
            if (flush_args()) return 1;
            submit(Q, sStarts, s1, G, 256, true, HSA_FENCE_SCOPE_SYSTEM, 0, none);
            submit(Q, sStarts, s2, G, 256, false, 0, HSA_FENCE_SCOPE_SYSTEM, none);
            submit(Q, sStamp, s3, 1, 64, true, 0, HSA_FENCE_SCOPE_SYSTEM, sig);
            if (!wait_sig()) return 1;
            std::vector<unsigned long long> ha(G), hb(G);
            CK(hipMemcpy(ha.data(), sa, G * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hb.data(), sb, G * 8, hipMemcpyDeviceToHost));
            unsigned long long amin = ~0ull, amax = 0, bmin = ~0ull, bmax = 0;
            for (uint32_t i = 0; i < G; ++i) {
                amin = std::min(amin, ha[i]); amax = std::max(amax, ha[i]);
                bmin = std::min(bmin, hb[i]); bmax = std::max(bmax, hb[i]);
            }
            uint32_t early = 0;   // B workgroups that started before A's last start
            for (uint32_t i = 0; i < G; ++i) early += hb[i] < amax;
            printf("P2 rep=%d A starts [0, %.2f] us, B starts [%.2f, %.2f] us; B before A's last start: %u\n",
                   rep, (amax - amin) * 0.01, ((double)bmin - amin) * 0.01, ((double)bmax - amin) * 0.01, early);
        }
    }

    // ---- P3/P4: frame chains ----
    const uint32_t nslots = 16384, G = nslots / 4;
    float4 *b0, *b1;
    unsigned *flags, *cost;
    CK(hipMalloc(&b0, (size_t)nslots * 64 * 16));
    CK(hipMalloc(&b1, (size_t)nslots * 64 * 16));
    CK(hipMalloc(&flags, nslots * 4));
    CK(hipMalloc(&cost, nslots * 4));
    std::vector<unsigned> hc(nslots);
    for (uint32_t i = 0; i < nslots; ++i) {
        uint32_t x = i * 2654435769u;
        x ^= x >> 15;
        hc[i] = 40 + (x % 7 == 0 ? 600 : (x % 300));     // uneven: a few slots 10x the rest
    }
    CK(hipMemcpy(cost, hc.data(), nslots * 4, hipMemcpyHostToDevice));
    hipStream_t hs;
    CK(hipStreamCreate(&hs));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    unsigned seq = 0;
    struct FArgs {
        const float4* in; float4* out; unsigned* flags; unsigned wait_seq, pub_seq;
        const unsigned* cost; unsigned* err; unsigned nslots, mapmul, mapadd;
    };
    auto check = [&](float4* buf, int nfr, const char* what) -> int {
        std::vector<float4> h((size_t)nslots * 64);
        CK(hipMemcpy(h.data(), buf, h.size() * 16, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (auto& v : h) bad += v.x != (float)nfr;
        unsigned he[4];
        CK(hipMemcpy(he, err, 16, hipMemcpyDeviceToHost));
        printf("   %s: %zu stale words of %zu, timeouts %u\n", what, bad, h.size(), he[0]);
        return 0;
    };
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 4; ++mode) {
            // mode 0: HIP launches; 1: AQL barrier=1, fences system; 2: AQL barrier=1, no
            // fences between frames; 3: AQL barrier=0 + per-slot flags, no fences between
            const bool vary = true;
            CK(hipMemset(b0, 0, (size_t)nslots * 64 * 16));
            CK(hipMemset(b1, 0, (size_t)nslots * 64 * 16));
            CK(hipMemset(err, 0, 64));
            CK(hipDeviceSynchronize());
            Q.next = 0;
            std::vector<uint32_t> slot(frames);
            std::vector<FArgs> fa(frames);
            const unsigned base = seq;
            for (int f = 0; f < frames; ++f) {
                fa[f] = FArgs{f & 1 ? b1 : b0, f & 1 ? b0 : b1, flags,
                              (mode == 3 && f > 0) ? base + f : 0u, base + f + 1, cost, err,
                              nslots, vary ? (f % 3 == 0 ? 1u : f % 3 == 1 ? 7919u : 104729u) : 1u,
                              vary ? (unsigned)(f * 977) : 0u};
                if (mode) slot[f] = stage_args(Q, &fa[f], sizeof(FArgs), G, 256);
            }
            seq += frames + 1;
            if (mode && flush_args()) return 1;
            double h0 = 0, h1 = 0, hsub = 0;
            float ms = 0;
            if (mode == 0) {
                CK(hipEventRecord(e0, hs));
                h0 = now_us();
                for (int f = 0; f < frames; ++f)
                    hipLaunchKernelGGL(kFrame, dim3(G), dim3(256), 0, hs, fa[f].in, fa[f].out,
                                       fa[f].flags, fa[f].wait_seq, fa[f].pub_seq, fa[f].cost,
                                       fa[f].err, fa[f].nslots, fa[f].mapmul, fa[f].mapadd);
                hsub = now_us() - h0;
                CK(hipEventRecord(e1, hs));
                CK(hipEventSynchronize(e1));
                h1 = now_us();
                CK(hipEventElapsedTime(&ms, e0, e1));
            } else {
                struct { unsigned long long* t; unsigned slot; } a0{t, 4}, a9{t, 5};
                uint32_t s0 = stage_args(Q, &a0, 12, 1, 64), s9 = stage_args(Q, &a9, 12, 1, 64);
                if (flush_args()) return 1;
                h0 = now_us();
                submit(Q, sStamp, s0, 1, 64, true, HSA_FENCE_SCOPE_SYSTEM, 0, none);
                for (int f = 0; f < frames; ++f) {
                    const bool bar = mode != 3;
                    const int acq = mode == 1 ? HSA_FENCE_SCOPE_SYSTEM : f == 0 ? HSA_FENCE_SCOPE_AGENT : 0;
                    const int rel = mode == 1 ? HSA_FENCE_SCOPE_SYSTEM : 0;
                    submit(Q, sFrame, slot[f], G, 256, bar || f == 0, acq, rel, none);
                }
                hsub = now_us() - h0;
                submit(Q, sStamp, s9, 1, 64, true, 0, HSA_FENCE_SCOPE_SYSTEM, sig);
                if (!wait_sig()) return 1;
                h1 = now_us();
                unsigned long long ht[2];
                CK(hipMemcpy(ht, t + 4, 16, hipMemcpyDeviceToHost));
                ms = (float)((ht[1] - ht[0]) * 1e-5);
            }
            printf("P3 rep=%d mode=%d frames=%d: %.2f us/frame (gpu span), host submit %.2f us/frame, wall %.2f us/frame\n",
                   rep, mode, frames, ms * 1e3 / frames, hsub / frames, (h1 - h0) / frames);
            if (check(frames & 1 ? b1 : b0, frames, "final buffer")) return 1;
        }
    }

    // ---- P5: joining a HIP stream ----
    {
      for (int alloc = 0; alloc < 3; ++alloc) {
        unsigned *go = nullptr, *done = nullptr;
        hipError_t ea, eb;
        if (alloc == 0) {
            ea = hipExtMallocWithFlags((void**)&go, 8, hipMallocSignalMemory);
            eb = hipExtMallocWithFlags((void**)&done, 8, hipMallocSignalMemory);
        } else if (alloc == 1) {
            ea = hipExtMallocWithFlags((void**)&go, 64, hipDeviceMallocFinegrained);
            eb = hipExtMallocWithFlags((void**)&done, 64, hipDeviceMallocFinegrained);
        } else {
            ea = hipMalloc((void**)&go, 64);
            eb = hipMalloc((void**)&done, 64);
        }
        printf("P5 alloc=%d (0 signal, 1 finegrained, 2 hipMalloc): %s / %s\n", alloc,
               hipGetErrorString(ea), hipGetErrorString(eb));
        if (ea != hipSuccess || eb != hipSuccess) continue;
        if (alloc) { CK(hipMemset(go, 0, 64)); CK(hipMemset(done, 0, 64)); }
        CK(hipMemset(err, 0, 64));
        CK(hipDeviceSynchronize());
        for (int rep = 0; rep < 3; ++rep) {
            const unsigned want = 100 + rep + 10 * alloc;
            Q.next = 0;
            struct { const unsigned* go; unsigned want; unsigned* err; } ag{go, want, err};
            struct { unsigned* w; unsigned v; } ad{done, want};
            struct { unsigned long long* t; unsigned slot; } a6{t, 6}, a7{t, 7}, a8{t, 8};
            uint32_t sg = stage_args(Q, &ag, 20, 1, 64), s6 = stage_args(Q, &a6, 12, 1, 64),
                     sd = stage_args(Q, &ad, 12, 1, 64);
            if (flush_args()) return 1;
            // HIP stream: a long kernel, then stamp 7 and the go value; our queue: go-wait,
            // stamp 6, done; HIP stream waits for done, then stamp 8
            hipLaunchKernelGGL(kLong, dim3(1), dim3(64), 0, hs, t + 16, 2000ull);
            hipLaunchKernelGGL(kStamp, dim3(1), dim3(64), 0, hs, t, 7u);
            hipError_t ew = hipStreamWriteValue32(hs, go, want, 0);
            hipError_t ev = hipStreamWaitValue32(hs, done, want, hipStreamWaitValueGte, 0xFFFFFFFFu);
            if (ew != hipSuccess || ev != hipSuccess) {
                printf("P5 alloc=%d write %s wait %s\n", alloc, hipGetErrorString(ew), hipGetErrorString(ev));
                CK(hipStreamSynchronize(hs));
                break;
            }
            hipLaunchKernelGGL(kStamp, dim3(1), dim3(64), 0, hs, t, 8u);
            const double w0 = now_us();
            submit(Q, sGo, sg, 1, 64, true, HSA_FENCE_SCOPE_SYSTEM, 0, none);
            submit(Q, sStamp, s6, 1, 64, true, 0, 0, none);
            submit(Q, sDone, sd, 1, 64, true, 0, HSA_FENCE_SCOPE_SYSTEM, sig);
            if (!wait_sig()) return 1;
            CK(hipStreamSynchronize(hs));
            const double w1 = now_us();
            unsigned long long h[9];
            CK(hipMemcpy(h, t, 72, hipMemcpyDeviceToHost));
            unsigned he[1];
            CK(hipMemcpy(he, err, 4, hipMemcpyDeviceToHost));
            printf("P5 alloc=%d rep=%d: stamp6 - stamp7 = %.2f us (go latency), stamp8 - stamp6 = %.2f us (join latency), wall %.1f us, timeouts %u\n",
                   alloc, rep, ((double)h[6] - (double)h[7]) * 0.01, ((double)h[8] - (double)h[6]) * 0.01,
                   w1 - w0, he[0]);
        }
      }
    }
    hsa_signal_destroy(sig);
    hsa_queue_destroy(Q.q);
    printf("done\n");
    return 0;
}
