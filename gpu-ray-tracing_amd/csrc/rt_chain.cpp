// rt_chain.cpp — one-frame `update` dispatches submitted as AQL packets on HSA queues the
// context owns (rt_set_update_submit; AUTO uses it for mid-sized rank shares, rt_abi.cpp
// usable_chain): the per-frame dispatch loop of ComputeShaderNode::run (lib.rs:366-374,
// 408-417) with a host cost of a packet write per frame instead of a HIP launch.
//
// A HIP launch costs the host 2.7-4.4 µs (profiles/r03*_launch_rate.jsonl), which bounds
// how many concurrent parts a small rank share can use, and HIP's dispatches carry cache
// fences at every kernel boundary.  Here every frame of every part is one
// hsa_kernel_dispatch_packet_t on that part's queue (≈0.25 µs of host time each,
// profiles/r03/r03r_aql_probe.txt):
//   * a part's frames run in order on its queue (barrier bit set: frame f + 1 reads the
//     pixels frame f wrote); parts run concurrently on their own queues, as the HIP path's
//     streams do;
//   * no cache fence between the frames of a segment: the chain kernels store the image
//     write-through (sc1) and load the accumulator with sc1 loads (L1 bypassed), the
//     hand-off form of MI355X_MICROARCH.md §inter-workgroup visibility; each queue's first
//     packet of a segment acquires at system scope (kernel arguments, lists, the input image
//     written before the segment), the done packet releases at system scope;
//   * ordering with the caller's stream: if the stream is busy when the segment is submitted,
//     it writes a "go" word (hipStreamWriteValue32) and queue 0's first packet is a one-wave
//     kernel that waits for it (bounded); the other queues wait for that packet through an
//     AQL barrier-AND packet.  The segment ends with a barrier-AND on queue 0 over the other
//     queues' last packets and a one-wave kernel that writes a "done" word, which the
//     caller's stream waits for (hipStreamWaitValue32) — the call stays asynchronous and
//     ordered on the caller's stream like the HIP path.
// Kernel arguments: written by the host before their packet is submitted (the command
// processor reads a packet's preloaded leading arguments when it fetches the packet, which
// can be before the packet's barrier resolves), in pinned host memory allocated non-coherent
// so that the waves' scalar loads of the parameter block are served by L2 after the first
// miss (fine-grained host memory is read over PCIe by every wave: 115 µs per K3 update
// against 19.5, profiles/r03/r03r_ab.log).  Each queue's first packet of a segment acquires at
// system scope, which drops any line of a reused argument slot cached before the host
// rewrote it.  A set's slots are rewritten only after its previous segment has completed.
#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_internal.h"
#include "rt_kernels.h"

namespace rtc {

namespace {

constexpr uint32_t kMaxQueues = 4;
constexpr uint32_t kQueuePackets = 1024;      // per queue (power of two)
constexpr uint32_t kSlotBytes = 512;          // kernel arguments per packet (>= chain_args)
constexpr uint32_t kSets = 4;                 // segments in flight (signals, argument buffers)
// VRAM argument ring: a slot is rewritten only after ~kRingSlots other packets (at most kSets
// segments of at most kMaxSegmentPackets each are in flight), so no cache can still hold the
// line it read last time; each queue's first packet of a segment acquires at system scope too.
constexpr uint32_t kRingSlots = 65536;
static_assert(kSets * kMaxSegmentPackets * 8 <= kRingSlots, "argument ring");

struct KernelObj {
    uint64_t object = 0;
    uint32_t kernarg = 0, group = 0, priv = 0;
};

// A segment in flight: its signals, kernel-argument buffers and packed frame packets.
struct Pending {
    uint32_t part, gx, gy, threads;
    int which;
};
struct SignalSet {
    hsa_signal_t go{}, last[kMaxQueues]{}, done{};
    bool used = false;
    unsigned char* args = nullptr;    // pinned host, non-coherent: kMaxSegmentPackets slots
    unsigned char* small = nullptr;   // host kernarg pool: the go and the done packet's
    std::vector<Pending> frames;
};

}  // namespace

struct Chain {
    int device = 0;
    bool ok = false;
    bool hsa_up = false;                   // hsa_init succeeded (hsa_shut_down in destroy)
    std::string why = "not initialised";
    // A failed chain (a go wait that gave up, a queue error, a segment that did not complete
    // within the bound) takes no more segments: the context runs HIP launches from then on.
    bool failed = false;
    std::atomic<int> queue_error{0};       // hsa_status_t from the queues' error callback
    hsa_agent_t gpu{}, cpu{};
    hsa_queue_t* q[kMaxQueues] = {};
    KernelObj k[rtk::kChainKernels];
    unsigned char* small = nullptr;        // host kernarg pool, 2 slots per set
    // frame packets' arguments: a ring in VRAM the host writes through its large-BAR mapping
    // (one HDP flush + read-back per segment), or per-set non-coherent host buffers
    unsigned char* ring = nullptr;
    uint32_t ring_head = 0;
    uint32_t* hdp_flush = nullptr;
    unsigned char* seg_args = nullptr;     // the open segment's first slot
    SignalSet sets[kSets];
    uint32_t set = 0;                      // set of the open / next segment
    uint32_t* go = nullptr;                // signal memory: the caller's stream writes seq
    uint32_t* done = nullptr;              // signal memory: the done packet writes seq
    // A go wait that gives up writes both words: `abort` in device memory (every chain
    // kernel checks it before its image stores, so no frame of a segment runs before the
    // caller's stream has reached it: the segment's frames are dropped instead) and
    // `gave_up` in coherent host memory (read by the host without a synchronisation).
    uint32_t* abort = nullptr;
    volatile uint32_t* gave_up = nullptr;
    uint64_t go_ticks = 0;                 // the go wait's bound (s_memrealtime, 100 MHz)
    uint32_t seq = 0;
    // the open segment
    bool open = false;
    uint32_t seg_parts = 0;
    uint64_t packets = 0;                  // submitted since creation (diagnostic)
};

namespace {

struct FindAgent {
    uint32_t bdf, domain;
    hsa_agent_t gpu{}, cpu{};
    bool have_gpu = false, have_cpu = false;
};

hsa_status_t agent_cb(hsa_agent_t a, void* d) {
    FindAgent* f = static_cast<FindAgent*>(d);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) {
        f->cpu = a;
        f->have_cpu = true;
    } else if (t == HSA_DEVICE_TYPE_GPU) {
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        if ((bdf & ~7u) == f->bdf && dom == f->domain) {
            f->gpu = a;
            f->have_gpu = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

struct FindSyms {
    hsa_agent_t agent;
    KernelObj* out;
};

hsa_status_t sym_cb(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void* d) {
    FindSyms* f = static_cast<FindSyms*>(d);
    hsa_symbol_kind_t kind;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) !=
            HSA_STATUS_SUCCESS ||
        kind != HSA_SYMBOL_KIND_KERNEL)
        return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    std::string nm(len, '\0');
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &nm[0]);
    for (int i = 0; i < rtk::kChainKernels; ++i) {
        if (nm.find(rtk::chain_kernel_symbol(i)) == std::string::npos) continue;
        KernelObj& k = f->out[i];
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE,
                                       &k.kernarg);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE,
                                       &k.group);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE,
                                       &k.priv);
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t exec_cb(hsa_executable_t e, void* d) {
    FindSyms* f = static_cast<FindSyms*>(d);
    hsa_executable_iterate_agent_symbols(e, f->agent, sym_cb, d);
    return HSA_STATUS_SUCCESS;
}

hsa_status_t vram_pool_cb(hsa_amd_memory_pool_t pool, void* d) {
    hsa_amd_segment_t seg;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) !=
            HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    bool alloc = false;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && alloc) {
        *static_cast<hsa_amd_memory_pool_t*>(d) = pool;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t kernarg_pool_cb(hsa_amd_memory_pool_t pool, void* d) {
    hsa_amd_segment_t seg;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) !=
            HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
        *static_cast<hsa_amd_memory_pool_t*>(d) = pool;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

uint16_t header(hsa_packet_type_t type, bool barrier, int acquire, int release) {
    return (uint16_t)((type << HSA_PACKET_HEADER_TYPE) |
                      ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                      (acquire << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                      (release << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
}

// The next packet slot of q (waits while the queue is full: the command processor frees
// slots as it consumes packets).
uint64_t reserve(hsa_queue_t* q, void** pkt) {
    const uint64_t idx = hsa_queue_add_write_index_scacq_screl(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
    }
    *pkt = static_cast<unsigned char*>(q->base_address) + (idx & (q->size - 1)) * 64;
    return idx;
}

void publish(hsa_queue_t* q, uint64_t idx, void* pkt, uint32_t full_header) {
    __atomic_store_n(static_cast<uint32_t*>(pkt), full_header, __ATOMIC_RELEASE);
    hsa_signal_store_relaxed(q->doorbell_signal, (hsa_signal_value_t)idx);
}

void dispatch(Chain* c, uint32_t qi, const KernelObj& k, const void* karg, uint32_t gx,
              uint32_t gy, uint32_t threads, int acquire, int release, hsa_signal_t done) {
    hsa_queue_t* q = c->q[qi];
    void* v = nullptr;
    const uint64_t idx = reserve(q, &v);
    hsa_kernel_dispatch_packet_t* p = static_cast<hsa_kernel_dispatch_packet_t*>(v);
    p->workgroup_size_x = (uint16_t)threads;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = gx * threads;
    p->grid_size_y = gy;
    p->grid_size_z = 1;
    p->private_segment_size = k.priv;
    p->group_segment_size = k.group;
    p->kernel_object = k.object;
    p->kernarg_address = const_cast<void*>(karg);
    p->reserved2 = 0;
    p->completion_signal = done;
    const uint32_t dims = gy > 1 ? 2u : 1u;
    publish(q, idx, v,
            header(HSA_PACKET_TYPE_KERNEL_DISPATCH, true, acquire, release) |
                ((dims << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16));
    c->packets++;
}

void barrier_and(Chain* c, uint32_t qi, const hsa_signal_t* deps, uint32_t n) {
    hsa_queue_t* q = c->q[qi];
    void* v = nullptr;
    const uint64_t idx = reserve(q, &v);
    hsa_barrier_and_packet_t* p = static_cast<hsa_barrier_and_packet_t*>(v);
    p->reserved0 = 0;
    p->reserved1 = 0;
    for (uint32_t i = 0; i < 5; ++i) p->dep_signal[i] = i < n ? deps[i] : hsa_signal_t{0};
    p->reserved2 = 0;
    p->completion_signal = hsa_signal_t{0};
    publish(q, idx, v, header(HSA_PACKET_TYPE_BARRIER_AND, true, HSA_FENCE_SCOPE_NONE,
                              HSA_FENCE_SCOPE_NONE));
    c->packets++;
}

// The go wait's bound (RT_CHAIN_GO_MS, default 10 s: the caller's stream work queued ahead
// of a segment) and the host's bound on a segment's completion: the go bound plus 10 s.
uint64_t go_bound_ms() {
    const char* e = std::getenv("RT_CHAIN_GO_MS");
    const long v = e ? std::strtol(e, nullptr, 10) : 0;
    return v > 0 ? (uint64_t)v : 10000u;
}

// Waits until s reaches 0, at most `ms` milliseconds; false on timeout (the caller fails the
// chain instead of hanging the process).
bool wait_zero(hsa_signal_t s, uint64_t ms) {
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
    for (;;) {
        // (the timeout is a hint: the loop re-checks the clock)
        if (hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_EQ, 0, 100000000ull,
                                      HSA_WAIT_STATE_BLOCKED) == 0)
            return true;
        if (std::chrono::steady_clock::now() >= t_end) return false;
    }
}

uint64_t wait_bound_ms(const Chain* c) { return c->go_ticks / 100000u + 10000u; }

// Queue errors (a malformed packet, a memory fault in a chain kernel) arrive here on the
// runtime's thread: the chain is marked failed.
void queue_error_cb(hsa_status_t status, hsa_queue_t*, void* data) {
    static_cast<Chain*>(data)->queue_error.store((int)status);
}

hsa_status_t make_queue(Chain* c, hsa_queue_t** q) {
    return hsa_queue_create(c->gpu, kQueuePackets, HSA_QUEUE_TYPE_SINGLE, queue_error_cb, c,
                            UINT32_MAX, UINT32_MAX, q);
}

rt_status setup(Chain* c) {
    hipDeviceProp_t prop;
    hipError_t he = hipGetDeviceProperties(&prop, c->device);
    if (he != hipSuccess) return rti::hip_fail(he, "hipGetDeviceProperties");
    // (the code object's symbols appear to HSA once HIP has loaded it on this device)
    he = rtk::chain_load_kernels();
    if (he != hipSuccess) return rti::hip_fail(he, "chain kernels (hipGetFuncBySymbol)");
    if (hsa_init() != HSA_STATUS_SUCCESS) {
        c->why = "hsa_init failed";
        return RT_OK;
    }
    c->hsa_up = true;
    c->go_ticks = go_bound_ms() * 100000ull;
    FindAgent fa;
    fa.bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
    fa.domain = (uint32_t)prop.pciDomainID;
    hsa_iterate_agents(agent_cb, &fa);
    if (!fa.have_gpu || !fa.have_cpu) {
        c->why = "no HSA agent with the HIP device's PCI address";
        return RT_OK;
    }
    c->gpu = fa.gpu;
    c->cpu = fa.cpu;
    hsa_ven_amd_loader_1_03_pfn_t ld;
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ld), &ld) !=
        HSA_STATUS_SUCCESS) {
        c->why = "no HSA loader extension";
        return RT_OK;
    }
    FindSyms fs{c->gpu, c->k};
    ld.hsa_ven_amd_loader_iterate_executables(exec_cb, &fs);
    for (int i = 0; i < rtk::kChainKernels; ++i) {
        if (!c->k[i].object) {
            c->why = std::string("chain kernel not found: ") + rtk::chain_kernel_symbol(i);
            return RT_OK;
        }
        if (c->k[i].kernarg > kSlotBytes) {
            c->why = "chain kernel arguments exceed a slot";
            return RT_OK;
        }
    }
    hsa_amd_memory_pool_t pool{};
    if (hsa_amd_agent_iterate_memory_pools(c->cpu, kernarg_pool_cb, &pool) !=
            HSA_STATUS_INFO_BREAK ||
        hsa_amd_memory_pool_allocate(pool, (size_t)kSets * 2 * kSlotBytes, 0,
                                     reinterpret_cast<void**>(&c->small)) != HSA_STATUS_SUCCESS) {
        c->why = "no kernarg memory";
        c->small = nullptr;
        return RT_OK;
    }
    if (hsa_amd_agents_allow_access(1, &c->gpu, nullptr, c->small) != HSA_STATUS_SUCCESS) {
        c->why = "kernarg memory not accessible by the GPU";
        return RT_OK;
    }
    for (uint32_t i = 0; i < kSets; ++i) c->sets[i].small = c->small + (size_t)i * 2 * kSlotBytes;
    // the argument ring in VRAM, host-visible (large BAR) and flushed through the HDP
    hsa_amd_memory_pool_t vpool{};
    hsa_amd_hdp_flush_t hdp{};
    void* ring = nullptr;
    if (hsa_amd_agent_iterate_memory_pools(c->gpu, vram_pool_cb, &vpool) == HSA_STATUS_INFO_BREAK &&
        hsa_agent_get_info(c->gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp) ==
            HSA_STATUS_SUCCESS &&
        hdp.HDP_MEM_FLUSH_CNTL &&
        hsa_amd_memory_pool_allocate(vpool, (size_t)kRingSlots * kSlotBytes, 0, &ring) ==
            HSA_STATUS_SUCCESS) {
        hsa_amd_pointer_info_t info;
        std::memset(&info, 0, sizeof(info));
        info.size = sizeof(info);
        if (hsa_amd_agents_allow_access(1, &c->cpu, nullptr, ring) == HSA_STATUS_SUCCESS &&
            hsa_amd_pointer_info(ring, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
            info.hostBaseAddress == ring) {
            c->ring = static_cast<unsigned char*>(ring);
            c->hdp_flush = hdp.HDP_MEM_FLUSH_CNTL;
        } else {
            hsa_amd_memory_pool_free(ring);
        }
    }
    for (uint32_t i = 0; i < kSets && !c->ring; ++i) {
        const size_t bytes = (size_t)rtc::kMaxSegmentPackets * kSlotBytes;
        he = hipHostMalloc(reinterpret_cast<void**>(&c->sets[i].args), bytes,
                           hipHostMallocNonCoherent);
        if (he != hipSuccess) return rti::hip_fail(he, "chain argument buffers");
    }
    for (SignalSet& s : c->sets) s.frames.reserve(rtc::kMaxSegmentPackets);
    for (SignalSet& s : c->sets) {
        bool ok = hsa_signal_create(0, 0, nullptr, &s.go) == HSA_STATUS_SUCCESS &&
                  hsa_signal_create(0, 0, nullptr, &s.done) == HSA_STATUS_SUCCESS;
        for (uint32_t i = 0; ok && i < kMaxQueues; ++i)
            ok = hsa_signal_create(0, 0, nullptr, &s.last[i]) == HSA_STATUS_SUCCESS;
        if (!ok) {
            c->why = "hsa_signal_create failed";
            return RT_OK;
        }
    }
    // go and done words: signal memory (hipStreamWriteValue32 / hipStreamWaitValue32
    // targets); the go kernel's abort word (device) and give-up flag (coherent host memory)
    he = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->go), 8, hipMallocSignalMemory);
    if (he == hipSuccess)
        he = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->done), 8, hipMallocSignalMemory);
    if (he == hipSuccess) he = hipMalloc(&c->abort, sizeof(uint32_t));
    if (he == hipSuccess) he = hipMemset(c->abort, 0, sizeof(uint32_t));
    void* gu = nullptr;
    if (he == hipSuccess) he = hipHostMalloc(&gu, sizeof(uint32_t), hipHostMallocCoherent);
    if (he == hipSuccess) {
        c->gave_up = static_cast<volatile uint32_t*>(gu);
        *c->gave_up = 0u;
    }
    if (he == hipSuccess) he = hipMemset(c->go, 0, 8);
    if (he == hipSuccess) he = hipMemset(c->done, 0, 8);
    if (he == hipSuccess) he = hipDeviceSynchronize();
    if (he != hipSuccess) return rti::hip_fail(he, "chain words");
    // (queues are created as segments need them: chain_queues; an idle context holds none)
    c->why = "";
    c->ok = true;
    return RT_OK;
}

}  // namespace

Chain* chain_create(int device, rt_status* status) {
    Chain* c = new (std::nothrow) Chain;
    if (!c) {
        *status = rti::fail(RT_ERR_NO_MEMORY, "chain: out of memory");
        return nullptr;
    }
    c->device = device;
    *status = setup(c);
    return c;
}

rt_status chain_destroy(Chain* c) {
    if (!c) return RT_OK;
    // every segment in flight completes within the bound (its go wait is bounded too); one
    // that does not leaves its queues, signals and argument memory in place (the GPU may
    // still read them) and the call reports the error
    for (SignalSet& s : c->sets)
        if (s.used && !wait_zero(s.done, wait_bound_ms(c)))
            return rti::fail(RT_ERR_HIP, "AQL segment did not complete: chain resources leaked");
    for (hsa_queue_t* q : c->q)
        if (q) hsa_queue_destroy(q);
    for (SignalSet& s : c->sets) {
        if (s.go.handle) hsa_signal_destroy(s.go);
        if (s.done.handle) hsa_signal_destroy(s.done);
        for (hsa_signal_t t : s.last)
            if (t.handle) hsa_signal_destroy(t);
    }
    for (SignalSet& s : c->sets) (void)hipHostFree(s.args);
    if (c->ring) hsa_amd_memory_pool_free(c->ring);
    if (c->small) hsa_amd_memory_pool_free(c->small);
    (void)hipFree(c->go);
    (void)hipFree(c->done);
    (void)hipFree(c->abort);
    if (c->gave_up) (void)hipHostFree(const_cast<uint32_t*>(c->gave_up));
    if (c->hsa_up) hsa_shut_down();
    delete c;
    return RT_OK;
}

// Marks the chain failed (and why) if a go wait gave up or a queue reported an error since
// the last check; true if it has failed.  No synchronisation: both flags live in host memory.
bool chain_failed(Chain* c) {
    if (!c) return false;
    if (!c->failed) {
        const int qe = c->queue_error.load();
        if (qe != 0) {
            c->failed = true;
            c->why = "HSA queue error " + std::to_string(qe);
        } else if (c->gave_up && *c->gave_up != 0u) {
            c->failed = true;
            c->why = "a segment's go wait gave up (the caller's stream had not reached it "
                     "within the bound): its frames were dropped";
        }
    }
    return c->failed;
}

bool chain_ok(const Chain* c, const char** why) {
    if (why) *why = c ? c->why.c_str() : "no chain";
    return c && c->ok && !c->failed;
}

bool chain_queues(Chain* c, uint32_t parts) {
    // one HSA queue per part, created on first use (idle queues still occupy the device's
    // hardware queue slots, which HIP's own streams share)
    if (!c || !c->ok || c->failed) return false;
    for (uint32_t k = 0; k < parts && k < kMaxQueues; ++k) {
        if (c->q[k]) continue;
        if (make_queue(c, &c->q[k]) != HSA_STATUS_SUCCESS) {
            c->q[k] = nullptr;
            return false;
        }
    }
    return true;
}

rt_status chain_begin(Chain* c, hipStream_t stream, uint32_t parts) {
    (void)stream;
    if (!c->ok || c->open) return rti::fail(RT_ERR_INVALID_ARGUMENT, "chain_begin");
    if (chain_failed(c)) return rti::fail(RT_ERR_HIP, "AQL submission failed: " + c->why);
    parts = parts < 1u ? 1u : parts > kMaxQueues ? kMaxQueues : parts;
    if (!chain_queues(c, parts)) return rti::fail(RT_ERR_HIP, "hsa_queue_create failed");
    SignalSet& s = c->sets[c->set];
    // this set's previous segment (and its buffers) is done
    if (s.used && !wait_zero(s.done, wait_bound_ms(c))) {
        c->failed = true;
        c->why = "an AQL segment did not complete within the bound";
        return rti::fail(RT_ERR_HIP, c->why);
    }
    s.frames.clear();
    if (c->ring) {
        if (c->ring_head + kMaxSegmentPackets > kRingSlots) c->ring_head = 0;
        c->seg_args = c->ring + (size_t)c->ring_head * kSlotBytes;
    } else {
        c->seg_args = s.args;
    }
    c->open = true;
    c->seg_parts = parts;
    return RT_OK;
}

rt_status chain_frame(Chain* c, const rtk::TraceParams& p, int kernel, uint32_t part) {
    if (!c->open || part >= c->seg_parts) return rti::fail(RT_ERR_INVALID_ARGUMENT, "chain_frame");
    SignalSet& s = c->sets[c->set];
    if (s.frames.size() >= kMaxSegmentPackets)
        return rti::fail(RT_ERR_INVALID_ARGUMENT, "chain segment too long");
    unsigned char* a = c->seg_args + s.frames.size() * kSlotBytes;
    uint32_t grid[2] = {0, 0}, threads = 0;
    int which = 0;
    const uint32_t n =
        rtk::chain_args(p, kernel, c->abort, a, kSlotBytes, grid, &threads, &which);
    if (n == 0) return RT_OK;                // an empty part
    if (c->k[which].kernarg > n) return rti::fail(RT_ERR_HIP, "chain kernel argument size mismatch");
    s.frames.push_back(Pending{part, grid[0], grid[1], threads, which});
    return RT_OK;
}

void chain_abort(Chain* c) {
    // nothing of an open segment has been published yet: its packed frames are dropped
    if (!c || !c->open) return;
    c->open = false;
    c->sets[c->set].frames.clear();
}

rt_status chain_end(Chain* c, hipStream_t stream) {
    if (!c->open) return rti::fail(RT_ERR_INVALID_ARGUMENT, "chain_end");
    c->open = false;
    SignalSet& s = c->sets[c->set];
    if (s.frames.empty()) return RT_OK;
    c->set = (c->set + 1u) % kSets;
    if (c->ring) {
        // the arguments written through the BAR reach VRAM before any packet is published:
        // drain the write-combining buffers, flush the HDP, read back (MI355X: 2.4 µs)
        c->ring_head += (uint32_t)s.frames.size();
        _mm_sfence();
        *c->hdp_flush = 1u;
        (void)*reinterpret_cast<volatile uint32_t*>(c->hdp_flush);
        (void)*reinterpret_cast<volatile uint32_t*>(c->seg_args +
                                                     (s.frames.size() - 1) * kSlotBytes);
    }
    s.used = true;
    const uint32_t seq = ++c->seq;
    const uint32_t parts = c->seg_parts;
    // ordering after the caller's stream: nothing to wait for if it is idle now; else the
    // stream writes the go value and queue 0's go packet waits for it, the others for that
    const hipError_t q = hipStreamQuery(stream);
    if (q != hipSuccess && q != hipErrorNotReady) return rti::hip_fail(q, "hipStreamQuery");
    const bool go = q == hipErrorNotReady;
    hipError_t e = go ? hipStreamWriteValue32(stream, c->go, seq, 0) : hipSuccess;
    if (e != hipSuccess) return rti::hip_fail(e, "hipStreamWriteValue32 (chain go)");
    struct {
        const uint32_t* go;
        uint32_t want;
        uint32_t pad;
        uint32_t* abort;
        uint32_t* gave_up;
        uint64_t ticks;
    } ga{c->go, seq, 0u, c->abort, const_cast<uint32_t*>(c->gave_up), c->go_ticks};
    static_assert(sizeof(ga) == 40, "rt_chain_go_kernel's argument layout");
    std::memset(s.small, 0, 2 * kSlotBytes);
    std::memcpy(s.small, &ga, sizeof(ga));
    if (go) {
        hsa_signal_store_relaxed(s.go, 1);
        dispatch(c, 0, c->k[rtk::kChainGo], s.small, 1, 1, 64, HSA_FENCE_SCOPE_SYSTEM,
                 HSA_FENCE_SCOPE_NONE, s.go);
        for (uint32_t k = 1; k < parts; ++k) barrier_and(c, k, &s.go, 1);
    }
    // the frames, in order on their part's queue; each queue's first packet acquires at
    // system scope (reused argument slots, the lists, the input image), the rest none
    bool first[kMaxQueues];
    for (uint32_t k = 0; k < kMaxQueues; ++k) first[k] = true;
    for (size_t i = 0; i < s.frames.size(); ++i) {
        const Pending& f = s.frames[i];
        dispatch(c, f.part, c->k[f.which], c->seg_args + i * kSlotBytes, f.gx, f.gy, f.threads,
                 first[f.part] ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_NONE,
                 HSA_FENCE_SCOPE_NONE, hsa_signal_t{0});
        first[f.part] = false;
    }
    // queue 0 waits for the other queues' packets: a marker on each (a barrier-AND with no
    // dependency completes after every earlier packet of its queue: barrier bit)
    hsa_signal_t deps[kMaxQueues];
    uint32_t nd = 0;
    for (uint32_t k = 1; k < parts; ++k) {
        hsa_signal_store_relaxed(s.last[k], 1);
        hsa_queue_t* q = c->q[k];
        void* v = nullptr;
        const uint64_t idx = reserve(q, &v);
        hsa_barrier_and_packet_t* pk = static_cast<hsa_barrier_and_packet_t*>(v);
        pk->reserved0 = 0;
        pk->reserved1 = 0;
        for (auto& d : pk->dep_signal) d = hsa_signal_t{0};
        pk->reserved2 = 0;
        pk->completion_signal = s.last[k];
        publish(q, idx, v, header(HSA_PACKET_TYPE_BARRIER_AND, true, HSA_FENCE_SCOPE_NONE,
                                  HSA_FENCE_SCOPE_NONE));
        c->packets++;
        deps[nd++] = s.last[k];
    }
    if (nd) barrier_and(c, 0, deps, nd);
    struct {
        uint32_t* done;
        uint32_t value;
    } da{c->done, seq};
    unsigned char* dk = s.small + kSlotBytes;
    std::memcpy(dk, &da, sizeof(da));
    hsa_signal_store_relaxed(s.done, 1);
    dispatch(c, 0, c->k[rtk::kChainDone], dk, 1, 1, 64, HSA_FENCE_SCOPE_NONE,
             HSA_FENCE_SCOPE_SYSTEM, s.done);
    e = hipStreamWaitValue32(stream, c->done, seq, hipStreamWaitValueGte, 0xFFFFFFFFu);
    return e == hipSuccess ? RT_OK : rti::hip_fail(e, "hipStreamWaitValue32 (chain done)");
}

rt_status chain_errors(Chain* c, uint32_t* out) {
    for (SignalSet& s : c->sets)
        if (s.used && !wait_zero(s.done, wait_bound_ms(c))) {
            c->failed = true;
            c->why = "an AQL segment did not complete within the bound";
            return rti::fail(RT_ERR_HIP, c->why);
        }
    *out = (c->gave_up && *c->gave_up) ? 1u : 0u;
    return RT_OK;
}

const uint32_t* chain_abort_word(const Chain* c) { return c ? c->abort : nullptr; }

uint64_t chain_packets(const Chain* c) { return c ? c->packets : 0; }

}  // namespace rtc
