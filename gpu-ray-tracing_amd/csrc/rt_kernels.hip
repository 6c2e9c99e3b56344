// rt_kernels.hip — gfx950 kernels for the per-pixel ray tracer.
//
// Replaces the reference's WGSL compute kernels (assets/compute_shader.wgsl):
//   rt_trace_kernel   == `update` (wgsl:333-364), optionally fused over several frames
//   rt_init_kernel    == `init`   (wgsl:65-70)
//   rt_deinterleave   root-side scatter of gathered stripe tiles (multi-GPU)
//
// Mapping onto CDNA4: one wave64 = one 8x8 pixel tile (the reference's 8x8 workgroup,
// wgsl:333), four waves per 256-thread workgroup.  The sphere scan (wgsl:164-221) walks
// a wave-uniform index, so the 16-byte scan records are fetched with scalar loads into
// SGPRs and consumed directly as VALU operands — no VGPRs and no LDS traffic per test.
// The 32-byte material record is fetched only for the winning hit.  Each lane keeps its
// pixel's accumulator in registers across fused frames and writes it back with one
// coalesced 16-byte store (one HBM read + one write per pixel per launch).
#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_kernels.h"

namespace rtk {

using namespace rtd;

struct Hit {
    int idx;     // winning sphere, -1 = miss
    float t;     // its root
};

// sphere_list_hit (wgsl:164-180) + sphere_hit (wgsl:182-201) without the hit record:
// only the closest root and its index are tracked; the record (p, normal, face,
// material) is rebuilt once for the winner, bit-identical to the WGSL's last assignment.
__device__ __forceinline__ Hit scan_spheres(const float4* __restrict__ geom, uint32_t count,
                                            v3 o, v3 d) {
    const float a = dot(d, d);                 // wgsl:184 (ray-invariant)
    float tmax = 0x1.05ed2ep+118f;             // 3.4e35 (wgsl:266)
    int idx = -1;
#pragma unroll 4
    for (uint32_t i = 0; i < count; ++i) {
        const float4 g = geom[i];              // wave-uniform -> s_load into SGPRs
        const float ocx = g.x - o.x;           // wgsl:183
        const float ocy = g.y - o.y;
        const float ocz = g.z - o.z;
        const float h = fmaf(ocz, d.z, fmaf(ocy, d.y, ocx * d.x));          // wgsl:185
        const float c = fmaf(ocz, ocz, fmaf(ocy, ocy, ocx * ocx)) - g.w;    // wgsl:186
        const float disc = fmaf(h, h, -(a * c));                            // wgsl:187
        if (!(disc < 0.0f)) {                                               // wgsl:189
            const float q = sqrtf(disc);
            float root = (h - q) / a;
            if (root <= 0x1.0624dep-10f || tmax <= root) {                  // wgsl:196
                root = (h + q) / a;
                if (root <= 0x1.0624dep-10f || tmax <= root) continue;      // wgsl:198
            }
            tmax = root;
            idx = (int)i;
        }
    }
    return Hit{idx, tmax};
}

struct Cam {
    v3 center, vul, pdu, pdv, ddu, ddv;
    float defocus_angle;
};

// get_ray (wgsl:305-325) with the pixel-invariant hash(hash(x*73) ^ hash(y*51)) part
// precomputed per pixel: seed = hash(hxy ^ (sample_index*25 + B)).
__device__ __forceinline__ void get_ray(const Cam& cam, uint32_t x, uint32_t y, uint32_t hxy,
                                        uint32_t sample_index, uint32_t B, v3& o, v3& d) {
    const uint32_t seed = hash(hxy ^ (sample_index * 25u + B));
    const float offx = rf(seed) - 0.5f;                 // sample_square wgsl:299-303
    const float offy = rf(seed * seed) - 0.5f;
    const float sx = ((float)x + 0.5f) + offx;
    const float sy = ((float)y + 0.5f) + offy;
    const v3 pc = fmas(sy, cam.pdv, fmas(sx, cam.pdu, cam.vul));
    if (cam.defocus_angle > 0.0f) {                     // defocus_disk_sample wgsl:327-331
        const float ang = 0x1.921fb4p+2f * rf(seed + 1u);  // 2.0*3.1415926 as f32
        float sa, ca;
        sincos_c(ang, sa, ca);
        const float len = sqrtf(fmaf(sa, sa, ca * ca));
        o = fmas(sa / len, cam.ddv, fmas(ca / len, cam.ddu, cam.center));
    } else {
        o = cam.center;
    }
    d = sub(pc, o);
}

// ray_color (wgsl:261-297).
__device__ __forceinline__ v3 ray_color(const TraceParams& p, const float4* __restrict__ geom,
                                        const float4* __restrict__ sph, uint32_t depth, v3 o,
                                        v3 d, uint32_t seed) {
    v3 cf = mk(1.0f, 1.0f, 1.0f);
    for (uint32_t i = 0; i < depth; ++i) {
        const Hit hit = scan_spheres(geom, p.count, o, d);
        if (hit.idx < 0) break;                                   // wgsl:288-290
        // Hit record of the winner (wgsl:205-218).
        const float4 pr = sph[2 * hit.idx];       // position, radius
        const float4 mat = sph[2 * hit.idx + 1];  // material color
        const v3 C = mk(pr.x, pr.y, pr.z);
        const v3 hp = fmas(hit.t, d, o);
        const v3 outward = divs(sub(hp, C), pr.w);
        const bool front = dot(d, outward) < 0.0f;
        const v3 n = front ? outward : neg(outward);
        const uint32_t sb = hash(seed + i * 1000u);               // wgsl:268
        v3 att, nd;
        if (mat.w < -1.0f) {                                      // lambertian wgsl:84-93
            v3 dir = add(n, random_unit_vector(sb));
            if (dot(dir, dir) < 0x1.0c6f7ap-20f) dir = n;
            nd = dir;
            att = mk(mat.x, mat.y, mat.z);
        } else if (mat.w <= 1.0f) {                               // metal wgsl:95-100
            const v3 refl = fmas(mat.w, random_unit_vector(sb), normalize(reflect(d, n)));
            if (!(dot(refl, n) > 0.0f)) return mk(0.0f, 0.0f, 0.0f);
            nd = normalize(refl);
            att = mk(mat.x, mat.y, mat.z);
        } else {                                                  // dielectric wgsl:102-135
            att = mk(1.0f, 1.0f, 1.0f);
            const float ratio = front ? 1.0f / mat.x : mat.x;
            const v3 u = normalize(d);
            const float cos_t = fminf(dot(neg(u), n), 1.0f);
            const float sin_t = sqrtf(fmaf(-cos_t, cos_t, 1.0f));
            const bool cannot = ratio * sin_t > 1.0f;
            const bool refl = cannot || reflectance(cos_t, ratio) > rf(sb);
            const v3 dir = refl ? reflect(u, n) : refract(u, n, ratio);
            nd = normalize(dir);
        }
        cf = mul(cf, att);
        o = hp;
        d = nd;
    }
    // Sky (wgsl:293-296): only normalize(d).y is used.
    const float uy = d.y / sqrtf(dot(d, d));
    const float a = 0.5f * (uy + 1.0f);
    const float om = 1.0f - a;
    return mul(cf, mk(fmaf(a, 0.5f, om), fmaf(a, 0x1.666666p-1f, om), fmaf(a, 1.0f, om)));
}

// One wave = one 8x8 tile of the (local) image; lanes are row-major inside the tile.
__global__ __launch_bounds__(256) void rt_trace_kernel(const TraceParams p) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t tile = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t tiles_x = (p.width + 7u) >> 3;
    const uint32_t lband = tile / tiles_x;
    if (lband >= p.local_bands) return;                // whole wave exits together
    const uint32_t x = (tile - lband * tiles_x) * 8u + (lane & 7u);
    const uint32_t gband = p.band_first + lband * p.band_step;
    const uint32_t y = gband * RT_STRIPE_ROWS + (lane >> 3);
    const uint32_t ly = lband * RT_STRIPE_ROWS + (lane >> 3);
    const bool valid = (x < p.width) && (y < p.height);
    const size_t idx = (size_t)ly * p.width + x;

    Cam cam;
    cam.center = mk(p.center[0], p.center[1], p.center[2]);
    cam.vul = mk(p.vul[0], p.vul[1], p.vul[2]);
    cam.pdu = mk(p.pdu[0], p.pdu[1], p.pdu[2]);
    cam.pdv = mk(p.pdv[0], p.pdv[1], p.pdv[2]);
    cam.ddu = mk(p.ddu[0], p.ddu[1], p.ddu[2]);
    cam.ddv = mk(p.ddv[0], p.ddv[1], p.ddv[2]);
    cam.defocus_angle = p.defocus_angle;

    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (valid) acc = p.in[idx];                                   // wgsl:339
    v3 c = mk(acc.x, acc.y, acc.z);
    uint32_t n = f2u(acc.w);
    const uint32_t spp = f2u(p.spp);                              // wgsl:343
    const uint32_t depth = f2u(p.max_depth);
    const uint32_t hxy = hash(x * 73u) ^ hash(y * 51u);           // wgsl:309-310

    for (uint32_t f = 0; f < p.frames; ++f) {
        const uint32_t B = f2u(p.seeds[f] * 4294967296.0f);      // wgsl:311,353
        if (f == 0 && p.reset_first) {                            // wgsl:345-350
            c = mk(0.0f, 0.0f, 0.0f);
            n = 0u;
        }
        if (n < spp) {                                            // wgsl:352
            const uint32_t seed = 1u + n + B;
            v3 o, d;
            get_ray(cam, x, y, hxy, seed, B, o, d);
            const v3 col = ray_color(p, p.geom, p.sph, depth, o, d, seed + 1u);
            const float k = (float)(n + 1u);                      // wgsl:356
            c = mk(c.x + (col.x - c.x) / k, c.y + (col.y - c.y) / k, c.z + (col.z - c.z) / k);
            n += 1u;
        }
        // The chained form stores f32(n) and reloads u32(.) each frame (wgsl:341,362).
        n = f2u((float)n);
    }
    if (valid) p.out[idx] = make_float4(c.x, c.y, c.z, (float)n); // wgsl:362-363
}

__global__ __launch_bounds__(256) void rt_init_kernel(float4* __restrict__ out, uint64_t n) {
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = z;
}

// gathered = nranks x max_local_rows x width texels; band b of the full image is local
// band b / nranks of rank b % nranks.
__global__ __launch_bounds__(256) void rt_deinterleave_kernel(const float4* __restrict__ g,
                                                              float4* __restrict__ out,
                                                              uint32_t width, uint32_t height,
                                                              uint32_t nranks,
                                                              uint32_t max_local_rows) {
    const uint64_t total = (uint64_t)width * height;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t y = (uint32_t)(i / width);
        const uint32_t x = (uint32_t)(i - (uint64_t)y * width);
        const uint32_t band = y / RT_STRIPE_ROWS;
        const uint32_t rank = band % nranks;
        const uint32_t lrow = (band / nranks) * RT_STRIPE_ROWS + (y % RT_STRIPE_ROWS);
        out[i] = g[((uint64_t)rank * max_local_rows + lrow) * width + x];
    }
}

hipError_t launch_trace(const TraceParams& p, hipStream_t stream) {
    const uint64_t tiles = (uint64_t)((p.width + 7u) >> 3) * p.local_bands;
    const uint32_t blocks = (uint32_t)((tiles + 3u) / 4u);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_trace_kernel, dim3(blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_init(float4* out, uint64_t texels, hipStream_t stream) {
    if (texels == 0) return hipSuccess;
    uint64_t blocks = (texels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(rt_init_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, out,
                       texels);
    return hipGetLastError();
}

hipError_t launch_deinterleave(const float4* gathered, float4* out, uint32_t width,
                               uint32_t height, uint32_t nranks, uint32_t max_local_rows,
                               hipStream_t stream) {
    const uint64_t texels = (uint64_t)width * height;
    if (texels == 0) return hipSuccess;
    uint64_t blocks = (texels + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(rt_deinterleave_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream,
                       gathered, out, width, height, nranks, max_local_rows);
    return hipGetLastError();
}

const char* trace_kernel_name() { return "rt_trace_kernel"; }

}  // namespace rtk
