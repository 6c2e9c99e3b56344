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
//
// The scan walks the list in chunks of 4 spheres.  The 16-byte scan records of the next
// chunk are fetched with scalar loads while the current chunk is computed (the index is
// wave-uniform, so the records live in SGPRs and feed the VALU directly).  Per sphere the
// common (miss) path is 12 VALU ops for the discriminant; the chunk's four "!(D < 0)"
// tests collapse into one integer max + compare on the float bit patterns (exact: D is
// never -0, see below), so the root-finding path is entered once per chunk at most.

// Discriminant of wgsl:183-187 for one sphere record g = (center, r*r).
__device__ __forceinline__ float discriminant(const float4 g, v3 o, v3 d, float a, float& h) {
    const float ocx = g.x - o.x;                                        // wgsl:183
    const float ocy = g.y - o.y;
    const float ocz = g.z - o.z;
    h = fmaf(ocz, d.z, fmaf(ocy, d.y, ocx * d.x));                      // wgsl:185
    const float c = fmaf(ocz, ocz, fmaf(ocy, ocy, ocx * ocx)) - g.w;    // wgsl:186
    return fmaf(h, h, -(a * c));                                        // wgsl:187
}

// Root selection of wgsl:189-201 for sphere i, given its discriminant.
__device__ __forceinline__ void consider(float disc, float h, float a, uint32_t i, float& tmax,
                                         int& idx) {
    if (!(disc < 0.0f)) {                                               // wgsl:189
        const float q = sqrtf(disc);
        float root = (h - q) / a;
        if (root <= 0x1.0624dep-10f || tmax <= root) {                  // wgsl:196
            root = (h + q) / a;
            if (root <= 0x1.0624dep-10f || tmax <= root) return;        // wgsl:198
        }
        tmax = root;
        idx = (int)i;
    }
}

// "!(D < 0)" for any of K discriminants, on the bit patterns: a float is < 0 exactly
// when its int32 view is <= 0xFF800000 (-inf) and it is not -0.  D = fma(h, h, -(a*c))
// with h*h >= +0 and a >= +0 cannot round to -0, so the test is one max-tree and one
// compare per chunk (max_bits below).

// Scan variant selection (compile-time, for A/B builds only; the product uses the
// default).  0: one sphere per iteration; 1: chunks of 4 + prefetch + one test per chunk;
// 2: as 1, but the records are staged in LDS once per workgroup (ds_read broadcast).
#ifndef RT_SCAN_VARIANT
#define RT_SCAN_VARIANT 1
#endif

#if RT_SCAN_VARIANT == 0
__device__ __forceinline__ Hit scan_spheres(const float4* __restrict__ geom, uint32_t count,
                                            v3 o, v3 d) {
    const float a = dot(d, d);
    float tmax = 0x1.05ed2ep+118f;
    int idx = -1;
    for (uint32_t i = 0; i < count; ++i) {
        float h;
        const float disc = discriminant(geom[i], o, d, a, h);
        consider(disc, h, a, i, tmax, idx);
    }
    return Hit{idx, tmax};
}
#elif RT_SCAN_VARIANT == 3
// Scan records in SoA blocks of 4 spheres (64 B = one s_load_dwordx16):
//   {cx0..cx3, cy0..cy3, cz0..cz3, rr0..rr3}.
// On gfx950 a VALU op with an SGPR operand issues at half rate (~4.2 vs ~2.3 cycles per
// wave64 instruction, tools/valu_microbench.hip), while a packed op reading an SGPR pair
// costs the same 4.2 cycles for two elements.  So the four SGPR-consuming ops per sphere
// (oc = C - O and c = dot(oc,oc) - r*r) are issued as v_pk_add_f32 on sphere pairs, and
// everything else runs as full-rate single-precision VGPR ops.
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void disc_pair(f2v cx, f2v cy, f2v cz, f2v rr, v3 o, v3 d, float a,
                                          float& h0, float& h1, float& d0, float& d1) {
    const f2v ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const f2v ocx = cx - ox, ocy = cy - oy, ocz = cz - oz;                   // wgsl:183
    h0 = fmaf(ocz.x, d.z, fmaf(ocy.x, d.y, ocx.x * d.x));                    // wgsl:185
    h1 = fmaf(ocz.y, d.z, fmaf(ocy.y, d.y, ocx.y * d.x));
    f2v cc;
    cc.x = fmaf(ocz.x, ocz.x, fmaf(ocy.x, ocy.x, ocx.x * ocx.x));
    cc.y = fmaf(ocz.y, ocz.y, fmaf(ocy.y, ocy.y, ocx.y * ocx.y));
    const f2v c = cc - rr;                                                   // wgsl:186
    d0 = fmaf(h0, h0, -(a * c.x));                                           // wgsl:187
    d1 = fmaf(h1, h1, -(a * c.y));
}

__device__ __forceinline__ Hit scan_spheres(const float4* __restrict__ geom4, uint32_t count,
                                            v3 o, v3 d) {
    const float a = dot(d, d);                 // wgsl:184 (ray-invariant)
    float tmax = 0x1.05ed2ep+118f;             // 3.4e35 (wgsl:266)
    int idx = -1;
    const uint32_t nchunks = (count + 3u) >> 2;
    // one zero block of padding after the last chunk keeps the prefetch in bounds
    float4 c0 = geom4[0], c1 = geom4[1], c2 = geom4[2], c3 = geom4[3];
    for (uint32_t k = 0; k < nchunks; ++k) {
        const float4* nb = geom4 + 4u * (k + 1u);
        const float4 n0 = nb[0], n1 = nb[1], n2 = nb[2], n3 = nb[3];
        float h[4], dd[4];
        disc_pair(f2v{c0.x, c0.y}, f2v{c1.x, c1.y}, f2v{c2.x, c2.y}, f2v{c3.x, c3.y}, o, d, a,
                  h[0], h[1], dd[0], dd[1]);
        disc_pair(f2v{c0.z, c0.w}, f2v{c1.z, c1.w}, f2v{c2.z, c2.w}, f2v{c3.z, c3.w}, o, d, a,
                  h[2], h[3], dd[2], dd[3]);
        const int m = max(max(__float_as_int(dd[0]), __float_as_int(dd[1])),
                          max(__float_as_int(dd[2]), __float_as_int(dd[3])));
        if (__builtin_expect(m > (int)0xFF800000, 0)) {
            const uint32_t i0 = 4u * k;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (i0 + j < count) consider(dd[j], h[j], a, i0 + j, tmax, idx);
        }
        c0 = n0;
        c1 = n1;
        c2 = n2;
        c3 = n3;
    }
    return Hit{idx, tmax};
}
#else
#ifndef RT_SCAN_CHUNK
#define RT_SCAN_CHUNK 4
#endif
#ifndef RT_SCAN_PIN_LOADS
#define RT_SCAN_PIN_LOADS 0
#endif
#ifndef RT_SCAN_ABLATE_RARE
#define RT_SCAN_ABLATE_RARE 0
#endif
// max over the int32 views of K discriminants
template <int K>
__device__ __forceinline__ int max_bits(const float (&dd)[K]) {
    int m = __float_as_int(dd[0]);
#pragma unroll
    for (int k = 1; k < K; ++k) m = max(m, __float_as_int(dd[k]));
    return m;
}

__device__ __forceinline__ Hit scan_spheres(const float4* __restrict__ geom, uint32_t count,
                                            v3 o, v3 d) {
    constexpr int K = RT_SCAN_CHUNK;
    const float a = dot(d, d);                 // wgsl:184 (ray-invariant)
    float tmax = 0x1.05ed2ep+118f;             // 3.4e35 (wgsl:266)
    int idx = -1;
    const uint32_t nk = count - count % K;
    // geom is padded with zero records, so the prefetch of the chunk after the last one
    // stays inside the allocation.
    float4 cur[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cur[k] = geom[k];
    uint32_t i = 0;
#if RT_SCAN_ABLATE_RARE
    float sink = 0.0f;
#endif
    for (; i < nk; i += K) {
        float4 nxt[K];
#pragma unroll
        for (int k = 0; k < K; ++k) nxt[k] = geom[i + K + k];
#if RT_SCAN_PIN_LOADS
        __builtin_amdgcn_sched_barrier(0);
#endif
        float hh[K], dd[K];
#pragma unroll
        for (int k = 0; k < K; ++k) dd[k] = discriminant(cur[k], o, d, a, hh[k]);
#if RT_SCAN_ABLATE_RARE
#pragma unroll
        for (int k = 0; k < K; ++k) sink += dd[k] + hh[k];
#else
        if (__builtin_expect(max_bits<K>(dd) > (int)0xFF800000, 0)) {
#pragma unroll
            for (int k = 0; k < K; ++k) consider(dd[k], hh[k], a, i + k, tmax, idx);
        }
#endif
#pragma unroll
        for (int k = 0; k < K; ++k) cur[k] = nxt[k];
    }
#if RT_SCAN_ABLATE_RARE
    if (sink == 12345.0f) idx = 0;
#endif
    for (; i < count; ++i) {
        float h;
        const float disc = discriminant(geom[i], o, d, a, h);
        consider(disc, h, a, i, tmax, idx);
    }
    return Hit{idx, tmax};
}
#endif

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
#ifndef RT_TRACE_MIN_WAVES
#define RT_TRACE_MIN_WAVES 8
#endif
__global__ __launch_bounds__(256, RT_TRACE_MIN_WAVES) void rt_trace_kernel(const TraceParams p) {
#if RT_SCAN_VARIANT == 2
    extern __shared__ float4 lds_geom[];
    for (uint32_t j = threadIdx.x; j < p.count + 8u; j += blockDim.x) lds_geom[j] = p.geom[j];
    __syncthreads();
    const float4* scan_geom = lds_geom;
#else
    const float4* scan_geom = p.geom;
#endif
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
            const v3 col = ray_color(p, scan_geom, p.sph, depth, o, d, seed + 1u);
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
#if RT_SCAN_VARIANT == 2
    const size_t lds = ((size_t)p.count + 8u) * sizeof(float4);
    if (lds > 65536) return hipErrorInvalidValue;
#else
    const size_t lds = 0;
#endif
    hipLaunchKernelGGL(rt_trace_kernel, dim3(blocks), dim3(256), lds, stream, p);
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

int scan_layout() { return RT_SCAN_VARIANT == 3 ? 1 : 0; }

}  // namespace rtk
