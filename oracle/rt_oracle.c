/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's per-pixel
 * ray tracer (assets/compute_shader.wgsl of Sur091/GPU-Ray-Tracing), used as the parity
 * checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
 * the product (librt_hip.so, the Python package) includes, links or calls this file.
 *
 * PARITY UNPINNED against the reference itself: the reference ships no tests, golden
 * images or fixtures, and its WGSL cannot be executed here (Rust/cargo,
 * wgpu, naga and Vulkan are absent).  The restatement is pinned instead by
 * (1) known-answer tests of the integer RNG computed independently in Python,
 * (2) analytic ray/sphere cases, (3) a float64 numpy restatement with libm
 * transcendentals (tests/test_oracle.py), and (4) committed golden fixtures.
 *
 * Canonical float semantics.  WGSL leaves FMA contraction and the
 * precision of sin/cos/pow implementation-defined, so this restatement fixes them:
 *   - f32 everywhere, IEEE round-to-nearest-even, subnormals kept, compiled with
 *     -ffp-contract=off; every fused multiply-add is an explicit fmaf();
 *   - dot(a,b) = fmaf(a.z,b.z, fmaf(a.y,b.y, a.x*b.x)); "p + q*r" = fmaf(q,r,p);
 *   - sqrt and division are the correctly rounded IEEE operations;
 *   - normalize(v) = v / sqrt(dot(v,v)), one IEEE division per component;
 *   - sin/cos: Cody-Waite reduction by pi/2 in three f32 parts + Cephes minimax
 *     polynomials (canon_sincos below);  pow(x, 5.0) = ((x*x)*(x*x))*x;
 *   - u32(f) = truncate toward zero, saturating, NaN -> 0 (v_cvt_u32_f32);
 *   - f32(u32) = round to nearest even.
 * The HIP kernels implement the same semantics independently, so CPU and GPU agree
 * bit for bit (the parity tests require it).
 */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

typedef struct {
    float x, y, z;
} v3;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline v3 vdivs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
/* p + s*q, contracted */
static inline v3 vfma_s(float s, v3 q, v3 p) {
    return V(fmaf(s, q.x, p.x), fmaf(s, q.y, p.y), fmaf(s, q.z, p.z));
}
static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 normalize3(v3 v) { return vdivs(v, sqrtf(dot3(v, v))); }

/* ---- integer RNG: wgsl:50-63 -------------------------------------------------------- */
EXPORT uint32_t oracle_hash(uint32_t s) {
    s = s ^ 2747636419u; /* wgsl:52 */
    s = s * 2654435769u; /* wgsl:53 */
    s = s ^ (s >> 16);   /* wgsl:54: '>>' binds tighter than '^' */
    s = s * 2654435769u;
    s = s ^ (s >> 16);
    s = s * 2654435769u;
    return s;
}
/* wgsl:61-63: f32(hash(v)) / 4294967295.0 — the literal is 2^32 once rounded to f32,
 * so the division is an exact scaling by 2^-32. */
EXPORT float oracle_random_float(uint32_t v) { return (float)oracle_hash(v) * 0x1p-32f; }

/* WGSL u32(f32): truncation toward zero, saturating to [0, 2^32-1], NaN -> 0. */
static inline uint32_t f2u(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

/* ---- canonical sin/cos -------------------------------------------------------------- */
EXPORT void oracle_sincos(float x, float* s_out, float* c_out) {
    const float q = rintf(x * 0x1.45f306p-1f); /* x * (2/pi), nearest integer */
    const int k = (q == q) ? (int)q : 0;
    float r = fmaf(q, -0x1.921fb6p+0f, x);     /* x - q*pi/2, three-part Cody-Waite */
    r = fmaf(q, 0x1.777a5cp-25f, r);
    r = fmaf(q, 0x1p-49f, r);
    const float r2 = r * r;
    const float ps = fmaf(fmaf(-0x1.9943f2p-13f, r2, 0x1.11073cp-7f), r2, -0x1.555546p-3f);
    const float sr = fmaf(r * r2, ps, r);
    const float pc = fmaf(fmaf(0x1.99eb9cp-16f, r2, -0x1.6c0c34p-10f), r2, 0x1.55554ap-5f);
    const float cr = fmaf(r2 * r2, pc, fmaf(-0.5f, r2, 1.0f));
    switch (k & 3) {
        case 0: *s_out = sr; *c_out = cr; break;
        case 1: *s_out = cr; *c_out = -sr; break;
        case 2: *s_out = -sr; *c_out = -cr; break;
        default: *s_out = -cr; *c_out = sr; break;
    }
}

/* pow(x, 5.0) (wgsl:140). */
static inline float pow5(float x) {
    const float x2 = x * x;
    const float x4 = x2 * x2;
    return x4 * x;
}

/* ---- camera blob (wgsl:7-40 == camera.rs:256-291), read by byte offset --------------- */
typedef struct {
    v3 center, vul, pdu, pdv, ddu, ddv;
    float defocus_angle, max_depth, spp, moved, random_seed;
} cam_t;

static cam_t load_cam(const float* c) {
    cam_t k;
    k.center = V(c[0], c[1], c[2]);          /* offset 0 */
    k.vul = V(c[4], c[5], c[6]);             /* 16 */
    k.pdu = V(c[8], c[9], c[10]);            /* 32 */
    k.defocus_angle = c[11];                 /* 44 */
    k.pdv = V(c[12], c[13], c[14]);          /* 48 */
    k.ddu = V(c[16], c[17], c[18]);          /* 64 */
    k.ddv = V(c[24], c[25], c[26]);          /* 96 */
    k.max_depth = c[27];                     /* 108 */
    k.spp = c[31];                           /* 124 */
    k.moved = c[35];                         /* 140 */
    k.random_seed = c[39];                   /* 156 */
    return k;
}

typedef struct {
    v3 o, d;
} ray_t;

typedef struct {
    float t;
    v3 p, n;
    int front;
    float mat[4];
} hit_t;

/* ---- wgsl:164-221 ------------------------------------------------------------------- */
static int sphere_hit(const float* s, ray_t r, float tmin, float tmax, hit_t* rec) {
    const v3 C = V(s[0], s[1], s[2]);
    const float R = s[3];
    const v3 oc = vsub(C, r.o);                       /* wgsl:183 */
    const float a = dot3(r.d, r.d);                   /* wgsl:184 */
    const float h = dot3(oc, r.d);                    /* wgsl:185 */
    const float c = dot3(oc, oc) - R * R;             /* wgsl:186 */
    const float disc = fmaf(h, h, -(a * c));          /* wgsl:187: h*h - a*c */
    if (disc < 0.0f) return 0;                        /* wgsl:189 */
    const float sq = sqrtf(disc);                     /* wgsl:193 */
    float root = (h - sq) / a;                        /* wgsl:195 */
    if (root <= tmin || tmax <= root) {               /* wgsl:196 */
        root = (h + sq) / a;
        if (root <= tmin || tmax <= root) return 0;
    }
    rec->t = root;
    rec->p = vfma_s(root, r.d, r.o);                  /* wgsl:205 */
    const v3 outward = vdivs(vsub(rec->p, C), R);     /* wgsl:206 */
    rec->front = dot3(r.d, outward) < 0.0f;           /* wgsl:159 */
    rec->n = rec->front ? outward : vneg(outward);    /* wgsl:160 */
    memcpy(rec->mat, s + 4, sizeof(rec->mat));
    return 1;
}

static int sphere_list_hit(const float* spheres, uint32_t count, ray_t r, hit_t* rec) {
    hit_t tmp;
    int any = 0;
    float closest = 0x1.05ed2ep+118f; /* 3.4e35 (wgsl:266) */
    for (uint32_t i = 0; i < count; ++i) {           /* wgsl:169 */
        if (sphere_hit(spheres + 8 * (size_t)i, r, 0x1.0624dep-10f /* 0.001 */, closest,
                       &tmp)) {
            any = 1;
            closest = tmp.t;
            *rec = tmp;
        }
    }
    return any;
}

/* wgsl:234-243 */
static v3 random_unit_vector(uint32_t seed) {
    const float z = fmaf(2.0f, oracle_random_float(seed), -1.0f);
    const float a = oracle_random_float(seed + 1u) * 0x1.921fb6p+2f; /* 6.283185307 */
    const float r = sqrtf(fmaf(-z, z, 1.0f));
    float sa, ca;
    oracle_sincos(a, &sa, &ca);
    return V(r * ca, r * sa, z);
}

/* WGSL reflect(e1, e2) = e1 - 2*dot(e2,e1)*e2 */
static v3 reflect3(v3 e1, v3 e2) {
    const float k = 2.0f * dot3(e2, e1);
    return vfma_s(-k, e2, e1);
}

/* WGSL refract(e1, e2, eta): k = 1 - eta^2 (1 - dot(e2,e1)^2); k < 0 -> 0, else
 * eta*e1 - (eta*dot(e2,e1) + sqrt(k))*e2 */
static v3 refract3(v3 e1, v3 e2, float eta) {
    const float d = dot3(e2, e1);
    const float k = fmaf(-(eta * eta), fmaf(-d, d, 1.0f), 1.0f);
    if (k < 0.0f) return V(0.0f, 0.0f, 0.0f);
    const float m = fmaf(eta, d, sqrtf(k));
    return V(fmaf(eta, e1.x, -(m * e2.x)), fmaf(eta, e1.y, -(m * e2.y)),
             fmaf(eta, e1.z, -(m * e2.z)));
}

/* wgsl:137-141 */
static float reflectance(float cos_theta, float ri) {
    float r0 = (1.0f - ri) / (1.0f + ri);
    r0 = r0 * r0;
    return fmaf(1.0f - r0, pow5(1.0f - cos_theta), r0);
}

/* wgsl:261-297; *segs counts sphere_list_hit calls (the algorithmic unit). */
static v3 ray_color(const cam_t* cam, const float* spheres, uint32_t count, ray_t r,
                    uint32_t seed, uint64_t* segs) {
    v3 cf = V(1.0f, 1.0f, 1.0f);
    const uint32_t depth = f2u(cam->max_depth);
    for (uint32_t i = 0; i < depth; ++i) {
        hit_t rec = {0};
        ++*segs;
        if (!sphere_list_hit(spheres, count, r, &rec)) break; /* wgsl:288-290 */
        const uint32_t sb = oracle_hash(seed + i * 1000u);   /* wgsl:268 */
        v3 att;
        ray_t sc;
        if (rec.mat[3] < -1.0f) {                            /* lambertian wgsl:84-93 */
            v3 dir = vadd(rec.n, random_unit_vector(sb));
            if (dot3(dir, dir) < 0x1.0c6f7ap-20f /* 1e-6 */) dir = rec.n;
            sc.o = rec.p;
            sc.d = dir;
            att = V(rec.mat[0], rec.mat[1], rec.mat[2]);
        } else if (rec.mat[3] <= 1.0f) {                     /* metal wgsl:95-100 */
            const v3 refl = vfma_s(rec.mat[3], random_unit_vector(sb),
                                   normalize3(reflect3(r.d, rec.n)));
            sc.o = rec.p;
            sc.d = normalize3(refl);
            att = V(rec.mat[0], rec.mat[1], rec.mat[2]);
            if (!(dot3(refl, rec.n) > 0.0f)) return V(0.0f, 0.0f, 0.0f); /* wgsl:277-279 */
        } else {                                             /* dielectric wgsl:102-135 */
            att = V(1.0f, 1.0f, 1.0f);
            const float ratio = rec.front ? 1.0f / rec.mat[0] : rec.mat[0];
            const v3 u = normalize3(r.d);
            const float cos_t = fminf(dot3(vneg(u), rec.n), 1.0f);
            const float sin_t = sqrtf(fmaf(-cos_t, cos_t, 1.0f));
            const int cannot = ratio * sin_t > 1.0f;
            const int refl = cannot || reflectance(cos_t, ratio) > oracle_random_float(sb);
            const v3 dir = refl ? reflect3(u, rec.n) : refract3(u, rec.n, ratio);
            sc.o = rec.p;
            sc.d = normalize3(dir);
        }
        cf = vmul(cf, att);                                  /* wgsl:285 */
        r = sc;
    }
    /* wgsl:293-296: only the y component of normalize(r.direction) is used. */
    const float uy = r.d.y / sqrtf(dot3(r.d, r.d));
    const float a = 0.5f * (uy + 1.0f);
    const float om = 1.0f - a;
    const v3 sky = V(fmaf(a, 0.5f, om), fmaf(a, 0x1.666666p-1f /* 0.7 */, om), fmaf(a, 1.0f, om));
    return vmul(cf, sky);
}

/* wgsl:305-325 (+ sample_square 299-303, defocus_disk_sample 327-331) */
static ray_t get_ray(const cam_t* cam, uint32_t x, uint32_t y, uint32_t sample_index) {
    const uint32_t B = f2u(cam->random_seed * 4294967296.0f);
    const uint32_t seed = oracle_hash(oracle_hash(x * 73u) ^ oracle_hash(y * 51u) ^
                                      (sample_index * 25u + B));
    const float offx = oracle_random_float(seed) - 0.5f;
    const float offy = oracle_random_float(seed * seed) - 0.5f;
    const float sx = ((float)x + 0.5f) + offx;
    const float sy = ((float)y + 0.5f) + offy;
    const v3 pc = vfma_s(sy, cam->pdv, vfma_s(sx, cam->pdu, cam->vul));
    ray_t r;
    if (cam->defocus_angle > 0.0f) {
        const float ang = 0x1.921fb4p+2f /* 2.0*3.1415926 */ * oracle_random_float(seed + 1u);
        float sa, ca;
        oracle_sincos(ang, &sa, &ca);
        const float len = sqrtf(fmaf(sa, sa, ca * ca));
        const float px = ca / len, py = sa / len;
        r.o = vfma_s(py, cam->ddv, vfma_s(px, cam->ddu, cam->center));
    } else {
        r.o = cam->center;
    }
    r.d = vsub(pc, r.o);
    return r;
}

/* One invocation of `update` (wgsl:333-364) for pixel (x, y): in/out are 4 floats. */
static void update_pixel(const cam_t* cam, const float* spheres, uint32_t count, uint32_t x,
                         uint32_t y, const float* in, float* out, uint64_t* segs) {
    v3 c = V(in[0], in[1], in[2]);
    uint32_t n = f2u(in[3]);
    const uint32_t spp = f2u(cam->spp);
    if (cam->moved > 0.5f) {
        c = V(0.0f, 0.0f, 0.0f);
        n = 0u;
    }
    if (n < spp) {
        const uint32_t seed = 1u + n + f2u(cam->random_seed * 4294967296.0f);
        const ray_t r = get_ray(cam, x, y, seed);
        const v3 col = ray_color(cam, spheres, count, r, seed + 1u, segs);
        const float k = (float)(n + 1u);
        c = V(c.x + (col.x - c.x) / k, c.y + (col.y - c.y) / k, c.z + (col.z - c.z) / k);
        n += 1u;
    }
    out[0] = c.x;
    out[1] = c.y;
    out[2] = c.z;
    out[3] = (float)n;
}

/* ---- exported entry points ---------------------------------------------------------- */

/* One `update` dispatch over rows [y0, y1) of a width x height image.  camera = the
 * 176-byte blob as 44 floats, spheres = count x 8 floats.  Returns segments traced. */
EXPORT uint64_t oracle_update_rows(const float* in, float* out, uint32_t width,
                                   uint32_t height, uint32_t y0, uint32_t y1,
                                   const float* camera, const float* spheres,
                                   uint32_t count) {
    (void)height;
    const cam_t cam = load_cam(camera);
    uint64_t segs = 0;
    for (uint32_t y = y0; y < y1; ++y)
        for (uint32_t x = 0; x < width; ++x) {
            const size_t i = ((size_t)y * width + x) * 4;
            update_pixel(&cam, spheres, count, x, y, in + i, out + i, &segs);
        }
    return segs;
}

EXPORT uint64_t oracle_update(const float* in, float* out, uint32_t width, uint32_t height,
                              const float* camera, const float* spheres, uint32_t count) {
    return oracle_update_rows(in, out, width, height, 0, height, camera, spheres, count);
}

/* The same update on `threads` POSIX threads, each claiming `band`-row bands from a shared
 * counter (the CPU baseline on all host cores, SURVEY §8d5: no Python between the bands). */
typedef struct {
    const float *in, *camera, *spheres;
    float* out;
    uint32_t width, height, count, band;
    atomic_uint next;
    atomic_ullong segs;
} pool_t;

static void* pool_run(void* arg) {
    pool_t* p = (pool_t*)arg;
    uint64_t segs = 0;
    for (;;) {
        const uint32_t y0 = atomic_fetch_add(&p->next, p->band);
        if (y0 >= p->height) break;
        const uint32_t y1 = y0 + p->band < p->height ? y0 + p->band : p->height;
        segs += oracle_update_rows(p->in, p->out, p->width, p->height, y0, y1, p->camera,
                                   p->spheres, p->count);
    }
    atomic_fetch_add(&p->segs, segs);
    return NULL;
}

EXPORT uint64_t oracle_update_threads(const float* in, float* out, uint32_t width,
                                      uint32_t height, const float* camera,
                                      const float* spheres, uint32_t count, uint32_t threads,
                                      uint32_t band) {
    pool_t p;
    p.in = in;
    p.out = out;
    p.camera = camera;
    p.spheres = spheres;
    p.width = width;
    p.height = height;
    p.count = count;
    p.band = band ? band : 1u;
    atomic_init(&p.next, 0u);
    atomic_init(&p.segs, 0ull);
    if (threads < 1u) threads = 1u;
    if (threads > 1024u) threads = 1024u;
    pthread_t tid[1024];
    uint32_t started = 0;
    for (uint32_t t = 1; t < threads; ++t)
        if (pthread_create(&tid[started], NULL, pool_run, &p) == 0) ++started;
    pool_run(&p);                       /* the caller's thread works too */
    for (uint32_t t = 0; t < started; ++t) pthread_join(tid[t], NULL);
    return (uint64_t)atomic_load(&p.segs);
}

/* `frames` chained updates on a list of pixels (px[i], py[i]); state[i] holds the
 * RGBA accumulator of pixel i and is updated in place.  Frame f uses random_seeds[f]
 * and camera_has_moved = (f == 0 ? camera's flag : 0) — the contract of rt_render. */
EXPORT uint64_t oracle_render_pixels(float* state, const uint32_t* px, const uint32_t* py,
                                     uint64_t npix, const float* camera,
                                     const float* spheres, uint32_t count, uint32_t frames,
                                     const float* random_seeds) {
    cam_t cam = load_cam(camera);
    const float moved0 = cam.moved;
    uint64_t segs = 0;
    for (uint32_t f = 0; f < frames; ++f) {
        cam.random_seed = random_seeds[f];
        cam.moved = (f == 0) ? moved0 : 0.0f;
        for (uint64_t i = 0; i < npix; ++i) {
            float o[4];
            update_pixel(&cam, spheres, count, px[i], py[i], state + 4 * i, o, &segs);
            memcpy(state + 4 * i, o, sizeof(o));
        }
    }
    return segs;
}

/* `init` (wgsl:65-70). */
EXPORT void oracle_init(float* out, uint32_t width, uint32_t height) {
    memset(out, 0, (size_t)width * height * 4 * sizeof(float));
}

/* Test hook: sphere_hit (wgsl:182-221) for one 8-float sphere and ray = (o, d).
 * out = t, p.xyz, normal.xyz, front_face. */
EXPORT int oracle_sphere_hit(const float* sphere, const float* ray, float tmin, float tmax,
                             float* out) {
    ray_t r;
    r.o = V(ray[0], ray[1], ray[2]);
    r.d = V(ray[3], ray[4], ray[5]);
    hit_t rec = {0};
    if (!sphere_hit(sphere, r, tmin, tmax, &rec)) return 0;
    out[0] = rec.t;
    out[1] = rec.p.x; out[2] = rec.p.y; out[3] = rec.p.z;
    out[4] = rec.n.x; out[5] = rec.n.y; out[6] = rec.n.z;
    out[7] = rec.front ? 1.0f : 0.0f;
    return 1;
}
