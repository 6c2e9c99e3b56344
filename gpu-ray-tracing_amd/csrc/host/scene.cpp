// scene.cpp — host mirror of src/scene/sphere.rs: create_default_spheres (45-153),
// made reproducible.  The reference draws from rand::random (unseeded, sphere.rs:61-91);
// here the variates come from splitmix64(seed) mapped like rand 0.9's f32
// ((u32 >> 8) * 2^-24, so every value is k * 2^-24 with k < 2^24).
// Built with -ffp-contract=off: each expression is the Rust f32 expression, unfused.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "rt_abi.h"

namespace {

struct SplitMix64 {
    uint64_t state;
    uint64_t next() {
        uint64_t z = (state += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    // rand 0.9 StandardUniform for f32: (next_u32 >> 8) as f32 * 2^-24
    float f32() { return (float)((uint32_t)(next() >> 32) >> 8) * 0x1p-24f; }
};

rt_sphere make(float x, float y, float z, float r, float c0, float c1, float c2, float c3) {
    rt_sphere s;
    s.position[0] = x;
    s.position[1] = y;
    s.position[2] = z;
    s.radius = r;
    s.color[0] = c0;
    s.color[1] = c1;
    s.color[2] = c2;
    s.color[3] = c3;
    return s;
}

// sphere.rs:114-136, in push order: glass, diffuse, metal.
void push_large(std::vector<rt_sphere>& v) {
    v.push_back(make(0.0f, 1.0f, 0.0f, 1.0f, 1.5f, 0.0f, 0.0f, 2.0f));
    v.push_back(make(-4.0f, 1.0f, 0.0f, 1.0f, 0.4f, 0.2f, 0.1f, -2.0f));
    v.push_back(make(4.0f, 1.0f, 0.0f, 1.0f, 0.7f, 0.6f, 0.5f, 0.0f));
}

// sphere.rs:59-111 over a in [-e, e), b in [-e, e), stopping once `limit` grid spheres
// have been placed.
void push_grid(std::vector<rt_sphere>& v, SplitMix64& rng, int e, size_t limit) {
    size_t placed = 0;
    for (int a = -e; a < e; ++a) {
        for (int b = -e; b < e; ++b) {
            if (placed >= limit) return;
            const float choose_mat = rng.f32();                       // sphere.rs:61
            const float cx = (float)a + 0.9f * rng.f32();              // sphere.rs:63
            const float cz = (float)b + 0.9f * rng.f32();              // sphere.rs:65
            const float dx = cx - 4.0f, dy = 0.2f - 0.2f, dz = cz - 0.0f;
            const float len = std::sqrt((dx * dx + dy * dy) + dz * dz);
            if (!(len > 0.9f)) continue;                               // sphere.rs:69
            if (choose_mat < 0.8f) {                                   // diffuse 70-83
                const float r1 = rng.f32(), r2 = rng.f32();
                const float ax = r1 * r2;
                const float r3 = rng.f32(), r4 = rng.f32();
                const float ay = r3 * r4;
                const float r5 = rng.f32(), r6 = rng.f32();
                const float az = r5 * r6;
                v.push_back(make(cx, 0.2f, cz, 0.2f, ax, ay, az, -2.0f));
            } else if (choose_mat < 0.95f) {                           // metal 84-98
                const float ax = 0.5f * (1.0f + rng.f32());
                const float ay = 0.5f * (1.0f + rng.f32());
                const float az = 0.5f * (1.0f + rng.f32());
                const float fuzz = 0.5f * rng.f32();
                v.push_back(make(cx, 0.2f, cz, 0.2f, ax, ay, az, fuzz));
            } else {                                                   // glass 99-107
                v.push_back(make(cx, 0.2f, cz, 0.2f, 1.5f, 0.0f, 0.0f, 2.0f));
            }
            ++placed;
        }
    }
}

}  // namespace

extern "C" {

rt_status rt_scene_generate(uint32_t kind, uint32_t n_spheres, uint64_t seed, rt_sphere* out,
                            uint32_t capacity, uint32_t* out_count) {
    if (!out_count) return RT_ERR_INVALID_ARGUMENT;
    std::vector<rt_sphere> v;
    SplitMix64 rng{seed};
    if (kind == 0) {
        push_large(v);
    } else if (kind == 1 || kind == 2) {
        v.push_back(make(0.0f, -1000.0f, 0.0f, 1000.0f, 0.5f, 0.5f, 0.5f, -2.0f));  // 49-55
        if (kind == 1) {
            push_grid(v, rng, 7, (size_t)-1);  // a, b in -7..7 (sphere.rs:59-60)
        } else {
            if (n_spheres < 4) return RT_ERR_INVALID_SIZE;
            const size_t want = n_spheres - 4u;
            int e = 12;  // a, b in -12..12
            while ((size_t)(4 * e * e) * 95u / 100u < want) ++e;
            push_grid(v, rng, e, want);
            if (v.size() != want + 1) return RT_ERR_INVALID_SIZE;
        }
        push_large(v);
    } else {
        return RT_ERR_INVALID_ARGUMENT;
    }
    *out_count = (uint32_t)v.size();
    if (out) std::memcpy(out, v.data(), std::min<size_t>(capacity, v.size()) * sizeof(rt_sphere));
    return RT_OK;
}

void rt_frame_seeds(uint64_t seed, uint32_t frames, float* out_seeds) {
    if (!out_seeds) return;
    SplitMix64 rng{seed};
    for (uint32_t f = 0; f < frames; ++f)
        out_seeds[f] = (float)(uint32_t)(rng.next() >> 40) * 0x1p-24f;
}

}  // extern "C"
