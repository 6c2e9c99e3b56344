// camera.cpp — host mirror of src/camera.rs: CameraSettings::default (30-46) and
// SceneCamera::from(&CameraSettings) (293-351).
//
// glam 0.29 `Vec3` is a plain f32 struct; its operations are reproduced in their exact
// order (Rust does not contract a*b+c into an FMA; this file is built with
// -ffp-contract=off):
//   dot(a,b)      = (a.x*b.x + a.y*b.y) + a.z*b.z
//   length(v)     = sqrt(dot(v,v))
//   normalize(v)  = v * (1.0 / length(v))         (Vec3::normalize -> length_recip)
//   cross(a,b)    = (a.y*b.z - b.y*a.z, a.z*b.x - b.z*a.x, a.x*b.y - b.x*a.y)
//   v / s, s * v  = component-wise IEEE ops
//   f32::to_radians(d) = d * (PI_f32 / 180_f32)
//   f32::tan       = libm tanf
#include <cmath>
#include <cstring>

#include "rt_abi.h"

namespace {

struct Vec3 {
    float x, y, z;
};

Vec3 v(float x, float y, float z) { return Vec3{x, y, z}; }
Vec3 operator-(Vec3 a, Vec3 b) { return v(a.x - b.x, a.y - b.y, a.z - b.z); }
Vec3 operator*(float s, Vec3 a) { return v(s * a.x, s * a.y, s * a.z); }
Vec3 operator*(Vec3 a, float s) { return v(a.x * s, a.y * s, a.z * s); }
Vec3 operator/(Vec3 a, float s) { return v(a.x / s, a.y / s, a.z / s); }
float dot(Vec3 a, Vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
float length(Vec3 a) { return std::sqrt(dot(a, a)); }
Vec3 normalize(Vec3 a) { return a * (1.0f / length(a)); }
Vec3 cross(Vec3 a, Vec3 b) {
    return v(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
float to_radians(float deg) {
    const float rads_per_deg = 3.14159274101257324f / 180.0f;  // consts::PI / 180.0 in f32
    return deg * rads_per_deg;
}
Vec3 load(const float* p) { return v(p[0], p[1], p[2]); }
void store(float* p, Vec3 a) {
    p[0] = a.x;
    p[1] = a.y;
    p[2] = a.z;
}

}  // namespace

extern "C" {

void rt_camera_settings_default(rt_camera_settings* out) {
    if (!out) return;
    std::memset(out, 0, sizeof(*out));
    out->samples_per_pixel = 500;   // camera.rs:33
    out->max_depth = 30;            // camera.rs:34
    out->camera_has_moved = 1;      // camera.rs:35
    out->field_of_view = 20.0f;     // camera.rs:37
    out->look_from[0] = 13.0f;      // camera.rs:38
    out->look_from[1] = 2.0f;
    out->look_from[2] = 3.0f;
    out->vup[1] = 1.0f;             // camera.rs:40 (look_at = 0, camera.rs:39)
    out->defocus_angle = 0.6f;      // camera.rs:42
    out->focus_distance = 10.0f;    // camera.rs:43
}

rt_status rt_camera_from_settings(const rt_camera_settings* s, uint32_t width, uint32_t height,
                                  float random_seed, rt_scene_camera* out) {
    if (!s || !out) return RT_ERR_INVALID_ARGUMENT;
    if (width == 0 || height == 0) return RT_ERR_INVALID_SIZE;
    std::memset(out, 0, sizeof(*out));
    const float aspect_ratio = (float)width / (float)height;              // camera.rs:296
    const Vec3 look_from = load(s->look_from), look_at = load(s->look_at), vup = load(s->vup);
    const Vec3 camera_center = look_from;                                  // camera.rs:298
    const float theta = to_radians(s->field_of_view);                      // camera.rs:300
    const float h = std::tan(theta / 2.0f);                                // camera.rs:301
    const float viewport_height = 2.0f * h * s->focus_distance;            // camera.rs:302
    const float viewport_width = viewport_height * aspect_ratio;           // camera.rs:303
    const Vec3 w = normalize(look_from - look_at);                         // camera.rs:307
    const Vec3 u = normalize(cross(vup, w));                               // camera.rs:308
    const Vec3 vv = cross(w, u);                                           // camera.rs:309
    const Vec3 viewport_u = viewport_width * u;                            // camera.rs:311
    const Vec3 viewport_v = (-viewport_height) * vv;                       // camera.rs:312
    const Vec3 pixel_delta_u = viewport_u / (float)width;                  // camera.rs:315
    const Vec3 pixel_delta_v = viewport_v / (float)height;                 // camera.rs:316
    const Vec3 viewport_upper_left =                                       // camera.rs:319-320
        ((camera_center - s->focus_distance * w) - viewport_u / 2.0f) - viewport_v / 2.0f;
    const float defocus_radius =                                           // camera.rs:322-323
        s->focus_distance * std::tan(to_radians(s->defocus_angle / 2.0f));
    const Vec3 defocus_disk_u = u * defocus_radius;                        // camera.rs:324
    const Vec3 defocus_disk_v = vv * defocus_radius;                       // camera.rs:325

    store(out->center, look_from);
    out->viewport_height = viewport_height;
    store(out->viewport_upper_left, viewport_upper_left);
    out->viewport_width = viewport_width;
    store(out->pixel_delta_u, pixel_delta_u);
    out->defocus_angle = s->defocus_angle;
    store(out->pixel_delta_v, pixel_delta_v);
    out->aspect_ratio = aspect_ratio;
    store(out->defocus_disk_u, defocus_disk_u);
    store(out->viewport_u, viewport_u);
    store(out->defocus_disk_v, defocus_disk_v);
    out->max_depth = (float)s->max_depth;                                   // camera.rs:343
    store(out->look_from, look_from);
    out->samples_per_pixel = (float)s->samples_per_pixel;                   // camera.rs:344
    store(out->look_at, look_at);
    out->camera_has_moved = s->camera_has_moved ? 1.0f : 0.0f;              // camera.rs:345
    store(out->vup, vup);
    out->random_seed = random_seed;                                         // camera.rs:346
    store(out->viewport_v, viewport_v);
    out->defocus_radius = defocus_radius;
    return RT_OK;
}

}  // extern "C"
