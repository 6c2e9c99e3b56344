// compute_shader.cpp — host mirror of the reference's render-graph node (src/lib.rs):
// ComputeShaderState / ComputeShaderNode (326-421) as a headless frame driver over the
// C-ABI kernels, with the two ping-pong images of prepare_bind_group (209-229):
//   bind group 0 = (input A, output B), bind group 1 = (input B, output A).
// Per frame: update() advances the state machine (345-377), then run() dispatches
// (379-421).  There is no asynchronous shader compilation, so Loading -> Init happens
// on the first frame.
#include <new>

#include "rt_abi.h"

namespace {

enum class State { Loading, Init, Update0, Update1 };

}  // namespace

struct rt_frame_driver {
    rt_ctx* ctx;
    float* images[2];  // A, B (device, caller-owned, zero-filled by the caller or init)
    uint32_t width, height;
    State state;
};

extern "C" {

rt_status rt_driver_create(rt_ctx* ctx, float* image_a, float* image_b, uint32_t width,
                           uint32_t height, rt_frame_driver** out) {
    if (!out) return RT_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!ctx) return RT_ERR_INVALID_CONTEXT;
    if (!image_a || !image_b || image_a == image_b) return RT_ERR_INVALID_ARGUMENT;
    if (width == 0 || height == 0) return RT_ERR_INVALID_SIZE;
    rt_frame_driver* d = new (std::nothrow) rt_frame_driver{ctx, {image_a, image_b}, width,
                                                            height, State::Loading};
    if (!d) return RT_ERR_NO_MEMORY;
    *out = d;
    return RT_OK;
}

rt_status rt_driver_destroy(rt_frame_driver* drv) {
    if (!drv) return RT_ERR_INVALID_ARGUMENT;
    delete drv;
    return RT_OK;
}

int rt_driver_state(const rt_frame_driver* drv) {
    if (!drv) return -1;
    switch (drv->state) {
        case State::Loading: return 0;
        case State::Init: return 1;
        case State::Update0: return 2;
        default: return 3;
    }
}

rt_status rt_driver_frame(rt_frame_driver* drv, const rt_scene_camera* camera,
                          const rt_sphere* spheres, uint32_t sphere_count, void* stream,
                          int* out_newest) {
    if (!drv || !camera) return RT_ERR_INVALID_ARGUMENT;
    // node.update() — lib.rs:350-376
    switch (drv->state) {
        case State::Loading: drv->state = State::Init; break;     // pipeline ready
        case State::Init: drv->state = State::Update1; break;     // lib.rs:362-367
        case State::Update0: drv->state = State::Update1; break;  // lib.rs:369-371
        case State::Update1: drv->state = State::Update0; break;  // lib.rs:372-374
    }
    // node.run() — lib.rs:396-418
    rt_status s = RT_OK;
    int newest = 1;
    if (drv->state == State::Init) {
        // init is dispatched with bind group 0, so it zeroes image B (lib.rs:402-406).
        s = rt_init_image(drv->ctx, drv->images[1], drv->width, drv->height, stream);
        newest = 1;
    } else {
        const int index = drv->state == State::Update0 ? 0 : 1;  // bind group index
        s = rt_update(drv->ctx, drv->images[index], drv->images[1 - index], drv->width,
                      drv->height, camera, spheres, sphere_count, stream);
        newest = 1 - index;
    }
    if (s == RT_OK && out_newest) *out_newest = newest;
    return s;
}

}  // extern "C"
