/*
 * rt_abi.h — C-ABI drop-in boundary of the MI355X ray tracer (librt_hip.so).
 *
 * Replaces the reference's compute-shader plugin surface for the per-pixel hot path
 * (Sur091/GPU-Ray-Tracing @ /root/reference):
 *   - ComputeShaderComputePlugin           src/lib.rs:104-136
 *   - ComputeShaderPipeline (3 layouts)    src/lib.rs:231-324
 *   - prepare_* bind-group systems         src/lib.rs:151-229
 *   - ComputeShaderNode::run dispatch      src/lib.rs:379-421
 *   - WGSL kernels `init` / `update`       assets/compute_shader.wgsl:65-70, 333-364
 *
 * Plain C types only: pointers, sizes, fixed-width integers. No C++ or torch types.
 * Every function returns an rt_status (0 = ok).
 *
 * Data contract (identical to the reference's bind groups):
 *   group 0  input / output images: RGBA32F, row-major, tightly packed (pitch = width
 *            texels = width*16 bytes). RGB = running mean, A = sample count
 *            (wgsl:4-5, 339-341, 362-363).  Device pointers, caller-owned.
 *   group 1  rt_scene_camera, 176 bytes (wgsl:7-42 == camera.rs:256-291). Host pointer,
 *            read during the call; passed to the kernel by value (kernarg -> SGPRs).
 *   group 2  sphere_count + array of rt_sphere, 32-byte stride (wgsl:46-47, 151-155 ==
 *            sphere.rs:14-26).  Host pointer; uploaded to the device only when its bytes
 *            change (the reference re-uploads every frame, lib.rs:177-207).
 *   dispatch one progressive sample per pixel per update (wgsl:352-358).
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define RT_API __attribute__((visibility("default")))
#else
#define RT_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------ */
/* Data layouts                                                                          */
/* ------------------------------------------------------------------------------------ */

/* SceneCamera — camera.rs:256-291 (#[repr(C)], 11 x (Vec3 + f32) = 176 B), wgsl:7-40.
 * Fields marked "unused" are carried for layout parity only (wgsl "No uses"). */
typedef struct rt_scene_camera {
    float center[3];              /*   0  used: ray origin without defocus (wgsl:319) */
    float viewport_height;        /*  12  unused */
    float viewport_upper_left[3]; /*  16  used (wgsl:315) */
    float viewport_width;         /*  28  unused */
    float pixel_delta_u[3];       /*  32  used (wgsl:316) */
    float defocus_angle;          /*  44  used: > 0 enables the thin lens (wgsl:319) */
    float pixel_delta_v[3];       /*  48  used (wgsl:317) */
    float aspect_ratio;           /*  60  unused */
    float defocus_disk_u[3];      /*  64  used (wgsl:330) */
    float _padding0;              /*  76 */
    float viewport_u[3];          /*  80  unused */
    float _padding1;              /*  92 */
    float defocus_disk_v[3];      /*  96  used (wgsl:330) */
    float max_depth;              /* 108  used: bounce limit, u32(max_depth) (wgsl:264) */
    float look_from[3];           /* 112  unused */
    float samples_per_pixel;      /* 124  used: accumulation cap (wgsl:343,352) */
    float look_at[3];             /* 128  unused */
    float camera_has_moved;       /* 140  used: > 0.5 resets the accumulator (wgsl:345) */
    float vup[3];                 /* 144  unused */
    float random_seed;            /* 156  used: per-frame seed in [0,1) (wgsl:311,353) */
    float viewport_v[3];          /* 160  unused */
    float defocus_radius;         /* 172  unused */
} rt_scene_camera;

/* GpuSphere — sphere.rs:20-26 (position: Vec3, radius: f32, material.color: Vec4), 32 B,
 * == WGSL Sphere (wgsl:151-155).  Material type is encoded in color[3] (wgsl:272-284):
 *   color[3] < -1          Lambertian, albedo = color.rgb
 *   -1 <= color[3] <= 1    metal, albedo = color.rgb, fuzz = color[3]
 *   color[3] > 1           dielectric, refraction index = color[0]                      */
typedef struct rt_sphere {
    float position[3];
    float radius;
    float color[4];
} rt_sphere;

/* Compile-time layout locks: the byte offsets a Rust binder's #[repr(C)] structs have
 * (SceneCamera camera.rs:256-291, GpuSphere sphere.rs:20-26; WGSL wgsl:7-40, 151-155).
 * Any reordering or resizing of a field fails the build of every translation unit. */
#if defined(__cplusplus)
#define RT_STATIC_ASSERT(cond, msg) static_assert(cond, msg)
#else
#define RT_STATIC_ASSERT(cond, msg) _Static_assert(cond, msg)
#endif
RT_STATIC_ASSERT(sizeof(rt_scene_camera) == 176, "SceneCamera is 176 bytes (camera.rs:256-291)");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, center) == 0, "center @ 0");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, viewport_height) == 12, "viewport_height @ 12");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, viewport_upper_left) == 16, "viewport_upper_left @ 16");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, viewport_width) == 28, "viewport_width @ 28");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, pixel_delta_u) == 32, "pixel_delta_u @ 32");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, defocus_angle) == 44, "defocus_angle @ 44");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, pixel_delta_v) == 48, "pixel_delta_v @ 48");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, aspect_ratio) == 60, "aspect_ratio @ 60");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, defocus_disk_u) == 64, "defocus_disk_u @ 64");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, _padding0) == 76, "_padding0 @ 76");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, viewport_u) == 80, "viewport_u @ 80");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, _padding1) == 92, "_padding1 @ 92");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, defocus_disk_v) == 96, "defocus_disk_v @ 96");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, max_depth) == 108, "max_depth @ 108");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, look_from) == 112, "look_from @ 112");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, samples_per_pixel) == 124, "samples_per_pixel @ 124");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, look_at) == 128, "look_at @ 128");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, camera_has_moved) == 140, "camera_has_moved @ 140");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, vup) == 144, "vup @ 144");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, random_seed) == 156, "random_seed @ 156");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, viewport_v) == 160, "viewport_v @ 160");
RT_STATIC_ASSERT(offsetof(rt_scene_camera, defocus_radius) == 172, "defocus_radius @ 172");
RT_STATIC_ASSERT(sizeof(rt_sphere) == 32, "GpuSphere is 32 bytes (sphere.rs:20-26)");
RT_STATIC_ASSERT(offsetof(rt_sphere, position) == 0, "position @ 0");
RT_STATIC_ASSERT(offsetof(rt_sphere, radius) == 12, "radius @ 12");
RT_STATIC_ASSERT(offsetof(rt_sphere, color) == 16, "material.color @ 16");

/* CameraSettings — camera.rs:9-28 (main-world settings the camera builder consumes). */
typedef struct rt_camera_settings {
    float field_of_view;          /* degrees (camera.rs:37: 20) */
    uint32_t samples_per_pixel;   /* camera.rs:33: 500 */
    uint32_t camera_has_moved;    /* bool (camera.rs:35: true) */
    uint32_t max_depth;           /* camera.rs:34: 30 */
    float vup[3];                 /* camera.rs:40 */
    float look_from[3];           /* camera.rs:38 */
    float look_at[3];             /* camera.rs:39 */
    float defocus_angle;          /* degrees (camera.rs:42: 0.6) */
    float focus_distance;         /* camera.rs:43: 10 */
} rt_camera_settings;

/* Image stripe partition for multi-GPU rendering.  The image is cut into
 * bands of RT_STRIPE_ROWS rows; band s belongs to rank (s mod nranks).  A rank's local
 * buffer holds its bands back to back (local row = local_band * RT_STRIPE_ROWS + r).
 * Pixel coordinates (and therefore every RNG seed) stay global. */
#define RT_STRIPE_ROWS 8u

/* A rank's share as an arithmetic set of bands (ABI 7): global bands first, first + step,
 * ..., first + (count - 1) * step, held at local rows RT_STRIPE_ROWS * j ... of the rank's
 * compact images (local band j = global band first + j * step).  The round-robin stripes of
 * rank r of n are {r, n, ceil((bands - r) / n)}; a contiguous range of bands is {first, 1,
 * count} — what rt_partition_bands gives for a cost-balanced partition.  first < 65536 and
 * step < 32768 (the kernels' packed stripe map). */
typedef struct rt_band_set {
    uint32_t first;
    uint32_t step;
    uint32_t count;
} rt_band_set;

/* ------------------------------------------------------------------------------------ */
/* Status codes (the reference panics / unwraps instead: lib.rs:216-217, 356-358, 399-411) */
/* ------------------------------------------------------------------------------------ */
typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARGUMENT = 1, /* null pointer, zero size, in == out where forbidden */
    RT_ERR_INVALID_SIZE = 2,     /* width/height/count out of range */
    RT_ERR_INVALID_DEVICE = 3,   /* device ordinal does not exist */
    RT_ERR_HIP = 4,              /* a HIP runtime call failed (rt_last_error has text) */
    RT_ERR_NO_MEMORY = 5,
    RT_ERR_INVALID_CONTEXT = 6,
    RT_ERR_COMM = 7              /* an RCCL call failed (rt_last_error has RCCL's text) */
} rt_status;

/* One context per device; calls on one ctx are externally serialized.  A context keeps
 * device state that its launches read (sphere records, candidate lists, tile costs): use
 * ONE stream per context, or synchronize before switching streams — a scene change or a
 * list rebuild is ordered only on the stream of the call that makes it. */
typedef struct rt_ctx rt_ctx;

/* Version / introspection ------------------------------------------------------------ */
RT_API uint32_t rt_abi_version(void); /* RT_ABI_VERSION */
#define RT_ABI_VERSION 7u
/* Text of the last error on this thread (never NULL). */
RT_API const char* rt_last_error(void);
/* Trace-kernel instances (rt_launch_info.kernel) and their names as rocprofv3 lists them
 * (rt_kernel_name).  The library picks the instance per launch: the reference's exhaustive
 * scan, the culled scan (bounce rays), the camera-ray-only instance with candidate lists
 * (max_depth <= 1; one wave per tile), and its frame groups of two / four waves per tile
 * (fused multi-frame launches) or per pair of tiles (two pixels per lane). */
#define RT_KERNEL_EXHAUSTIVE 0
#define RT_KERNEL_CULLED 1
#define RT_KERNEL_LIST 2
#define RT_KERNEL_LIST_PAIR 3
#define RT_KERNEL_LIST_QUAD 4
/* bounce rays (max_depth >= 2), several frames per launch (rt_set_path_compaction):
 * paths kept by the wave of their pixel, compacted across four waves, frame pairs */
#define RT_KERNEL_BOUNCE 5
#define RT_KERNEL_BOUNCE_COMPACT 6
#define RT_KERNEL_BOUNCE_PAIR 7
/* one `update` dispatch (one frame per launch) of the camera-ray-only case: several
 * adjacent tiles per wave, parameters in one compact block (rt_set_single_kernel) */
#define RT_KERNEL_SINGLE 8
/* the same with one tile per wave, for small per-rank shares */
#define RT_KERNEL_SINGLE_ONE 9
/* bounce rays, each tile's frames split into chunks traced by separate waves, the last
 * finisher accumulating them in order (RT_PATHS_SPLIT) */
#define RT_KERNEL_BOUNCE_SPLIT 10
/* frame groups of two / four waves per pair of horizontally adjacent tiles: each lane traces
 * one pixel of each tile (ABI 6) */
#define RT_KERNEL_LIST_PAIR2 11
#define RT_KERNEL_LIST_QUAD2 12
/* The instance's name as rocprofv3 lists it ("rt_trace_kernel<k>", "rt_bounce_kernel<m>",
 * "rt_single_kernel<p>", "rt_tpair_kernel<g>"), "rt_trace_kernel" for an unknown id. */
RT_API const char* rt_kernel_name(int which);
/* What the last rt_update / rt_render / rt_render_stripes / rt_update_frames call on this
 * context launched: trace launches, frames traced, the most frames one launch carried, the
 * instance of its last launch (RT_KERNEL_*, -1 before any launch), the concurrent parts
 * (streams or queues) its last frame ran as (rt_set_update_queues; each part is one launch)
 * and how its last launch was submitted (RT_SUBMIT_HIP or RT_SUBMIT_AQL). */
typedef struct rt_launch_info {
    uint32_t launches;
    uint32_t frames;
    uint32_t max_frames_per_launch;
    int32_t kernel;
    uint32_t queues;
    uint32_t submit;
    /* 1: the hit normal's division ran as one Markstein step per component (checked at
     * upload to give the IEEE quotient for every numerator and each of the scene's distinct
     * radii, at most 16 of them); 0: two correction steps */
    uint32_t normal_rn;
} rt_launch_info;
RT_API rt_status rt_last_launch_info(const rt_ctx* ctx, rt_launch_info* out);
/* Diagnostic: the per-tile candidate lists of camera rays the context built last (culled
 * scan; rebuilt when the camera geometry, image, stripe map or scene change).  A tile lists
 * every sphere its camera rays can hit, at most 19 (rt_kernels.h kCandMax); a tile whose
 * cone admits more, or is degenerate, has no list and its camera rays scan the whole scene
 * with the per-wave culling (same pixels, slower).  out[0] = tiles, out[1] = tiles without a
 * list, out[2] = entries over the listed tiles, out[3] = the longest list, out[4] = the list
 * capacity.  Synchronous (reads the counts back); all zero before any list was built. */
RT_API rt_status rt_candidate_stats(rt_ctx* ctx, uint64_t out[5]);

/* Context ---------------------------------------------------------------------------- */
/* Create a context on HIP device `device`.  Replaces ComputeShaderPipeline::from_world
 * (lib.rs:240-324): there is no shader compile step, code objects are linked in.
 * A context keeps device state its launches share (sphere records, candidate lists, tile
 * order, hash tables) and rewrites it in stream order: issue every call on one context
 * from one stream (as the reference's render node does), or synchronise before switching
 * streams.  Separate contexts are independent. */
RT_API rt_status rt_create(int device, rt_ctx** out_ctx);
RT_API rt_status rt_destroy(rt_ctx* ctx);

/* Sphere-list scan strategy of the trace kernel.  Both give bit-identical images.
 *   RT_SCAN_EXHAUSTIVE  the reference's linear walk: every ray tests every sphere
 *                       (wgsl:169-177).
 *   RT_SCAN_CULLED      (default) exact wave-level culling: spheres that provably miss
 *                       every ray of a 64-ray wave are skipped, the rest are tested
 *                       exactly in list order. */
#define RT_SCAN_EXHAUSTIVE 0
#define RT_SCAN_CULLED 1
RT_API rt_status rt_set_scan_mode(rt_ctx* ctx, int mode);

/* Scene upload (explicit form of prepare_sphere_buffer, lib.rs:177-207).  The update
 * calls below also accept host spheres and upload them only when their bytes change. */
RT_API rt_status rt_set_spheres(rt_ctx* ctx, const rt_sphere* spheres, uint32_t count,
                         void* stream);

/* `init` (wgsl:65-70; dispatched in the Init state, lib.rs:398-407):
 * out[x,y] = (0,0,0,0) for every texel of a width x height image. */
RT_API rt_status rt_init_image(rt_ctx* ctx, float* out_rgba, uint32_t width, uint32_t height,
                        void* stream);

/* `update` (wgsl:333-364; dispatched every frame, lib.rs:408-417): one progressive sample
 * per pixel.  in_rgba and out_rgba are device images (must not alias: the reference
 * ping-pongs two textures, lib.rs:218-227).  spheres/count/camera are host pointers.
 * in_rgba must be a valid, fully mapped width x height image even when the camera resets
 * the accumulator (camera_has_moved > 0.5): the kernels load it before they know the
 * reset and then discard the values (the same holds for every call's input images). */
RT_API rt_status rt_update(rt_ctx* ctx, const float* in_rgba, float* out_rgba, uint32_t width,
                    uint32_t height, const rt_scene_camera* camera,
                    const rt_sphere* spheres, uint32_t sphere_count, void* stream);

/* Fused multi-frame accumulate: bit-identical to `frames` chained rt_update calls where
 * call f uses `camera` with random_seed = random_seeds[f] and camera_has_moved =
 * (f == 0 ? camera->camera_has_moved : 0).  The accumulator stays in registers across
 * frames (one HBM read + one write per pixel).  in_rgba may equal out_rgba. */
RT_API rt_status rt_render(rt_ctx* ctx, const float* in_rgba, float* out_rgba, uint32_t width,
                    uint32_t height, const rt_scene_camera* camera,
                    const rt_sphere* spheres, uint32_t sphere_count, uint32_t frames,
                    const float* random_seeds, void* stream);

/* The reference's per-frame loop (ComputeShaderNode ping-pong, lib.rs:366-374, 408-417)
 * driven from C: `frames` progressive `update`s alternating between image_a and image_b
 * (frame f reads the image frame f-1 wrote; frame 0 reads image_a; frame f writes its
 * image to image_b for even f, image_a for odd f).  Frame f uses random_seeds[f] and
 * camera_has_moved = (f == 0 ? camera->camera_has_moved : 0).  Restricted to the stripe
 * bands of rank/nranks (nranks = 1: whole image; images are then compact local buffers as
 * for rt_render_stripes).  *out_newest receives 0 if image_a holds the result, 1 for
 * image_b.  Afterwards BOTH images hold exactly what `frames` chained rt_update calls leave
 * (the newest frame and the one before).  Frames run in launches of
 * rt_set_frames_per_launch frames (default 64) in the culled scan mode — camera rays only
 * (max_depth <= 1, the camera-ray-only instances) and bounce rays (max_depth >= 2, the
 * bounce instance) alike; within a launch each wave carries its pixels' accumulator in
 * registers from frame to frame and writes the images of the launch's last two frames (the
 * earlier ones would be overwritten unread).  The exhaustive scan mode, and cameras or
 * scenes outside the fast instances' proven domain at max_depth <= 1, run one frame per
 * launch.  No per-frame host round trip. */
/* Frames rt_update_frames runs per fused launch (see above): 0 = automatic (64), 1 = one
 * `update` dispatch per frame, exactly the reference's dispatch structure, n = up to n (at
 * most 128).  The cap applies to the camera-ray-only and the bounce launches. */
RT_API rt_status rt_set_frames_per_launch(rt_ctx* ctx, uint32_t frames_per_launch);
/* Images of fused multi-frame launches (rt_set_frames_per_launch above 1).  The reference
 * writes every frame's image to the texture its dispatch binds as output (lib.rs:218-227,
 * 366-374; wgsl:362-363).
 *   RT_FRAME_IMAGES_LAST_TWO  (default) a launch writes the images of its last two frames
 *                             only: each earlier frame's image would be overwritten two
 *                             frames later, unread, so both buffers end up the same.
 *   RT_FRAME_IMAGES_EVERY     every frame's image is written to the buffer its chained
 *                             update writes (frame f of a call: image_b for even f, image_a
 *                             for odd f) — the reference's per-frame memory traffic, with
 *                             only the launch boundary between the frames removed.  Used for
 *                             the per-frame steps of small rank shares (bench.py, DESIGN.md
 *                             §6), where one launch per frame is bound by the launch itself.
 * The camera-ray-only and the bounce instances; pixel results are identical. */
#define RT_FRAME_IMAGES_LAST_TWO 0
#define RT_FRAME_IMAGES_EVERY 1
RT_API rt_status rt_set_frame_images(rt_ctx* ctx, int mode);
/* rt_update_frames at max_depth <= 1 traces with several waves per 8x8 tile, each taking
 * a different frame of each group of frames (the others hand their colours to wave 0,
 * which accumulates every frame in order: the same bits), whenever every pixel
 * holds the sample count the context expects (otherwise the launch falls back to one wave
 * per tile).  The groups' waves own one tile (ON: 2 waves, QUAD: 4) or a pair of adjacent
 * tiles, each lane tracing one pixel of each (ON2: 2 waves, QUAD2: 4; ABI 6).  AUTO
 * (default): 4 waves per tile for launches of at most 6144 tiles (small per-rank shares),
 * 4 waves per pair of tiles up to 12288 tiles, 2 waves per pair above (whole images) — the
 * pair forms when candidate lists exist, else 2 waves per tile; OFF: one wave per tile. */
#define RT_FRAME_PAIRS_AUTO 0
#define RT_FRAME_PAIRS_OFF 1
#define RT_FRAME_PAIRS_ON 2
#define RT_FRAME_PAIRS_QUAD 3
#define RT_FRAME_PAIRS_ON2 4
#define RT_FRAME_PAIRS_QUAD2 5
RT_API rt_status rt_set_frame_pairs(rt_ctx* ctx, int mode);
/* Tile scheduling (culled scan mode).  AUTO (default): fused multi-frame launches (the
 * camera-ray-only kernels and the bounce instance): the first such launch for a camera
 * geometry / image / stripe map / scene records each 8x8 tile's duration on the device,
 * and later launches hand the costliest tiles to the first workgroups so that cheap tiles
 * fill the tail (strong scaling: a rank's share is only a few workgroups per SIMD);
 * one-frame launches (rt_single_kernel): from the second launch of a camera geometry on,
 * workgroups are dispatched by decreasing load of their tiles' candidate lists.  OFF:
 * raster order everywhere.  Pixel results are identical. */
#define RT_TILE_ORDER_AUTO 0
#define RT_TILE_ORDER_OFF 1
RT_API rt_status rt_set_tile_order(rt_ctx* ctx, int mode);
/* One-frame updates of rt_update_frames (rt_set_frames_per_launch(1), the one-frame
 * instances) as `queues` concurrent parts, each a launch on its own stream: the caller's
 * stream runs part 0, context-owned streams the others, forked from and joined back into
 * the caller's stream by events inside the call (the call's work stays ordered on the
 * caller's stream).  Each part takes every queues-th workgroup of the cost order (or every
 * queues-th band), so a part's next frame depends only on its own previous frame: one
 * part's kernel boundary and tail overlap the other parts' work.  0 = automatic, 1 = one
 * launch per update, at most RT_MAX_UPDATE_QUEUES.  Pixel results are identical. */
#define RT_MAX_UPDATE_QUEUES 4u
RT_API rt_status rt_set_update_queues(rt_ctx* ctx, uint32_t queues);
/* How rt_update_frames submits one-frame updates when a call carries two or more of them.
 *   RT_SUBMIT_HIP   HIP launches on the caller's stream (and the context's extra streams for
 *                   concurrent parts).
 *   RT_SUBMIT_AQL   every frame of every part is an AQL dispatch packet on an HSA queue the
 *                   context owns (one queue per part, frames in order on it), written by the
 *                   library (≈0.25 µs of host time per frame and part against 3-4 µs per HIP
 *                   launch) with no cache fence between a part's frames (the chain kernels
 *                   hand the image over through write-through stores and L1-bypassing
 *                   loads); ordered after the work issued on the caller's stream before the
 *                   call and before the work issued after it (when the stream is busy it
 *                   writes a value a one-wave kernel on the queues waits for; the stream
 *                   waits for a value the queues' last packet writes), so the call stays
 *                   asynchronous.  The packets' arguments live in VRAM written through the
 *                   host's large-BAR mapping (one HDP flush per call), else in host memory.
 *                   Measured at parity with HIP launches on whole images (K3 15.2-15.8 µs
 *                   per update at 2 queues against 14.9-15.8), faster on mid-sized rank
 *                   shares (a 4-rank K3 share 6.76 against 7.54-7.68 µs), slower on small
 *                   ones (an 8-rank share 5.8 against 5.0); four HSA queues beside HIP's are
 *                   oversubscribed.
 *   RT_SUBMIT_AUTO  (default) HIP launches: AQL submission is opt-in (it needs HSA queues,
 *                   host-visible VRAM or host memory for the arguments and the code object's
 *                   chain kernels, and has no multi-GPU record yet).
 * Parts under AQL (rt_set_update_queues 0): 2 for launches of 2 000 tiles or more, else 1.
 * Every wait of the AQL path is bounded: a segment whose caller's stream has not reached it
 * after RT_CHAIN_GO_MS milliseconds (environment, default 10 000) drops its frames instead
 * of running them early; that, an HSA queue error or a segment that does not complete in
 * time is returned as RT_ERR_HIP by the context's next call (rt_update_frames, rt_destroy,
 * rt_update_submit_status), and the context runs HIP launches from then on.
 * Pixel results are identical in every mode. */
#define RT_SUBMIT_AUTO 0
#define RT_SUBMIT_HIP 1
#define RT_SUBMIT_AQL 2
RT_API rt_status rt_set_update_submit(rt_ctx* ctx, int mode);
/* Launch timing (ABI 7, diagnostic): while enabled, the fused launches of each
 * rt_update_frames / rt_update_frames_bands call (the frame-chain, fused camera-ray and bounce
 * instances) carry the context's two timing events in their own dispatch packets
 * (hipExtModuleLaunchKernel: no marker packets on the stream); rt_last_call_kernel_time then
 * gives the time from the start of the call's first such launch to the end of its last
 * (milliseconds; synchronous: waits for that launch) and how many launches carried them.
 * RT_ERR_INVALID_ARGUMENT when the last call had none (one-frame launches, AQL packets).
 * Pixel results are identical; the ext launch path costs a call on an idle GPU ≈ 9 µs more
 * (profiles/r06/r06i/), so time what it measures apart from wall-clock regions. */
RT_API rt_status rt_set_launch_timing(rt_ctx* ctx, int enable);
RT_API rt_status rt_last_call_kernel_time(rt_ctx* ctx, float* out_ms, uint32_t* out_launches);
/* Whether AQL submission is available on the context's device (*aql_available; if not,
 * rt_last_error() says why), whether a go wait gave up (*go_give_ups, 0 or 1: a segment
 * whose caller's stream had not reached it within the bound; its frames were dropped; 0 in
 * a correct run) and the AQL packets submitted so far.  Synchronous: waits (bounded) for
 * the context's AQL work in flight.  Creates no HSA queue. */
RT_API rt_status rt_update_submit_status(rt_ctx* ctx, int* aql_available, uint32_t* go_give_ups,
                                         uint64_t* packets);
/* Bounce paths (max_depth >= 2): RT_PATHS_PER_WAVE keeps every path in the wave of its
 * pixel (one tile per workgroup); RT_PATHS_PAIR runs two waves per tile on alternate
 * frames, the second handing its colours to the first through LDS (shorter chains for
 * small per-rank shares); RT_PATHS_COMPACT repacks the live paths of a workgroup's four
 * waves into the fewest waves after every bounce (ballot + mbcnt prefix, path state through
 * LDS); RT_PATHS_SPLIT splits a tile's frames into consecutive chunks (2 or 4), each traced
 * by its own wave: the first keeps its accumulator in registers, the later ones store their
 * frames' colours (device scratch the context keeps: 1 KB per tile and frame), and the tile's
 * last finishing chunk accumulates them in order and writes the images; once a launch has
 * measured the tile costs, only the tiles costlier than a quarter of the launch's ideal span
 * split and every unit is dispatched by its own cost.  RT_PATHS_AUTO (default): RT_PATHS_SPLIT
 * with 4 chunks for launches of at most 20 000 tiles (small per-rank shares: a few waves per
 * SIMD) once their costs are measured, else RT_PATHS_PER_WAVE.  Pixel results
 * are identical in every mode. */
#define RT_PATHS_AUTO 0
#define RT_PATHS_PER_WAVE 1
#define RT_PATHS_COMPACT 2
#define RT_PATHS_PAIR 3
#define RT_PATHS_SPLIT 4
RT_API rt_status rt_set_path_compaction(rt_ctx* ctx, int mode);
/* One-frame launches of the camera-ray-only case (rt_update, rt_render / rt_update_frames
 * launches carrying one frame): AUTO (default) runs RT_KERNEL_SINGLE (two tiles per wave),
 * or RT_KERNEL_SINGLE_ONE for small launches; PAIR / ONE force either; OFF runs the general
 * RT_KERNEL_LIST instance.  Pixel results are identical. */
#define RT_SINGLE_AUTO 0
#define RT_SINGLE_OFF 1
#define RT_SINGLE_PAIR 2
#define RT_SINGLE_ONE 3
RT_API rt_status rt_set_single_kernel(rt_ctx* ctx, int mode);
/* The frames-per-launch cap rt_update_frames applies for `camera` (its max_depth) with the
 * context's settings.  The image size, stripe map and scene are not known here, and a
 * launch whose camera rays fall outside the fast instances' proven domain runs one frame
 * per launch: rt_last_launch_info reports what a call actually launched. */
RT_API rt_status rt_get_frames_per_launch(const rt_ctx* ctx, const rt_scene_camera* camera,
                                          uint32_t* out_frames);
RT_API rt_status rt_update_frames(rt_ctx* ctx, float* image_a, float* image_b, uint32_t width,
                                  uint32_t height, uint32_t rank, uint32_t nranks,
                                  const rt_scene_camera* camera, const rt_sphere* spheres,
                                  uint32_t sphere_count, uint32_t frames,
                                  const float* random_seeds, void* stream, int* out_newest);

/* Multi-GPU tile path: the same as rt_render (frames >= 1) restricted to the stripe
 * bands of `rank` out of `nranks` (RT_STRIPE_ROWS rows each, band s -> rank s % nranks).
 * in/out are compact local images of width x rt_stripe_local_rows(height,rank,nranks). */
RT_API rt_status rt_render_stripes(rt_ctx* ctx, const float* in_local, float* out_local,
                            uint32_t width, uint32_t height, uint32_t rank,
                            uint32_t nranks, const rt_scene_camera* camera,
                            const rt_sphere* spheres, uint32_t sphere_count,
                            uint32_t frames, const float* random_seeds, void* stream);
RT_API uint32_t rt_stripe_local_rows(uint32_t height, uint32_t rank, uint32_t nranks);

/* rt_update_frames over an explicit band set instead of the round-robin stripes of
 * rank / nranks: image_a and image_b are compact local images of width x (bands->count *
 * RT_STRIPE_ROWS) rows; every other argument, and the result, as rt_update_frames (the
 * round-robin call equals this one with {rank, nranks, ceil((bands - rank) / nranks)}). */
RT_API rt_status rt_update_frames_bands(rt_ctx* ctx, float* image_a, float* image_b,
                                        uint32_t width, uint32_t height,
                                        const rt_band_set* bands, const rt_scene_camera* camera,
                                        const rt_sphere* spheres, uint32_t sphere_count,
                                        uint32_t frames, const float* random_seeds,
                                        void* stream, int* out_newest);
/* The per-band costs the context's last cost-recording launch measured (the fused
 * launches' per-tile durations in device clock ticks, summed over each local band's tiles;
 * rt_set_tile_order), for that launch's share: out_cost[j] for local band j of `bands`,
 * which must be the band set (and width, height) that launch ran, with the same camera
 * geometry and scene since — RT_ERR_INVALID_ARGUMENT otherwise, or when no launch has
 * recorded costs.  Synchronous (reads the costs back on the
 * context's device with a blocking copy). */
RT_API rt_status rt_band_costs(rt_ctx* ctx, uint32_t width, uint32_t height,
                               const rt_band_set* bands, double* out_cost);
/* Cost-balanced partition (host only): the nbands bands, band b costing band_cost[b] >= 0,
 * cut into nranks contiguous ranges (out[r] = {first_r, 1, count_r}, in band order, a range
 * may be empty; empty ones are {0, 1, 0}) that minimise the largest range cost — exactly:
 * bisection over that cost with a greedy cut, O(nbands) memory; among optimal cuts one that
 * gives every rank a band while there are bands (ranges as long as fit, in order, each
 * leaving a band for every later rank).  Any partition gives bit-identical
 * pixels: every seed is a function of the global pixel (wgsl:309-311, 353). */
RT_API rt_status rt_partition_bands(const double* band_cost, uint32_t nbands, uint32_t nranks,
                                    rt_band_set* out);
/* Root side of a band-set gather: `gathered` holds nranks compact buffers back to back in
 * rank order, each padded to rows_per_rank rows (>= every sets[r].count * RT_STRIPE_ROWS);
 * scatter them into the width x height image out_rgba.  The sets must cover every band of
 * the image exactly once. */
RT_API rt_status rt_deinterleave_bands(rt_ctx* ctx, const float* gathered, float* out_rgba,
                                       uint32_t width, uint32_t height, uint32_t nranks,
                                       const rt_band_set* sets, uint32_t rows_per_rank,
                                       void* stream);

/* Root side of the gather: `gathered` holds nranks compact buffers back to back, each
 * padded to max-local-rows (rt_stripe_local_rows(height,0,nranks)) rows; scatter them
 * into the full width x height image `out_rgba` (device pointers). */
RT_API rt_status rt_deinterleave_stripes(rt_ctx* ctx, const float* gathered, float* out_rgba,
                                  uint32_t width, uint32_t height, uint32_t nranks,
                                  void* stream);

/* The multi-GPU collective: ONE RCCL gather over xGMI of every rank's
 * finished stripe bands to the root, then the de-interleave there.  The reference renders
 * on one device (ComputeShaderNode::run, lib.rs:379-421, one dispatch per frame); these
 * calls are what a host driving one context per GPU adds around rt_update_frames /
 * rt_render_stripes.  A communicator spans nranks ranks, one GPU each:
 *   - one process per GPU: rank 0 calls rt_comm_unique_id, sends the RT_COMM_ID_BYTES bytes
 *     to every rank by any means, and every rank calls rt_comm_create with them
 *     (ncclGetUniqueId + ncclCommInitRank, rccl.h:187, 220; collective: all ranks must call
 *     it concurrently);
 *   - one process driving several GPUs: rt_comm_create_all (ncclCommInitAll, rccl.h:236),
 *     with rt_comm_group_start / rt_comm_group_end around the per-device gathers.
 * RCCL's own error text is returned through rt_last_error with RT_ERR_COMM. */
#define RT_COMM_ID_BYTES 128
typedef struct rt_comm rt_comm;
RT_API rt_status rt_comm_unique_id(uint8_t out_id[RT_COMM_ID_BYTES]);
/* A communicator on ctx's device (the rank's GPU). */
RT_API rt_status rt_comm_create(rt_ctx* ctx, const uint8_t id[RT_COMM_ID_BYTES], uint32_t nranks,
                                uint32_t rank, rt_comm** out_comm);
/* ndev communicators, out_comms[i] on device devices[i] with rank i. */
RT_API rt_status rt_comm_create_all(uint32_t ndev, const int* devices, rt_comm** out_comms);
RT_API rt_status rt_comm_destroy(rt_comm* comm);
RT_API rt_status rt_comm_info(const rt_comm* comm, uint32_t* out_rank, uint32_t* out_nranks,
                              int* out_device);
RT_API rt_status rt_comm_group_start(void);
RT_API rt_status rt_comm_group_end(void);
/* Gathers the rank's compact local image `local` (width x rt_stripe_local_rows(height, 0,
 * nranks) rows — every rank's buffer padded to the root's row count) into `gathered` on
 * the root (nranks such buffers back to back, rank order; NULL = a buffer the communicator
 * keeps) with one ncclGather (rccl.h:745) on `stream`, then de-interleaves it into the
 * width x height image `out_rgba` on the root (rt_deinterleave_stripes).  Non-root ranks
 * ignore `gathered` and `out_rgba`.  ctx must be on the communicator's device. */
RT_API rt_status rt_gather_stripes(rt_ctx* ctx, rt_comm* comm, const float* local,
                                   float* gathered, float* out_rgba, uint32_t width,
                                   uint32_t height, uint32_t root, void* stream);
/* The same gather for a band-set partition (sets[r] = rank r's band set, identical on every
 * rank): each rank's `local` is padded to max_r sets[r].count * RT_STRIPE_ROWS rows (the
 * ncclGather's equal send count); `gathered` (root, NULL = the communicator's buffer) holds
 * nranks such buffers; the root de-interleaves with rt_deinterleave_bands. */
RT_API rt_status rt_gather_bands(rt_ctx* ctx, rt_comm* comm, const float* local,
                                 float* gathered, float* out_rgba, uint32_t width,
                                 uint32_t height, const rt_band_set* sets, uint32_t root,
                                 void* stream);

/* Presentation (replaces the sprite of lib.rs:79-102, which shows the newest
 * Rgba32Float image on the window): quantizes the accumulator's mean colour to 8-bit RGBA
 * for an image file.  out_rgba8 is a device buffer of width*height*4 bytes, row 0 = top
 * (the image's row order, wgsl:336).  Per channel c of (r, g, b):
 *   RT_ENCODE_LINEAR: u8 = floor(min(max(c, 0), 1) * 255 + 0.5)   (f32 mul, then add)
 *   RT_ENCODE_SRGB:   u8 = number of j in 1..255 with c >= T[j], T = rt_srgb_thresholds
 *                     (sRGB transfer curve, exact quantization boundaries)
 * NaN -> 0; alpha = 255.  The float image itself (.npy/PFM) needs no conversion. */
#define RT_ENCODE_LINEAR 0
#define RT_ENCODE_SRGB 1
RT_API rt_status rt_present_rgba8(rt_ctx* ctx, const float* in_rgba, uint8_t* out_rgba8,
                                  uint32_t width, uint32_t height, int encoding, void* stream);
/* T[0] = 0 (unused); T[j], j = 1..255: the smallest f32 >= the linear value whose sRGB
 * encoding is (j - 0.5) / 255, computed in double (IEC 61966-2-1 curve). */
RT_API void rt_srgb_thresholds(float out[256]);

/* Diagnostic (no reference counterpart): checks on the device that the exact fast paths
 * of f32 division and sqrt used by the trace kernel (rt_device.h: div_core, sqrt_core)
 * return the IEEE bits on their documented domains — exhaustively for the defocus-disk
 * normalisation (all 2^32 values of its random input) and on n_random random cases for
 * division, sqrt and the scan's root selection built on them (random camera-domain rays
 * and spheres, half grazing).  out[0..3] = mismatches (defocus, division, sqrt, roots),
 * out[4] = cases.  Synchronous. */
RT_API rt_status rt_selftest_fastmath(rt_ctx* ctx, uint64_t n_random, uint64_t out[5]);

/* ------------------------------------------------------------------------------------ */
/* Host-side mirror of the reference's main-world code (C++ implementation, no device)   */
/* ------------------------------------------------------------------------------------ */

/* CameraSettings::default() — camera.rs:30-46. */
RT_API void rt_camera_settings_default(rt_camera_settings* out);

/* SceneCamera::from(&CameraSettings) — camera.rs:293-351, with the image size as a
 * runtime argument (the reference hard-codes crate::SIZE = 1280x720, camera.rs:296,
 * 315-316) and the per-frame random_seed supplied by the caller (camera.rs:346 draws
 * rand::random()).  glam/Rust f32 operation order is reproduced exactly. */
RT_API rt_status rt_camera_from_settings(const rt_camera_settings* settings, uint32_t width,
                                  uint32_t height, float random_seed,
                                  rt_scene_camera* out);

/* Seeded scene generators (create_default_spheres, sphere.rs:45-153).
 *   kind 0: the three fixed large spheres (sphere.rs:114-136), glass / diffuse / metal.
 *   kind 1: "default-like": ground + 14x14 jittered grid (a,b in -7..7) + 3 large.
 *   kind 2: N-sphere: ground + grid a,b in -12..12 truncated to N-4 + 3 large (N>=4).
 * Uniform variates come from splitmix64(seed), f = (u32 >> 8) * 2^-24 (rand 0.9's f32).
 * Writes up to `capacity` spheres; *out_count receives the scene's sphere count. */
RT_API rt_status rt_scene_generate(uint32_t kind, uint32_t n_spheres, uint64_t seed,
                            rt_sphere* out, uint32_t capacity, uint32_t* out_count);

/* Per-frame seeds: random_seed_f = k_f / 2^24 with k_f the top 24 bits of splitmix64
 * outputs (seed 0x5EED in the bench).  Stands in for rand::random() (camera.rs:346). */
RT_API void rt_frame_seeds(uint64_t seed, uint32_t frames, float* out_seeds);

/* ComputeShaderNode state machine (lib.rs:326-421) as a headless frame driver:
 * Loading -> Init (dispatch init on image B) -> Update(1) <-> Update(0) ping-pong,
 * update(index) reads images[index] and writes images[1-index] (bind groups lib.rs:218-227:
 * group 0 = (A -> B), group 1 = (B -> A)).  `rt_driver_frame` advances one frame and
 * returns which image holds the newest result. */
typedef struct rt_frame_driver rt_frame_driver;
RT_API rt_status rt_driver_create(rt_ctx* ctx, float* image_a, float* image_b, uint32_t width,
                           uint32_t height, rt_frame_driver** out);
RT_API rt_status rt_driver_destroy(rt_frame_driver* drv);
/* Runs one render-graph frame: node.update() then node.run() (lib.rs:345-421).
 * *out_newest = 0 if image A holds the latest output, 1 for image B. */
RT_API rt_status rt_driver_frame(rt_frame_driver* drv, const rt_scene_camera* camera,
                          const rt_sphere* spheres, uint32_t sphere_count, void* stream,
                          int* out_newest);
/* 0 = Loading, 1 = Init, 2 = Update(0), 3 = Update(1). */
RT_API int rt_driver_state(const rt_frame_driver* drv);

#ifdef __cplusplus
}
#endif

#endif /* RT_ABI_H */
