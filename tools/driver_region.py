"""The driver's timed region, replayed (diagnostic): bench.py --gpus 1 --steps 20 --warmup 5's
K3 region — after bench.py's 50-ms warm-up, a reset + 5 frames, then 20 timed frames in one
rt_update_frames call (synchronize on both sides) — repeated R times per variant, the
variants interleaved repetition by repetition, so box drift cancels.  Per variant: median
and quartiles of the wall time per step (perf_counter around the call and the closing
synchronize, as bench.py's value), of the HIP-event time per step, and of the host issue
time of the call.

Variants: name=ENV=V[,ENV=V...][;queues=Q][;wait=spin|block], e.g.  fork0=RT_FORK=0
q3=;queues=3  ctypes=RT_FASTCALL=0  spin=;wait=spin.  The library reads its diagnostic switches (RT_FORK, ...) from the
environment on every call; each variant has its own renderer, bound under its environment.
usage: python tools/driver_region.py [R] [CFG] variant...   (CFG K3 | K2)"""
import json
import os
import statistics as st
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
if os.environ.get("RT_REGION_SPIN"):
    # (before anything initialises the device) host waits spin instead of sleeping
    import ctypes
    ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(1)     # hipDeviceScheduleSpin
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 15
CFG = sys.argv[2] if len(sys.argv) > 2 else "K3"
specs = sys.argv[3:] or ["base="]


def parse(spec):
    name, _, rest = spec.partition("=")
    env, *opts = rest.split(";")
    kv = dict(x.split("=", 1) for x in env.split(",") if x)
    o = dict(x.split("=", 1) for x in opts if x)
    return name, kv, int(o.get("queues", 0)), o.get("wait", "block")


variants = [parse(s) for s in specs]
w, h = 1920, 1080
kind, nsph = (rt.SCENE_N, 500) if CFG == "K3" else (rt.SCENE_THREE, 3)
sc = rt.SphereCollection.generate(kind, nsph, 1)
seeds = rt.frame_seeds(0x5EED, 25)
cam0 = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=65536),
                                    w, h, float(seeds[0]))
cam_t = cam0.with_fields(camera_has_moved=0.0)
pipe = rt.ComputeShaderPipeline(0)
pipe.set_spheres(sc)
pipe.set_frames_per_launch(1)
pipe.set_frame_images("last_two")
stream = torch.cuda.current_stream()
# one renderer per variant (its calls are bound under that variant's environment)
rend = {v[0]: None for v in variants}
scratch = StripeRenderer(pipe, w, h, 0, 1)
torch.cuda.synchronize()
t_w = time.perf_counter()
while time.perf_counter() - t_w < 0.05:               # bench.py's --warm-ms 50
    scratch.frames(cam0, sc, seeds[:20])
    torch.cuda.synchronize()
res = {v[0]: {"wall": [], "events": [], "issue": []} for v in variants}
base_env = dict(os.environ)
for rep in range(R + 1):
    for name, kv, queues, wait in variants:
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update(kv)
        pipe.set_update_queues(queues)
        if rend[name] is None:
            rend[name] = StripeRenderer(pipe, w, h, 0, 1)
        r = rend[name]
        r.frames(cam0, sc, seeds[:5])                  # the warmup steps (frame 0 resets)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        r.frames(cam_t, sc, seeds[5:25])
        t1 = time.perf_counter()
        e1.record(stream)
        if wait == "spin":                             # (bench.py --host-wait spin)
            while not e1.query():
                pass
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if rep == 0:
            continue                                   # (first round: per-variant set-up)
        d = res[name]
        d["wall"].append((t2 - t0) / 20 * 1e6)
        d["events"].append(e0.elapsed_time(e1) / 20 * 1e3)
        d["issue"].append((t1 - t0) * 1e6)
os.environ.clear()
os.environ.update(base_env)


def q(v):
    s = sorted(v)
    return [round(s[len(s) // 4], 2), round(st.median(s), 2), round(s[(3 * len(s)) // 4], 2)]


for name, kv, queues, wait in variants:
    d = res[name]
    print(json.dumps({"cfg": CFG, "variant": name, "env": kv, "queues": queues, "wait": wait,
                      "reps": R,
                      "wall_us_per_step_q1_med_q3": q(d["wall"]),
                      "events_us_per_step_q1_med_q3": q(d["events"]),
                      "issue_us_q1_med_q3": q(d["issue"])}))
pipe.close()
