"""Fixed cost of one timed call (diagnostic): a rank's K3 share (frame chains, every frame's
image written) timed wall-clock around one rt_update_frames call of F frames and a closing
wait, for several F, so that wall(F) = fixed + F * per_frame separates the call's fixed cost
(host issue, the dispatch reaching an idle GPU, completion reaching the host) from the
frames.  Variants of the region:
  ev     HIP events recorded around the call (bench.py's region before round 6)
  noev   no events: synchronize, clock, call, synchronize, clock
  stream the closing wait is the stream's synchronize instead of the device's
  ext    no events on the stream; the launch itself carries the timing events
         (rt_set_launch_timing: hipExtModuleLaunchKernel), read after the region
Also times an empty region (synchronize, clock, synchronize) and a 1-block kernel launch +
synchronize (torch's fill on a 4-byte tensor) for the host/runtime floor.
usage: python tools/call_latency.py [N] [rank] [reps]"""
import json
import statistics as st
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
RANK = int(sys.argv[2]) if len(sys.argv) > 2 else 0
R = int(sys.argv[3]) if len(sys.argv) > 3 else 15
FS = (1, 2, 5, 10, 20, 40)
w, h = 1920, 1080
sc = rt.SphereCollection.generate(rt.SCENE_N, 500, 1)
seeds = rt.frame_seeds(0x5EED, 5 + max(FS))
cam0 = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=65536),
                                    w, h, float(seeds[0]))
cam_t = cam0.with_fields(camera_has_moved=0.0)
pipe = rt.ComputeShaderPipeline(0)
pipe.set_spheres(sc)
pipe.set_frames_per_launch(0)
pipe.set_frame_images("every")
stream = torch.cuda.current_stream()
r = StripeRenderer(pipe, w, h, RANK, N)
scratch = StripeRenderer(pipe, w, h, RANK, N)
torch.cuda.synchronize()
t_w = time.perf_counter()
while time.perf_counter() - t_w < 0.05:
    scratch.frames(cam0, sc, seeds[:20])
    torch.cuda.synchronize()


def region(F, variant):
    r.frames(cam0, sc, seeds[:5])
    torch.cuda.synchronize()
    if variant == "ev":
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        r.frames(cam_t, sc, seeds[5:5 + F])
        e1.record(stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, e0.elapsed_time(e1) / 1e3
    pipe.set_launch_timing(variant == "ext")
    t0 = time.perf_counter()
    r.frames(cam_t, sc, seeds[5:5 + F])
    if variant == "stream":
        stream.synchronize()
    else:
        torch.cuda.synchronize()
    t = time.perf_counter() - t0
    if variant == "ext":
        try:
            return t, pipe.last_call_kernel_time()[0]
        except Exception:          # noqa: BLE001  (a one-frame call carries none)
            return t, None
    return t, None


out = {"share": f"rank {RANK} of {N}", "reps": R, "kernel": None, "frames": list(FS)}
for variant in ("ev", "noev", "stream", "ext", "noev"):
    rows = {}
    for F in FS:
        wall, ev = [], []
        for _ in range(R):
            a, b = region(F, variant)
            wall.append(a * 1e6)
            if b is not None:
                ev.append(b * 1e6)
        rows[str(F)] = {"wall_us_med": round(st.median(wall), 2),
                        "wall_us_min": round(min(wall), 2)}
        if ev:
            rows[str(F)]["events_us_med"] = round(st.median(ev), 2)
    # least-squares line through the medians: wall = fixed + F * per_frame
    xs = list(FS)
    ys = [rows[str(F)]["wall_us_med"] for F in FS]
    mx, my = st.mean(xs), st.mean(ys)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    rows["fit"] = {"fixed_us": round(my - b * mx, 2), "per_frame_us": round(b, 3)}
    out[variant if variant not in out else variant + "_again"] = rows
out["kernel"] = pipe.last_launch_info()["kernel_name"]

# host/runtime floor: an empty region, and one tiny kernel + synchronize
x = torch.zeros(1, device="cuda")
emp, one = [], []
for _ in range(50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    emp.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x.fill_(1.0)
    torch.cuda.synchronize()
    one.append((time.perf_counter() - t0) * 1e6)
out["empty_region_us_med"] = round(st.median(emp), 2)
out["tiny_kernel_region_us_med"] = round(st.median(one), 2)
print(json.dumps(out))
pipe.close()
