"""One rank's timed region at N ranks, replayed on one GPU (diagnostic): rank `rank`'s stripe
share of K3 (1920x1080, 500 spheres) as bench.py --gpus N times it — frame chains (fused
launches writing every frame's image), a reset + 5 frames, then 20 timed frames in one
rt_update_frames call — repeated R times.  Prints one JSON line: wall and HIP-event µs per
step (median and quartiles), and, for the last repetition, `timeline_host` stamps
(CLOCK_MONOTONIC / CLOCK_BOOTTIME ns at the call, its return and the closing synchronize)
so that tools/timeline.py can place the call on a rocprofv3 kernel trace of this process:
    rocprofv3 --kernel-trace -f csv -d DIR -- python3 tools/share_region.py 8 0 > line.json
    python tools/timeline.py DIR line.json
usage: python tools/share_region.py [N] [rank] [R] [frames] [pairs: auto|on|quad|on2|quad2|off]
(SHARE_CFG=K2: bench.py's K2 scene instead, three spheres)"""
import os
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
F = int(sys.argv[4]) if len(sys.argv) > 4 else 20
PAIRS = sys.argv[5] if len(sys.argv) > 5 else "auto"
w, h = 1920, 1080
CFG = os.environ.get("SHARE_CFG", "K3")
sc = (rt.SphereCollection.generate(rt.SCENE_THREE, 3, 1) if CFG == "K2" else
      rt.SphereCollection.generate(rt.SCENE_N, 500, 1))
seeds = rt.frame_seeds(0x5EED, 5 + F)
cam0 = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=65536),
                                    w, h, float(seeds[0]))
cam_t = cam0.with_fields(camera_has_moved=0.0)
pipe = rt.ComputeShaderPipeline(0)
pipe.set_spheres(sc)
pipe.set_frames_per_launch(0)
pipe.set_frame_images("every")
pipe.set_frame_pairs(PAIRS)
stream = torch.cuda.current_stream()
r = StripeRenderer(pipe, w, h, RANK, N)
scratch = StripeRenderer(pipe, w, h, RANK, N)
torch.cuda.synchronize()
t_w = time.perf_counter()
while time.perf_counter() - t_w < 0.05:                      # bench.py's --warm-ms 50
    scratch.frames(cam0, sc, seeds[:F])
    torch.cuda.synchronize()
wall, ev = [], []
clk = lambda: (time.clock_gettime_ns(time.CLOCK_MONOTONIC),   # noqa: E731
               time.clock_gettime_ns(time.CLOCK_BOOTTIME))
stamps = {}
for rep in range(R + 1):
    r.frames(cam0, sc, seeds[:5])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    stamps["t0"] = clk()
    t0 = time.perf_counter()
    e0.record(stream)
    r.frames(cam_t, sc, seeds[5:5 + F])
    stamps["issued"] = clk()
    e1.record(stream)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    stamps["synced"] = clk()
    if rep:
        wall.append((t2 - t0) / F * 1e6)
        ev.append(e0.elapsed_time(e1) / F * 1e3)
info = pipe.last_launch_info()


def q(v):
    s = sorted(v)
    return [round(s[len(s) // 4], 2), round(st.median(s), 2), round(s[(3 * len(s)) // 4], 2)]


print(json.dumps({"config": CFG, "share": f"rank {RANK} of {N}", "steps": F, "reps": R, "pairs": PAIRS,
                  "kernel": info["kernel_name"], "launches": info["launches"],
                  "wall_us_per_step_q1_med_q3": q(wall), "events_us_per_step_q1_med_q3": q(ev),
                  "ms_per_step": round(st.median(wall) / 1e3, 5),
                  "roofline": {"kernel_avg_us": round(st.median(ev), 2)},
                  "timeline_host": stamps}))
pipe.close()
