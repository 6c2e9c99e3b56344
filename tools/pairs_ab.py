"""Interleaved A/B of rt_set_frame_pairs modes on one GPU (diagnostic): rank 0's stripe share
of K3 (1920x1080, 500 spheres) at the given world sizes, one rt_update_frames call of F frames
per measurement (frame chains: fused launches; images 'every' as bench.py's chain shares, or
'last_two' as K4), the modes alternating call by call; prints each (world, mode)'s median and
quartiles of HIP-event µs per frame and the instance that ran.
usage: python tools/pairs_ab.py [reps] [worlds, e.g. 1,2,4] [modes, e.g. on,on2] [F] [images]"""
import json
import statistics as st
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
worlds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1").split(",")]
modes = (sys.argv[3] if len(sys.argv) > 3 else "on,on2").split(",")
F = int(sys.argv[4]) if len(sys.argv) > 4 else 20
images = sys.argv[5] if len(sys.argv) > 5 else "every"
w, h = 1920, 1080
sc = rt.SphereCollection.generate(rt.SCENE_N, 500, 1)
seeds = rt.frame_seeds(0x5EED, 5 + F)
cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=100000),
                                   w, h, float(seeds[0]))
cam_t = cam.with_fields(camera_has_moved=0.0)
pipe = rt.ComputeShaderPipeline(0)
pipe.set_spheres(sc)
pipe.set_frame_images(images)
for world in worlds:
    r = StripeRenderer(pipe, w, h, 0, world)
    for m in modes:          # tile costs recorded and the order built for each mode's units
        pipe.set_frame_pairs(m)
        r.frames(cam, sc, seeds[:5])
        for _ in range(3):
            r.frames(cam_t, sc, seeds[5:5 + F])
    torch.cuda.synchronize()
    res, kern = {m: [] for m in modes}, {}
    for _ in range(reps):
        for m in modes:
            pipe.set_frame_pairs(m)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            r.frames(cam_t, sc, seeds[5:5 + F])
            e1.record()
            torch.cuda.synchronize()
            res[m].append(e0.elapsed_time(e1) * 1e3 / F)
            kern[m] = pipe.last_launch_info()["kernel_name"]
    for m in modes:
        v = sorted(res[m])
        print(json.dumps({"world": world, "mode": m, "kernel": kern[m], "frames": F,
                          "images": images, "us_per_frame_q1_med_q3":
                          [round(v[len(v) // 4], 2), round(st.median(v), 2),
                           round(v[(3 * len(v)) // 4], 2)]}), flush=True)
    pipe.set_frame_pairs("auto")
pipe.close()
