"""Host cost of one update_frames call (diagnostic): the Python wrapper + rt_update_frames
with zero frames (argument checks, scene / list / hash-table checks: everything a call pays
before its first launch), then per frame for 1 / 4 / 20 one-frame updates (the issuing
call's own time, no synchronisation inside).  K3 at 1920x1080, one rank and an 8-rank share.
usage: python tools/call_overhead.py"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402


def main():
    w, h = 1920, 1080
    sc = rt.SphereCollection.generate(rt.SCENE_N, 500, 1)
    seeds = rt.frame_seeds(0x5EED, 4000)
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=100000),
                                       w, h, float(seeds[0]))
    cam_t = cam.with_fields(camera_has_moved=0.0)
    pipe = rt.ComputeShaderPipeline(0)
    pipe.set_spheres(sc)
    pipe.set_frames_per_launch(1)
    for world in (1, 8):
        rows = rt.stripe_local_rows(h, 0, world)
        a, b = pipe.new_image(w, rows), pipe.new_image(w, rows)
        pipe.update_frames(a, b, w, h, cam, sc, seeds[:8], 0, world)
        pipe.update_frames(a, b, w, h, cam_t, sc, seeds[8:16], 0, world)
        torch.cuda.synchronize()
        out = {"world": world}
        f = 16
        for n in (0, 1, 4, 20):
            ts = []
            for _ in range(30):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pipe.update_frames(a, b, w, h, cam_t, sc, seeds[f:f + n], 0, world)
                ts.append(time.perf_counter() - t0)
                f += n
            ts.sort()
            out[f"call_us_{n}_frames_median"] = round(ts[len(ts) // 2] * 1e6, 2)
        out["queues"] = pipe.last_launch_info().get("queues")
        print(json.dumps(out), flush=True)
    pipe.close()


if __name__ == "__main__":
    main()
