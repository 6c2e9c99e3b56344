"""Quick GPU probe: time rt_update / rt_render on the bench configs with HIP events."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np, torch
import gpu_ray_tracing as rt

def run(name, w, h, scene, depth, frames_fused=1, iters=20):
    pipe = rt.ComputeShaderPipeline(0)
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=depth, samples_per_pixel=100000), w, h, 0.5)
    a = pipe.new_image(w, h); b = pipe.new_image(w, h)
    seeds = rt.frame_seeds(0x5EED, max(frames_fused, iters + 3))
    # warmup
    for i in range(3):
        pipe.update(a, b, w, h, cam.with_fields(random_seed=float(seeds[i]), camera_has_moved=0.0), scene); a, b = b, a
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    if frames_fused == 1:
        for i in range(iters):
            pipe.update(a, b, w, h, cam.with_fields(random_seed=float(seeds[i]), camera_has_moved=0.0), scene); a, b = b, a
        nsamp = iters
    else:
        pipe.render(a, a, w, h, cam.with_fields(camera_has_moved=0.0), scene, seeds[:frames_fused])
        nsamp = frames_fused
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    rays = w * h * nsamp
    print(f"{name}: {ms/nsamp*1e3:.1f} us/frame  {rays/ms/1e3:.1f} Mrays/s  "
          f"({scene.count} spheres, depth {depth}, fused {frames_fused})", flush=True)
    pipe.close()

three = rt.three_spheres(); n500 = rt.synthetic_scene(500)
run("K2", 1920, 1080, three, 1)
run("K3", 1920, 1080, n500, 1)
run("K3-fused64", 1920, 1080, n500, 1, frames_fused=64)
run("K2-fused64", 1920, 1080, three, 1, frames_fused=64)
run("default-d8", 1920, 1080, rt.create_default_spheres(1), 8, iters=5)
