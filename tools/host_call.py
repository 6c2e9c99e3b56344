"""Host cost of one rt_update_frames call (diagnostic): the Python wrapper
(ComputeShaderPipeline.update_frames), the bound call (bind_update_frames, what
StripeRenderer.frames issues) and the bare ctypes call with its arguments built
once, per K3 rank share and launch structure; the GPU is idle at each call (synchronised
before), so the wall time is what the call costs the host before the stream runs.
usage: python tools/host_call.py [frames]"""
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing import _lib  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 20
w, h = 1920, 1080
sc = rt.SphereCollection.generate(rt.SCENE_N, 500, 1)
seeds = rt.frame_seeds(0x5EED, 200)
cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=65536),
                                   w, h, float(seeds[0]))
cam_t = cam.with_fields(camera_has_moved=0.0)
pipe = rt.ComputeShaderPipeline(0)
pipe.set_spheres(sc)
for mode in ("dispatch", "chain"):
    pipe.set_frames_per_launch(1 if mode == "dispatch" else 0)
    pipe.set_frame_images("every" if mode == "chain" else "last_two")
    for world in (1, 8):
        rows = rt.stripe_local_rows(h, 0, world)
        a, b = pipe.new_image(w, rows), pipe.new_image(w, rows)
        pipe.update_frames(a, b, w, h, cam, sc, seeds[:frames], 0, world)
        for _ in range(3):
            pipe.update_frames(a, b, w, h, cam_t, sc, seeds[:frames], 0, world)
        torch.cuda.synchronize()
        py = []
        for k in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipe.update_frames(a, b, w, h, cam_t, sc, seeds[:frames], 0, world)
            py.append((time.perf_counter() - t0) * 1e6)
        # the bound call (bind_update_frames: what StripeRenderer.frames issues)
        run = pipe.bind_update_frames(a, b, w, h, 0, world)
        bound = []
        for k in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(cam_t, sc, seeds[:frames])
            bound.append((time.perf_counter() - t0) * 1e6)
        # the bare C call, arguments built once
        c_cam = cam_t.to_c()
        p, n = pipe._spheres(sc)
        s = np.ascontiguousarray(seeds[:frames], np.float32)
        newest = ctypes.c_int(-1)
        fn = _lib.lib().rt_update_frames
        args = (pipe._ctx, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), w, h,
                0, world, ctypes.byref(c_cam), p, n, s.size, s.ctypes.data_as(ctypes.c_void_p),
                pipe._stream(), ctypes.byref(newest))
        cc = []
        for k in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            assert fn(*args) == 0
            cc.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
        print(json.dumps({"mode": mode, "world": world, "frames": frames,
                          "python_call_us": round(sorted(py)[15], 2),
                          "bound_call_us": round(sorted(bound)[15], 2),
                          "c_call_us": round(sorted(cc)[15], 2),
                          "launches": pipe.last_launch_info()["launches"]}), flush=True)
pipe.close()
