"""Where a K5 step's bounce work goes (diagnostic; needs a library built with
-DRT_BOUNCE_COUNTS=1, passed as RT_HIP_LIB): one 64-spp 3840x2160 depth-8 step (the K5
fixture, one 64-frame bounce launch from a reset) with the bounce instance's region counters
— per region the wave-level trips and the active lanes summed over them — printed per wave
and frame and as lane occupancy.  usage: RT_HIP_LIB=... python tools/bounce_counts.py [world]"""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

REGIONS = {0: "grid walk (fast roots)", 14: "grid walk (IEEE roots)", 2: "grid DDA step",
           4: "grid cell item", 6: "camera segment", 8: "bounce segment", 10: "scatter",
           12: "frame (hinted)", 16: "frame (not hinted)",
           18: "bounce exhaustive scan", 20: "camera exhaustive scan", 22: "bounce cone scan",
           24: "camera cone scan", 26: "grid-usable waves (incl. far lanes)"}
world = int(sys.argv[1]) if len(sys.argv) > 1 else 1
g = dict(np.load(ROOT / "tests" / "golden" / "k5.npz"))
w, h = int(g["width"]), int(g["height"])
cam, sc, seeds = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]), g["seeds"]
pipe = rt.ComputeShaderPipeline(0)
pipe.set_frames_per_launch(0)
pipe.set_frame_images("last_two")
L = rt._lib.lib()
L.rt_diag_bounce_counts.argtypes = [ctypes.c_void_p, ctypes.c_uint]
buf = (ctypes.c_ulonglong * 32)()
r = StripeRenderer(pipe, w, h, 0, world)
r.frames(cam, sc, seeds)
torch.cuda.synchronize()
assert L.rt_diag_bounce_counts(buf, 32) == 0          # (clears)
r.frames(cam, sc, seeds)
torch.cuda.synchronize()
assert L.rt_diag_bounce_counts(buf, 32) == 0
c = list(buf)
frames = c[12] + c[16]
out = {"world": world, "kernel": pipe.last_launch_info()["kernel_name"], "wave_frames": frames}
for k, name in REGIONS.items():
    trips, lanes = c[k], c[k + 1]
    out[name] = {"trips": trips, "per_wave_frame": round(trips / max(frames, 1), 3),
                 "lanes_per_trip": round(lanes / max(trips, 1), 2)}
print(json.dumps(out))
pipe.close()
