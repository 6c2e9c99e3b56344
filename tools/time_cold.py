"""Cold-camera update time (median of 30) for one library build (RT_HIP_LIB): every update
gets a new camera, so the candidate lists are rebuilt each time (rt_candidates_kernel +
one update).  usage: python tools/time_cold.py k3"""
import json, math, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np, torch
import gpu_ray_tracing as rt
cfg = sys.argv[1] if len(sys.argv) > 1 else "k3"
g = dict(np.load(ROOT / "tests" / "golden" / f"{cfg}.npz"))
w, h = int(g["width"]), int(g["height"])
sc = rt.SphereCollection(g["spheres"])
pipe = rt.ComputeShaderPipeline(0)
a, b = pipe.new_image(w, h), pipe.new_image(w, h)
cams = []
for f in range(40):
    ang = math.radians(0.05 * (f + 1))
    st = rt.CameraSettings(max_depth=1, samples_per_pixel=65536,
                           look_from=(13.0 * math.cos(ang) - 3.0 * math.sin(ang), 2.0,
                                      13.0 * math.sin(ang) + 3.0 * math.cos(ang)))
    cams.append(rt.SceneCamera.from_settings(st, w, h, 0.25 + f / 64))
st = torch.cuda.current_stream()
for c in cams[:5]:
    pipe.update(a, b, w, h, c, sc); a, b = b, a
torch.cuda.synchronize()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in cams[5:]]
for (e0, e1), c in zip(evs, cams[5:]):
    e0.record(st); pipe.update(a, b, w, h, c, sc); e1.record(st); a, b = b, a
torch.cuda.synchronize()
t = sorted(x.elapsed_time(y) * 1e3 for x, y in evs)
print(json.dumps({"cfg": cfg, "lib": Path(os.environ.get("RT_HIP_LIB", "default")).name,
                  "cold_median_us": round(t[len(t) // 2], 2), "min_us": round(t[0], 2)}))
