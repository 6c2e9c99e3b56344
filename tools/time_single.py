"""Single-frame update time (median of 40) for one library build (RT_HIP_LIB); no hash check
(diagnostic builds may compute other images).  usage: python tools/time_single.py k3"""
import json, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np, torch
import gpu_ray_tracing as rt
cfg = sys.argv[1] if len(sys.argv) > 1 else "k3"
g = dict(np.load(ROOT / "tests" / "golden" / f"{cfg}.npz"))
w, h = int(g["width"]), int(g["height"])
cam = rt.SceneCamera(g["camera"]); sc = rt.SphereCollection(g["spheres"])
pipe = rt.ComputeShaderPipeline(0)
a, b = pipe.new_image(w, h), pipe.new_image(w, h)
pipe.update(a, b, w, h, cam, sc); torch.cuda.synchronize(); a, b = b, a
c2 = cam.with_fields(camera_has_moved=0.0, samples_per_pixel=1e7)
st = torch.cuda.current_stream()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
for k in range(40):
    evs[k][0].record(st); pipe.update(a, b, w, h, c2, sc); evs[k][1].record(st); a, b = b, a
torch.cuda.synchronize()
t = sorted(x.elapsed_time(y) * 1e3 for x, y in evs)
print(json.dumps({"cfg": cfg, "lib": Path(__import__("os").environ.get("RT_HIP_LIB", "default")).name, "median_us": round(t[20], 2), "min_us": round(t[0], 2)}))
