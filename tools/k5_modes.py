"""K5 (3840x2160, 500 spheres, depth 8): one 64-spp rt_update_frames call per launch mode
(bounce paths per wave / compacted), timed with HIP events and checked against k5.npz's
sampled pixels (diagnostic).  usage: python tools/k5_modes.py [per_wave compact ...]"""
import json, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np, torch
import gpu_ray_tracing as rt

g = dict(np.load(ROOT / "tests" / "golden" / "k5.npz"))
w, h = int(g["width"]), int(g["height"])
cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
for mode in (sys.argv[1:] or ["auto", "per_wave", "pair", "compact"]):
    p = rt.ComputeShaderPipeline(0)
    p.set_path_compaction(mode)
    a, b = p.new_image(w, h), p.new_image(w, h)
    for k in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        nw = p.update_frames(a, b, w, h, cam, sc, g["seeds"])
        e1.record()
        torch.cuda.synchronize()
        img = (b if nw == 1 else a).cpu().numpy()
        ok = bool((img[g["py"], g["px"]].view(np.uint32) == g["pixels"].view(np.uint32)).all())
        print(json.dumps({"paths": mode, "launch": k, "ms_per_64spp": round(e0.elapsed_time(e1), 2),
                          "ok": ok, "info": p.last_launch_info()}), flush=True)
    p.close()
