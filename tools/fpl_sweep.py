"""Per-frame time of rt_update_frames at 1, 2, 4, 8, 16, 32, 64 frames per launch (K3 /
K2; diagnostic).  usage: python tools/fpl_sweep.py [k3|k2] [pairs: auto|off|on|quad]"""
import json, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np, torch
import gpu_ray_tracing as rt

def main(cfg="k3", pairs="auto"):
    g = dict(np.load(ROOT / "tests" / "golden" / f"{cfg}.npz"))
    w, h = int(g["width"]), int(g["height"])
    cam = rt.SceneCamera(g["camera"]); sc = rt.SphereCollection(g["spheres"])
    pipe = rt.ComputeShaderPipeline(0)
    pipe.set_frame_pairs(pairs)
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.update(a, b, w, h, cam, sc); torch.cuda.synchronize()
    a, b = b, a
    c2 = cam.with_fields(camera_has_moved=0.0, samples_per_pixel=1e7)
    st = torch.cuda.current_stream()
    seeds = rt.frame_seeds(0x5EED, 128)
    out = {"cfg": cfg, "pairs": pairs}
    for fpl in (1, 2, 4, 8, 16, 32, 64):
        pipe.set_frames_per_launch(fpl)
        res = []
        for rep in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            newest = pipe.update_frames(a, b, w, h, c2, sc, seeds)
            e1.record(st)
            if newest == 1: a, b = b, a
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / len(seeds))
        out[f"fpl{fpl}_us_per_frame"] = round(sorted(res)[1], 2)
    print(json.dumps(out), flush=True)

if __name__ == "__main__":
    main(*sys.argv[1:3])
