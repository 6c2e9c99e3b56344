"""Interleaved A/B of bounce path schedules on K5 rank shares (diagnostic): for each world
size, rank 0's share of the 3840x2160 depth-8 64-spp render, one 64-frame launch per
measurement, the modes alternating launch by launch (so clock and power drift hits every
mode alike); reports each mode's median and min us per step.
usage: python tools/k5_ab.py [reps] [worlds, e.g. 4,8] [modes, e.g. per_wave,split4,split2f25]
(split<S>f<P>: S chunks for the costliest P % of the tiles; split<S>a<P>: the unit order
with alpha = P / 100)"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
worlds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4,8").split(",")]
modes = (sys.argv[3] if len(sys.argv) > 3 else "per_wave,split2,split4").split(",")
g = dict(np.load(ROOT / "tests" / "golden" / "k5.npz"))
w, h = int(g["width"]), int(g["height"])
cam, sc, seeds = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]), g["seeds"]
pipe = rt.ComputeShaderPipeline(0)
pipe.set_spheres(sc)


def set_mode(m):
    # split<S>[f<P> | a<P>]: S chunks for the costliest P % of the tiles of the tile order
    # (f), or the unit order with alpha = P / 100 (a; default: the library's alpha)
    os.environ.pop("RT_SPLIT_FRAC", None)
    os.environ.pop("RT_SPLIT_ALPHA", None)
    if m.startswith("split"):
        rest = m[5:]
        key = "f" if "f" in rest else "a" if "a" in rest else None
        s, _, f = rest.partition(key) if key else (rest, "", "")
        os.environ["RT_BOUNCE_SPLIT"] = s or "4"
        if key:
            os.environ["RT_SPLIT_FRAC" if key == "f" else "RT_SPLIT_ALPHA"] = str(int(f) / 100)
        pipe.set_path_compaction("split")
    else:
        os.environ.pop("RT_BOUNCE_SPLIT", None)
        pipe.set_path_compaction(m)


# warm: two whole-image steps
warm = StripeRenderer(pipe, w, h, 0, 1)
for _ in range(2):
    warm.frames(cam, sc, seeds)
torch.cuda.synchronize()
del warm
for world in worlds:
    r = StripeRenderer(pipe, w, h, 0, world)
    for m in modes:                     # costs recorded, order built, buffers allocated
        set_mode(m)
        r.frames(cam, sc, seeds)
        r.frames(cam, sc, seeds)
    torch.cuda.synchronize()
    res = {m: [] for m in modes}
    for rep in range(reps):
        for m in modes:
            set_mode(m)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.frames(cam, sc, seeds)
            e1.record()
            torch.cuda.synchronize()
            res[m].append(e0.elapsed_time(e1) * 1e3)
    for m in modes:
        v = sorted(res[m])
        print(json.dumps({"world": world, "mode": m, "median_us": round(v[len(v) // 2], 1),
                          "min_us": round(v[0], 1), "us_per_spp_median": round(v[len(v) // 2] / 64, 2),
                          "kernel": None, "runs": [round(x, 1) for x in res[m]]}), flush=True)
pipe.close()
