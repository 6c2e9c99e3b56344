"""K5 8-rank share schedules (diagnostic): every rank's share of bench.py --config K5's step
(round-robin bands, one 64-frame bounce launch from a reset) under several path schedules —
per wave, pairs, and the split unit order at S chunks and threshold alpha (RT_BOUNCE_SPLIT,
RT_SPLIT_ALPHA, read by the library at every launch) — two untimed steps (costs, order), then
the median of three timed ones, wall-clock; the job's step is the slowest rank's.  Two
interleaved passes; the first pass's shares are checked band by band against the fixture.
usage: python tools/k5_share_sweep.py [world]"""
import json
import os
import statistics as st
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from conftest import bands_match  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

WORLD = int(sys.argv[1]) if len(sys.argv) > 1 else 8
g = dict(np.load(ROOT / "tests" / "golden" / "k5.npz"))
w, h = int(g["width"]), int(g["height"])
cam, sc, seeds = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]), g["seeds"]
CONFIGS = [("auto", "auto", {}), ("per_wave", "per_wave", {}), ("pair", "pair", {}),
           ("S2", "auto", {"RT_BOUNCE_SPLIT": "2"}), ("S8", "auto", {"RT_BOUNCE_SPLIT": "8"}),
           ("a0.125", "auto", {"RT_SPLIT_ALPHA": "0.125"}),
           ("a0.5", "auto", {"RT_SPLIT_ALPHA": "0.5"}),
           ("S8a0.125", "auto", {"RT_BOUNCE_SPLIT": "8", "RT_SPLIT_ALPHA": "0.125"})]
KNOBS = ("RT_BOUNCE_SPLIT", "RT_SPLIT_ALPHA")
pipe = rt.ComputeShaderPipeline(0)
pipe.set_frames_per_launch(0)
pipe.set_frame_images("last_two")


def share(rank, check):
    r = StripeRenderer(pipe, w, h, rank, WORLD)
    r.frames(cam, sc, seeds)
    r.frames(cam, sc, seeds)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.frames(cam, sc, seeds)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    ok = None
    if check:
        ok = bands_match(r.local.cpu().numpy(), r.band_list(), g["band_sha"]) == []
    return st.median(ts), pipe.last_launch_info()["kernel_name"], ok


res = {c[0]: [] for c in CONFIGS}
for pas in range(2):
    for name, mode, env in CONFIGS:
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(env)
        pipe.set_path_compaction(mode)
        per = [share(rk, pas == 0) for rk in range(WORLD)]
        us = [p[0] for p in per]
        row = {"pass": pas, "config": name, "max_us": round(max(us), 1),
               "rank_us": [round(x, 1) for x in us], "kernel": per[0][1],
               "ok": all(p[2] for p in per) if pas == 0 else None}
        res[name].append(row)
        print(json.dumps(row), flush=True)
print(json.dumps({"summary": {k: [r["max_us"] for r in v] for k, v in res.items()}}))
pipe.close()
