"""Per-phase wave timeline of ONE one-frame `update` launch (rt_single_kernel) for a whole
image and for rank shares (diagnostic; needs a library built with -DRT_SSTAMPS=1, passed as
RT_HIP_LIB).  For every wave the kernel stamps s_memtime when each phase's result is
available: entry -> order resolved -> seed tables + counts -> camera rays -> list walk ->
shading + sky -> accumulator consumed -> stores issued (rt_kernels.hip RT_SSTAMPS).  Prints,
per scenario, the mean / p90 duration of each phase (us at the stamped clock), the wave
lifetime, the launch span (s_memrealtime, per XCC), and the resident waves per SIMD.
Before each stamped launch the GPU is warmed with whole-image frames (RT_WARM_MS, default 50
ms first, 5 ms between launches; 0 = cold, as before round 3's warm-up).
usage: RT_HIP_LIB=... [RT_WARM_MS=50] python tools/stamps_single.py [K3|K2] [worlds, e.g. 1,8,135]"""
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402

CONF = {"K2": (1920, 1080, rt.SCENE_THREE, 3, 1), "K3": (1920, 1080, rt.SCENE_N, 500, 1)}
PHASES = ["order", "seeds+counts", "camera_ray", "list_walk", "shade+sky", "accumulate",
          "store_issue"]
NW = 1 << 17


def warm(pipe, cfg, cam, sc, seeds, ms):
    """Untimed whole-image update frames for `ms` milliseconds (bench.py --warm-ms): the
    stamped launch then runs at the clock a running render holds."""
    w, h, *_ = CONF[cfg]
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < ms / 1e3:
        pipe.update_frames(a, b, w, h, cam, sc, seeds[:20])
        torch.cuda.synchronize()


def scenario(pipe, L, buf, cfg, world, cam, sc, seeds, repeat=5):
    w, h, *_ = CONF[cfg]
    warm_ms = float(os.environ.get("RT_WARM_MS", "50"))
    rows = rt.stripe_local_rows(h, 0, world)
    a, b = pipe.new_image(w, rows), pipe.new_image(w, rows)
    pipe.set_frames_per_launch(1)
    pipe.update_frames(a, b, w, h, cam, sc, seeds[:4], 0, world)     # reset + warm + order
    c2 = cam.with_fields(camera_has_moved=0.0)
    pipe.update_frames(a, b, w, h, c2, sc, seeds[4:12], 0, world)
    out = []
    for r in range(repeat):
        if warm_ms > 0:
            warm(pipe, cfg, cam, sc, seeds, warm_ms if r == 0 else 5.0)
        torch.cuda.synchronize()
        assert L.rt_diag_single_stamps(buf, NW) == 0                 # clear
        pipe.update_frames(a, b, w, h, c2, sc, seeds[12 + r:13 + r], 0, world)
        torch.cuda.synchronize()
        assert L.rt_diag_single_stamps(buf, NW) == 0
        info = pipe.last_launch_info()
        s = np.frombuffer(bytes(buf), np.uint64).reshape(NW, 12).astype(np.int64)
        s = s[s[:, 9] > 0]                                        # waves that ran to the end
        t = s[:, :8]
        rt0, rt1 = s[:, 8].copy(), s[:, 9].copy()
        xcc = s[:, 11] & 0xF
        for x in np.unique(xcc):                                  # (clocks are per XCC)
            m = xcc == x
            base = rt0[m].min()
            rt0[m] -= base
            rt1[m] -= base
        span = float(rt1.max()) / 100.0                          # us (100 MHz)
        life_cyc = (t[:, 7] - t[:, 0]).astype(np.float64)
        life_us = (rt1 - rt0) / 100.0
        clk = float(np.median(life_cyc / np.maximum(life_us, 1e-3))) / 1e3   # GHz
        d = {"cfg": cfg, "world": world, "kernel": info["kernel_name"], "waves": int(len(s)),
             "span_us": round(span, 2), "clock_ghz": round(clk, 3),
             "mean_life_us": round(float(life_us.mean()), 3),
             "p90_life_us": round(float(np.percentile(life_us, 90)), 3),
             "last_start_frac": round(float(rt0.max()) / 100.0 / span, 3),
             "resident_waves_per_simd": round(float((rt1 - rt0).sum()) / 100.0 / span / 1024, 2)}
        for i, name in enumerate(PHASES):
            dt = (t[:, i + 1] - t[:, i]) / (clk * 1e3)
            d[name] = [round(float(dt.mean()), 3), round(float(np.percentile(dt, 90)), 3)]
        out.append(d)
    # the median launch by span
    out.sort(key=lambda d: d["span_us"])
    return out[len(out) // 2]


def main(cfg="K3", worlds="1,2,4,8,135"):
    w, h, kind, n, depth = CONF[cfg]
    sc = rt.SphereCollection.generate(kind, n, 1)
    seeds = rt.frame_seeds(0x5EED, 32)
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=depth, samples_per_pixel=1000),
                                       w, h, float(seeds[0]))
    pipe = rt.ComputeShaderPipeline(0)
    pipe.set_spheres(sc)
    # one launch per update: the stamps are indexed by the wave's place in its launch, and
    # concurrent parts (rt_set_update_queues) would overwrite each other's
    pipe.set_update_queues(1)
    L = rt._lib.lib()
    L.rt_diag_single_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    buf = (ctypes.c_ulonglong * (12 * NW))()
    for world in (int(x) for x in worlds.split(",")):
        print(json.dumps(scenario(pipe, L, buf, cfg, world, cam, sc, seeds)), flush=True)
    pipe.close()


if __name__ == "__main__":
    main(*sys.argv[1:3])
