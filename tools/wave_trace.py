"""Wave-level timeline of one fused launch of rank 0's stripe share (diagnostic; needs a
library built with -DRT_WAVE_TRACE=1, passed as RT_HIP_LIB).  Prints, for world sizes
1/2/4/8: the launch span, the spread of per-SIMD finishing times and of wave durations,
and the mean number of waves resident per SIMD over the span — i.e. how much of the
strong-scaling loss is tail imbalance.  usage: RT_HIP_LIB=... python tools/wave_trace.py [K3]"""
import ctypes
import json
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

import os
DEBUG = os.environ.get("WT_DEBUG") == "1"
NF = int(os.environ.get("WT_FRAMES", "64"))      # frames of the traced launch (bench.py's K3: 20)
CONF = {"K2": (1920, 1080, rt.SCENE_THREE, 3, 1), "K3": (1920, 1080, rt.SCENE_N, 500, 1),
        "K5": (3840, 2160, rt.SCENE_N, 500, 8)}


def analyse(raw, nwaves):
    """Times are per XCD (each XCD's s_memtime counter has its own origin)."""
    a = np.frombuffer(raw, np.uint64).reshape(-1, 4)[:nwaves].astype(np.int64)
    a = a[a[:, 1] > 0]
    if DEBUG:
        for x in np.unique(a[:, 3]):
            m = a[:, 3] == x
            print("xcc_raw", hex(int(x)), int(m.sum()), "start range", int(a[m, 0].min()),
                  int(a[m, 0].max()), "end max", int(a[m, 1].max()), flush=True)
    xcc = a[:, 3] & 0xF
    start = a[:, 0].copy()
    end = a[:, 1].copy()
    for x in np.unique(xcc):
        m = xcc == x
        t0 = start[m].min()
        start[m] -= t0
        end[m] -= t0
    span = end.max()
    simd = defaultdict(list)
    for s, e, hw, x in zip(start, end, a[:, 2], xcc):
        simd[(int(x), (int(hw) >> 4) & 0x7FF)].append((s, e))
    last = np.array([max(e for _, e in v) for v in simd.values()])
    first = np.array([min(s for s, _ in v) for v in simd.values()])
    resident = sum(e - s for s, e in zip(start, end)) / (len(simd) * span)
    dur = end - start
    pct = lambda v, q: float(np.percentile(v, q))
    xspan = [int(end[xcc == x].max()) for x in np.unique(xcc)]
    top = np.sort(dur)[::-1][:8]
    return {"waves": int(len(a)), "simds": len(simd), "span_cycles": int(span),
            "longest_waves_frac": [round(float(v) / span, 3) for v in top],
            "simd_resident_waves_p10_p50_p90": [round(pct(np.array([sum(e - s for s, e in v) for v in simd.values()]), q) / span, 3) for q in (10, 50, 90)],
            "xcd_span_min_max": [round(min(xspan) / span, 3), 1.0],
            "simd_first_start_max": round(float(first.max()) / span, 3),
            "simd_last_end_p10_p50_p90_max": [round(pct(last, q) / span, 3) for q in (10, 50, 90, 100)],
            "wave_dur_p10_p50_p90_max": [round(pct(dur, q) / span, 3) for q in (10, 50, 90, 100)],
            "mean_resident_waves_per_simd": round(resident, 2)}


def main(cfg="K3"):
    w, h, kind, n, depth = CONF[cfg]
    sc = rt.SphereCollection.generate(kind, n, 1)
    seeds = rt.frame_seeds(0x5EED, 140)
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=depth, samples_per_pixel=1000),
                                       w, h, float(seeds[0]))
    pipe = rt.ComputeShaderPipeline(0)
    pipe.set_spheres(sc)
    pipe.set_path_compaction(os.environ.get("RT_PATHS", "auto"))
    L = rt._lib.lib()
    L.rt_diag_wave_trace.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    buf = (ctypes.c_ulonglong * (4 * (1 << 18)))()
    worlds = [int(x) for x in os.environ["WT_WORLDS"].split(",")] if "WT_WORLDS" in os.environ else \
        ((2, 4, 8) if cfg == "K5" else (1, 2, 4, 8))
    for world in worlds:   # (K5 at 1 rank: > 2^16 WGs)
        r = StripeRenderer(pipe, w, h, 0, world)
        r.frames(cam, sc, seeds[:5])                       # reset + tile-cost recording
        r.frames(cam.with_fields(camera_has_moved=0.0), sc, seeds[69:133])  # long recording
        torch.cuda.synchronize()
        assert L.rt_diag_wave_trace(buf, 1 << 18) == 0     # (clears the trace)
        r.frames(cam.with_fields(camera_has_moved=0.0), sc, seeds[5:5 + NF])  # one NF-frame launch
        torch.cuda.synchronize()
        assert L.rt_diag_wave_trace(buf, 1 << 18) == 0
        raw = bytes(buf)
        if os.environ.get("WT_SAVE"):
            np.save(f"{os.environ['WT_SAVE']}_w{world}.npy",
                    np.frombuffer(raw, np.uint64).reshape(-1, 4))
        d = analyse(raw, 1 << 18)
        d.update(cfg=cfg, world=world, paths=os.environ.get("RT_PATHS", "auto"))
        print(json.dumps(d), flush=True)
    pipe.close()


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["K3"]))
