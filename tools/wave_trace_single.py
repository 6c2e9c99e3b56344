"""Wave-level timeline of ONE single-frame `update` launch (rt_update; the reference's
dispatch structure) on the whole image (diagnostic; needs a library built with
-DRT_WAVE_TRACE=1, passed as RT_HIP_LIB).  Prints the launch span, the dispatch ramp
(when the last wave started), wave durations and mean resident waves per SIMD, plus a
start-time histogram.  usage: RT_HIP_LIB=... python tools/wave_trace_single.py [K3|K2]"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT), str(ROOT / "tools")]
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from wave_trace import CONF, analyse  # noqa: E402


def main(cfg="K3"):
    w, h, kind, n, depth = CONF[cfg]
    sc = rt.SphereCollection.generate(kind, n, 1)
    seeds = rt.frame_seeds(0x5EED, 64)
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=depth, samples_per_pixel=1000),
                                       w, h, float(seeds[0]))
    pipe = rt.ComputeShaderPipeline(0)
    pipe.set_spheres(sc)
    L = rt._lib.lib()
    L.rt_diag_wave_trace.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    buf = (ctypes.c_ulonglong * (4 * (1 << 18)))()
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.update(a, b, w, h, cam, sc)                       # reset frame
    a, b = b, a
    c2 = cam.with_fields(camera_has_moved=0.0)
    for k in range(1, 10):                                  # warm
        pipe.update(a, b, w, h, c2.with_fields(random_seed=float(seeds[k])), sc)
        a, b = b, a
    torch.cuda.synchronize()
    assert L.rt_diag_wave_trace(buf, 1 << 18) == 0
    pipe.update(a, b, w, h, c2.with_fields(random_seed=float(seeds[10])), sc)
    torch.cuda.synchronize()
    assert L.rt_diag_wave_trace(buf, 1 << 18) == 0
    raw = bytes(buf)
    nw = ((w + 7) // 8) * ((h + 7) // 8) * 4          # the trace index has 4 slots per WG
    d = analyse(raw, nw)
    a4 = np.frombuffer(raw, np.uint64).reshape(-1, 4)[:nw].astype(np.int64)
    a4 = a4[a4[:, 1] > 0]
    xcc = a4[:, 3] & 0xF
    st, en = a4[:, 0].copy(), a4[:, 1].copy()
    for x in np.unique(xcc):
        m = xcc == x
        t0 = st[m].min()
        st[m] -= t0
        en[m] -= t0
    span = en.max()
    d["span_us"] = round(float(span) / 100.0, 2)          # s_memrealtime: 100 MHz
    d["last_start_frac"] = round(float(st.max()) / span, 3)
    d["mean_wave_us"] = round(float((en - st).mean()) / 100.0, 3)
    d["start_hist_10"] = np.histogram(st, bins=10, range=(0, span))[0].tolist()
    d["end_hist_10"] = np.histogram(en, bins=10, range=(0, span))[0].tolist()
    d.update(cfg=cfg, mode="single-frame")
    print(json.dumps(d), flush=True)
    pipe.close()


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["K3"]))
