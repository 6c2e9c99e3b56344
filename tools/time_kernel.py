"""Time the trace kernel for one library build (RT_HIP_LIB) on a config; check the K3/K2
golden hash.  Used by tools/ab_variants.py for interleaved A/B runs."""
import hashlib, json, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np, torch
import gpu_ray_tracing as rt

def main(cfg="k3", iters=40):
    g = dict(np.load(ROOT / "tests" / "golden" / f"{cfg}.npz"))
    w, h = int(g["width"]), int(g["height"])
    cam = rt.SceneCamera(g["camera"]); sc = rt.SphereCollection(g["spheres"])
    pipe = rt.ComputeShaderPipeline(0)
    import os
    pipe.set_scan_mode(os.environ.get('RT_SCAN_MODE', 'culled'))
    if hasattr(pipe, "set_tile_order") and hasattr(rt._lib.lib(), "rt_set_tile_order"):
        pipe.set_tile_order(os.environ.get("RT_TILE_ORDER", "auto"))
    if hasattr(rt._lib.lib(), "rt_set_single_kernel"):
        pipe.set_single_kernel(os.environ.get("RT_SINGLE", "auto"))
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.update(a, b, w, h, cam, sc); torch.cuda.synchronize()
    ok = hashlib.sha256(b.cpu().numpy().tobytes()).hexdigest() == str(g["sha256"]) if "sha256" in g else None
    a, b = b, a  # continue from the reset frame (its sample count is known to the library)
    c2 = cam.with_fields(camera_has_moved=0.0, samples_per_pixel=1e6)
    st = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for k in range(iters):
        evs[k][0].record(st); pipe.update(a, b, w, h, c2, sc); evs[k][1].record(st); a, b = b, a
    torch.cuda.synchronize()
    t = sorted(x.elapsed_time(y) * 1e3 for x, y in evs)
    # fused: rt_update_frames calls of 64 frames (frame groups when hinted), us per frame
    seeds = rt.frame_seeds(0x5EED, 64)
    fev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
    for k in range(6):
        fev[k][0].record(st)
        newest = pipe.update_frames(a, b, w, h, c2, sc, seeds)
        fev[k][1].record(st)
        if newest == 1: a, b = b, a
    torch.cuda.synchronize()
    ft = sorted(x.elapsed_time(y) * 1e3 / 64 for x, y in fev[1:])
    L = rt._lib.lib()
    stamps = None
    if hasattr(L, "rt_diag_stamps"):
        import ctypes
        buf = (ctypes.c_ulonglong * 8)()
        waves = ((w + 7) // 8) * ((h + 7) // 8)
        L.rt_diag_stamps(buf, ctypes.c_uint(waves))
        stamps = [round(buf[k] / waves, 1) for k in range(1, 8)]
    print(json.dumps({"cfg": cfg, "median_us": t[len(t) // 2], "min_us": t[0], "hash_ok": ok,
                      "fused_us": ft[len(ft) // 2],
                      "stamps_cycles_per_wave": stamps}))

if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["k3"]))
