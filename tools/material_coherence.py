"""How much would material-coherent shading save in the one-frame kernel? (CPU, no GPU.)

rt_single_kernel<2> gives each lane two pixels — the same position in two horizontally
adjacent 8x8 tiles (rt_kernels.hip tile_coord, single_body) — and shades each pixel slot in
turn (shade_hit): the Lambertian arithmetic on every lane, then the metal and / or dielectric
branch (wgsl:95-135) for the whole wave whenever any lane of that slot hit such a sphere.
Three ways to run those branches over a wave's 128 pixels, counted in branch passes per
wave (a pass = one execution of the metal or the dielectric code by the wave):
  now       per slot, a pass of each material present in the slot;
  merged    each lane takes its first pending slot, then its second (passes = the most
            pending slots of any lane), plus a per-lane select of the inputs and results;
  compacted the wave's pixels of each material packed into consecutive lanes with
            ballot / mbcnt (north_star's compaction): ceil(count / 64) passes per material.
Hits are taken at pixel centres (no sub-pixel jitter or defocus): per-sample hits differ
only at sphere edges, which changes these fractions by little.  K3: 1920x1080, 500 spheres
(SCENE_N, seed 1).  Prints one JSON line.
usage: python tools/material_coherence.py [W H N_SPHERES]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import gpu_ray_tracing as rt  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
NS = int(sys.argv[3]) if len(sys.argv) > 3 else 500

KIND = rt.SCENE_THREE if NS == 3 else rt.SCENE_N
sc = rt.SphereCollection.generate(KIND, NS, 1)
sph = np.frombuffer(sc.as_bytes(), dtype=np.float32).reshape(-1, 8).astype(np.float64)
cam = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=65536),
                                   W, H, 0.5).to_c()
o = np.array(cam.center)
du, dv = np.array(cam.pixel_delta_u), np.array(cam.pixel_delta_v)
p00 = np.array(cam.viewport_upper_left) + 0.5 * (du + dv)
ys, xs = np.mgrid[0:H, 0:W]
d = (p00 + xs[..., None] * du + ys[..., None] * dv - o).reshape(-1, 3)
a = (d * d).sum(1)
tbest = np.full(len(d), np.inf)
idx = np.full(len(d), -1)
for i, s in enumerate(sph):                       # wgsl:164-203, nearest root > 0.001
    oc = s[:3] - o
    h = d @ oc
    disc = h * h - a * (oc @ oc - s[3] * s[3])
    ok = disc >= 0
    q = np.sqrt(np.where(ok, disc, 0.0))
    r1, r2 = (h - q) / a, (h + q) / a
    t = np.where(ok, np.where(r1 > 0.001, r1, np.where(r2 > 0.001, r2, np.inf)), np.inf)
    m = t < tbest
    tbest[m], idx[m] = t[m], i
mw = sph[np.maximum(idx, 0), 7]                   # material selector (wgsl:272-283)
kind = np.where(idx < 0, 0, np.where(mw < -1, 1, np.where(mw <= 1, 2, 3)))  # miss/lamb/metal/diel
Hp, Wp = (H + 7) // 8 * 8, (W + 15) // 16 * 16
K = np.zeros((Hp, Wp), int)
K[:H, :W] = kind.reshape(H, W)
# waves: (tile row, tile-column pair, slot, lane)
T = K.reshape(Hp // 8, 8, Wp // 16, 2, 8).transpose(0, 2, 3, 1, 4).reshape(-1, 2, 64)
nw = len(T)
out = {"config": f"{W}x{H}, {NS} spheres, pixel-centre hits", "waves": nw,
       "pixel_frac": {n: round(float((kind == k).mean()), 4)
                      for k, n in enumerate(("miss", "lambertian", "metal", "dielectric"))}}
oth = T >= 2
first = np.where(oth[:, 0], T[:, 0], np.where(oth[:, 1], T[:, 1], 0))
second = np.where(oth[:, 0] & oth[:, 1], T[:, 1], 0)
for k, n in ((2, "metal"), (3, "dielectric")):
    m = T == k
    out[n] = {"waves_with_any": round(float(m.any((1, 2)).mean()), 4),
              "passes_per_wave_now": round(float(m.any(2).sum(1).mean()), 4),
              "passes_per_wave_merged": round(float((first == k).any(1).mean() + (second == k).any(1).mean()), 4),
              "passes_per_wave_compacted": round(float(np.ceil(m.sum((1, 2)) / 64).mean()), 4)}
print(json.dumps(out))
