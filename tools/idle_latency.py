"""Does an idle GPU add latency to a timed call? (diagnostic)  The K3 chain call of a rank's
share (and one tiny kernel) timed wall-clock around the call and the stream's synchronize,
with the GPU otherwise idle, after a 1-ms host pause, and while a 1-wave spin kernel
(torch.cuda._sleep) runs on a second stream.
usage: python tools/idle_latency.py [N] [reps]"""
import json
import statistics as st
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
R = int(sys.argv[2]) if len(sys.argv) > 2 else 25
g = dict(np.load(ROOT / "tests" / "golden" / "bench_k3.npz"))
w, h = int(g["width"]), int(g["height"])
cam, sc, seeds = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]), g["seeds"]
still = cam.with_fields(camera_has_moved=0.0)
pipe = rt.ComputeShaderPipeline(0)
pipe.set_frame_images("every")
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
r = StripeRenderer(pipe, w, h, 0, N)
x = torch.zeros(1, device="cuda")
t_w = time.perf_counter()
while time.perf_counter() - t_w < 0.05:
    r.frames(cam, sc, seeds[:25])
    torch.cuda.synchronize()


def region(kind, variant):
    if kind == "call":
        r.frames(cam, sc, seeds[:5])
    torch.cuda.synchronize()
    if variant == "pause":
        time.sleep(0.001)
    if variant == "spin":
        with torch.cuda.stream(side):
            torch.cuda._sleep(4_000_000)
        time.sleep(0.0002)
    t0 = time.perf_counter()
    if kind == "call":
        r.frames(still, sc, seeds[5:25])
    else:
        x.fill_(1.0)
    main.synchronize()
    t = time.perf_counter() - t0
    side.synchronize()
    return t * 1e6


out = {"share": f"rank 0 of {N}", "reps": R}
for kind in ("tiny", "call"):
    for variant in ("idle", "pause", "spin", "idle", "spin"):
        v = [region(kind, variant) for _ in range(R)]
        key = f"{kind}_{variant}"
        key = key if key not in out else key + "_again"
        out[key] = {"med_us": round(st.median(v), 2), "min_us": round(min(v), 2)}
        print(key, out[key], flush=True)
print(json.dumps(out))
pipe.close()
