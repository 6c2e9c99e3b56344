"""A fixed stream of 20-frame K3 chain calls of one rank's stripe share, for rocprofv3 --pmc
(diagnostic): one reset call, then CALLS calls continuing the accumulation with the still
camera — every launch of the timed instance a 20-frame launch of the same share, so the
per-dispatch medians of tools/pmc_bench_summary.py are those of the share bench.py times.
usage: rocprofv3 --pmc ... -- python3 tools/pmc_share.py N RANK PAIRS [CALLS]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
import torch  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

N, RANK, PAIRS = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
CALLS = int(sys.argv[4]) if len(sys.argv) > 4 else 20
w, h, F = 1920, 1080, 20
sc = rt.SphereCollection.generate(rt.SCENE_N, 500, 1)
seeds = rt.frame_seeds(0x5EED, F * (CALLS + 1))
cam0 = rt.SceneCamera.from_settings(rt.CameraSettings(max_depth=1, samples_per_pixel=65536),
                                    w, h, float(seeds[0]))
cam_t = cam0.with_fields(camera_has_moved=0.0)
pipe = rt.ComputeShaderPipeline(0)
pipe.set_spheres(sc)
pipe.set_frames_per_launch(0)
pipe.set_frame_images("every")
pipe.set_frame_pairs(PAIRS)
r = StripeRenderer(pipe, w, h, RANK, N)
r.frames(cam0, sc, seeds[:F])
for c in range(1, CALLS + 1):
    r.frames(cam_t, sc, seeds[c * F:(c + 1) * F])
torch.cuda.synchronize()
info = pipe.last_launch_info()
print(json.dumps({"share": f"rank {RANK} of {N}", "pairs": PAIRS, "calls": CALLS,
                  "kernel": info["kernel_name"], "launches": info["launches"]}))
pipe.close()
