"""Benchmark of the per-pixel ray-tracing hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config K3]

Workload (default K3 = BASELINE.json configs[2], the config the north-star target is
quoted on): 1920x1080, seeded 500-sphere scene, max_depth 1.  A "step" is one
progressive `update` (wgsl:333-364): one camera sample per pixel of this rank's stripe
bands, read-modify-write of the RGBA32F accumulator in HBM.  With N GPUs (one process per
GPU, launched by torch.distributed.run) the image is split into 8-row bands dealt
round-robin, and after the K timed steps the finished tiles are gathered to rank 0 with
ONE RCCL gather + the de-interleave kernel — both inside the timed region.

value = W*H*K camera rays / max-over-ranks wall time (Mrays/s, whole job).
roofline (trace kernel, average launch time from HIP events): for the default culled scan
the algorithmic HBM bytes (32 B/pixel/step) against 8 TB/s; for --scan exhaustive the
algorithmic FP32 work (23 FLOP per ray-sphere test) against the 157.3 TFLOP/s
FP32 vector peak.  The exhaustive kernel is also timed on the same frames
(fp32_exhaustive_scan) so both rooflines appear in one line.
cpu_baseline: the scalar C oracle on one host core over a bounded sample (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import gpu_ray_tracing as rt  # noqa: E402
from gpu_ray_tracing.distributed import StripeRenderer  # noqa: E402

BASELINE = json.loads((ROOT / "BASELINE.json").read_text())
PEAK_FP32_TFLOPS = 157.3      # MI355X FP32 vector peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E peak
FLOP_PER_TEST = 23            # oc 3, a 5, h 5, c 7, D 3 (wgsl:183-187)
BYTES_PER_PIXEL_STEP = 32     # 16 B load + 16 B store (wgsl:339, 363)
FRAME_SEED = 0x5EED

CONFIGS = {
    # name: (width, height, scene kind, n_spheres, max_depth, description)
    "K2": (1920, 1080, rt.SCENE_THREE, 3, 1, "configs[1]: 1920x1080, 3 spheres, 1 spp/step"),
    "K3": (1920, 1080, rt.SCENE_N, 500, 1, "configs[2]: 1920x1080, 500 spheres, 1 spp/step"),
    "K5": (3840, 2160, rt.SCENE_N, 500, 8, "configs[4]: 3840x2160, 500 spheres, 1 spp/step, 8 bounces"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="K3", choices=sorted(CONFIGS))
    ap.add_argument("--scan", default="culled", choices=["culled", "exhaustive"],
                    help="sphere-list scan: exact wave-level culling (default) or the "
                         "reference's exhaustive linear walk; images are bit-identical")
    ap.add_argument("--exhaustive-steps", type=int, default=20,
                    help="also time the exhaustive-scan kernel for its FP32 roofline")
    ap.add_argument("--cpu-frames", type=float, default=2.0,
                    help="CPU baseline sample size in frames of the workload (0 = skip)")
    return ap.parse_args()


def cpu_baseline(cam, spheres, w, h, frames):
    """Scalar C oracle, one thread, on `frames` x (a row subset of) the same workload."""
    from oracle import oracle as O
    rows = max(1, int(round(h * min(frames, 1.0))))
    reps = max(1, int(round(frames))) if frames >= 1 else 1
    img = np.zeros((h, w, 4), np.float32)
    O.lib()
    t0 = time.perf_counter()
    segs = 0
    for _ in range(reps):
        _, s = O.update(img, cam.blob, spheres.spheres, rows=(0, rows))
        segs += s
    dt = time.perf_counter() - t0
    rays = rows * w * reps
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x {w}x{rows} progressive update(s) of the same scene/camera, "
                      f"scalar C oracle (oracle/rt_oracle.c, gcc -O3), 1 thread, {dt:.1f} s"}


def load_pmc(config):
    """Per-launch HBM bytes from the committed rocprofv3 PMC passes, if present."""
    p = ROOT / "profiles" / f"pmc_{config}.json"
    if p.exists():
        d = json.loads(p.read_text())
        return d.get("hbm_bytes_per_launch")
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with "
                         f"torch.distributed.run --nproc-per-node N")
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    w, h, kind, nsph, depth, desc = CONFIGS[args.config]
    spheres = rt.SphereCollection.generate(kind, nsph, 1)
    frames = args.warmup + args.steps
    seeds = rt.frame_seeds(FRAME_SEED, frames + args.exhaustive_steps)
    # spp cap above every frame this run traces (so no frame is a no-op)
    settings = rt.CameraSettings(max_depth=depth,
                                 samples_per_pixel=max(500, frames + args.exhaustive_steps))
    cam0 = rt.SceneCamera.from_settings(settings, w, h, float(seeds[0]))
    cams = [cam0.with_fields(camera_has_moved=1.0 if f == 0 else 0.0) for f in range(2)]

    pipe = rt.ComputeShaderPipeline(local_rank)
    pipe.set_scan_mode(args.scan)
    pipe.set_spheres(spheres)
    r = StripeRenderer(pipe, w, h, rank, world)
    stream = torch.cuda.current_stream()

    # warmup (untimed) — frame 0 resets the accumulator (camera_has_moved = 1)
    if args.warmup:
        r.frames(cams[0], spheres, seeds[:args.warmup])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # timed: `steps` progressive frames = `steps` update dispatches issued by one C call
    # (rt_update_frames), then the single gather of the finished tiles.
    cam_t = cams[min(1, frames - 1)]          # camera_has_moved = 0 from here on
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    r.frames(cam_t, spheres, seeds[args.warmup:])
    ev1.record(stream)
    image = r.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # every pixel of the gathered image must hold exactly warmup + steps samples
    sample_ok = image is not None and bool(torch.all(image[..., 3] == frames).item())
    # HIP events around the timed dispatches: average per launch, inter-kernel gaps included
    launch_s = ev0.elapsed_time(ev1) / 1e3 / args.steps
    local_px = w * min(r.rows, h)
    # SURVEY §8d algorithmic units: the reference's exhaustive scan does N tests of 23 FLOP
    # per segment; at max_depth 1 every sample is exactly one segment.
    flops = local_px * nsph * FLOP_PER_TEST if depth == 1 else None
    hbm_bytes = local_px * BYTES_PER_PIXEL_STEP
    value = w * h * args.steps / dt / 1e6

    # The exhaustive (reference-algorithm) kernel on the same frames, for its FP32 roofline.
    exh = None
    if args.scan == "culled" and flops and args.exhaustive_steps > 0:
        pipe.set_scan_mode("exhaustive")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r.frames(cam_t, spheres, seeds[frames:frames + args.exhaustive_steps])
        e1.record(stream)
        torch.cuda.synchronize()
        pipe.set_scan_mode(args.scan)
        t_exh = e0.elapsed_time(e1) / 1e3 / args.exhaustive_steps
        exh = {"kernel_avg_us": round(t_exh * 1e6, 2),
               "achieved": round(flops / t_exh / 1e12, 3), "peak": PEAK_FP32_TFLOPS,
               "unit": "TFLOP/s", "frac": round(flops / t_exh / 1e12 / PEAK_FP32_TFLOPS, 4),
               "flop_per_launch": flops,
               "speedup_of_culled": round(t_exh / launch_s, 2)}

    if args.scan == "exhaustive" and flops:
        roof = {"bound": "valu", "achieved": round(flops / launch_s / 1e12, 3),
                "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(flops / launch_s / 1e12 / PEAK_FP32_TFLOPS, 4),
                "traffic": load_pmc(f"{args.config}_exhaustive"),
                "kernel_avg_us": round(launch_s * 1e6, 2), "flop_per_launch": flops}
    else:
        # Culled scan: the redundant ray-sphere tests are gone (exactly), so
        # the algorithm-independent unit left is the accumulator's 32 B/pixel of HBM.
        roof = {"bound": "hbm", "achieved": round(hbm_bytes / launch_s / 1e9, 1),
                "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(hbm_bytes / launch_s / 1e9 / PEAK_HBM_GBS, 4),
                "traffic": load_pmc(f"{args.config}_culled"),
                "kernel_avg_us": round(launch_s * 1e6, 2), "bytes_per_launch": hbm_bytes}

    if rank == 0:
        line = {
            "metric": BASELINE["metric"],
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene + per-frame seeds; SURVEY §8d)",
            "config": {"workload": f"{args.config} {desc}, max_depth {depth}",
                       "width": w, "height": h, "spheres": nsph, "spp_per_step": 1,
                       "max_depth": depth, "parallelism": f"stripes{world}",
                       "scan": args.scan,
                       "kernel": rt._lib.lib().rt_kernel_name(0).decode()},
            "roofline": roof,
            "fp32_exhaustive_scan": exh,
            "accumulated_spp_ok": sample_ok,
        }
        if world == 1 and args.cpu_frames > 0:
            line["cpu_baseline"] = cpu_baseline(cams[0], spheres, w, h, args.cpu_frames)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    pipe.close()


if __name__ == "__main__":
    main()
