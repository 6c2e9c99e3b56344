"""Benchmark of the per-pixel ray-tracing hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config K3]   (K=512, W=128)

Workload (default K3 = BASELINE.json configs[2], the config the north-star target is
quoted on): 1920x1080, seeded 500-sphere scene, max_depth 1.  A "step" is one
progressive `update` (wgsl:333-364): one camera sample per pixel of this rank's stripe
bands, read-modify-write of the RGBA32F accumulator in HBM.  With N GPUs (one process per
GPU, launched by torch.distributed.run) the image is split into 8-row bands dealt
round-robin, and after the K timed steps the finished tiles are gathered to rank 0 with
ONE RCCL gather + the de-interleave kernel — both inside the timed region.

The K steps are issued by one rt_update_frames call per rank: at max_depth <= 1 it runs up
to 64 frames per launch, each wave carrying its pixels' accumulator in registers from frame
to frame and storing every frame's image to the ping-pong buffers — both buffers end exactly
as K chained `update` dispatches leave them (tests/test_gpu_parity.py); per_frame_dispatch
times the same frames with one launch per frame (the reference's dispatch structure).

value = W*H*K camera rays / max-over-ranks wall time (Mrays/s, whole job).
roofline (trace kernel, average launch time from HIP events): for the default culled scan
the algorithmic HBM bytes of the reference's progressive update (32 B/pixel/frame, SURVEY
§8d) against 8 TB/s — the fused launches move 16 B/pixel/frame + 16 B/pixel/launch
(moved_bytes_per_launch; PMC traffic beside it); for --scan exhaustive the
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
    # defaults: whole 64-frame launches; the first warmup launch measures the tile costs
    # the timed launches are scheduled by and the second sorts them (rt_set_tile_order);
    # 512 timed frames (8 ms on one GPU) amortise the job's single gather at N > 1
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=128)
    ap.add_argument("--config", default="K3", choices=sorted(CONFIGS))
    ap.add_argument("--scan", default="culled", choices=["culled", "exhaustive"],
                    help="sphere-list scan: exact wave-level culling (default) or the "
                         "reference's exhaustive linear walk; images are bit-identical")
    ap.add_argument("--exhaustive-steps", type=int, default=20,
                    help="also time the exhaustive-scan kernel for its FP32 roofline")
    ap.add_argument("--per-frame-steps", type=int, default=20,
                    help="also time frames with one launch each (the reference's structure)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU baseline budget in seconds (0 = skip)")
    return ap.parse_args()


def host_threads():
    """Host cores for the threaded baseline: this process's CPU set, at most 16 (the GPU
    box's per-GPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_model():
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cam, spheres, w, h, seconds):
    """The scalar C oracle on the same frame: (i) one thread on a row band
    sized to ~seconds/3, (ii) host_threads() threads over 8-row bands of whole frames
    for ~2*seconds/3.  The threaded run is the reported value."""
    from oracle import oracle as O
    img = np.zeros((h, w, 4), np.float32)
    O.lib()
    # single thread: calibrate on 8 rows through the middle of the image, then size the band
    mid = (h // 2) & ~7
    t0 = time.perf_counter()
    O.update(img, cam.blob, spheres.spheres, rows=(mid, mid + 8))
    per_row = (time.perf_counter() - t0) / 8
    rows1 = int(min(h, max(8, seconds / 3 / max(per_row, 1e-9)))) & ~7 or 8
    y0 = max(0, (h - rows1) // 2) & ~7
    t0 = time.perf_counter()
    O.update(img, cam.blob, spheres.spheres, rows=(y0, y0 + rows1))
    single = rows1 * w / (time.perf_counter() - t0) / 1e6
    # threaded: whole frames
    T = host_threads()
    frames = max(1, int(round(2 * seconds / 3 / (w * h / (single * 1e6 * T)))))
    t0 = time.perf_counter()
    for _ in range(frames):
        O.update_parallel(img, cam.blob, spheres.spheres, T)
    dt = time.perf_counter() - t0
    return {"value": round(w * h * frames / dt / 1e6, 3), "unit": "Mrays/s", "cores": T,
            "kind": "port",
            "sample": f"{frames} full {w}x{h} update(s) on {T} threads (8-row bands from a "
                      f"queue), {dt:.1f} s; scalar C oracle (oracle/rt_oracle.c, gcc -O3)",
            "single_thread": {"value": round(single, 3), "cores": 1,
                              "sample": f"{w}x{rows1} rows of one update"},
            "cpu_model": cpu_model()}


def load_pmc(config, frames_per_launch=1):
    """Per-launch HBM bytes from the committed rocprofv3 PMC passes, if present and taken
    at the same frames per launch."""
    p = ROOT / "profiles" / f"pmc_{config}.json"
    if p.exists():
        d = json.loads(p.read_text())
        if d.get("frames_per_launch", 1) == frames_per_launch:
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
    # the side measurements keep accumulating into the same image after the timed frames:
    # the exhaustive frames first, then the one-launch-per-frame frames (own seeds each)
    extra = args.exhaustive_steps + args.per_frame_steps
    seeds = rt.frame_seeds(FRAME_SEED, frames + extra)
    # spp cap above every frame this run traces (so no frame is a no-op)
    settings = rt.CameraSettings(max_depth=depth,
                                 samples_per_pixel=max(500, frames + extra))
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
    r.frames(cam_t, spheres, seeds[args.warmup:frames])
    ev1.record(stream)
    image = r.finish()
    ev2 = torch.cuda.Event(enable_timing=True)
    ev2.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # breakdown (HIP events on this rank's stream): the K frames, then the gather +
    # de-interleave; both stay inside dt
    render_s, gather_s = ev0.elapsed_time(ev1) / 1e3, ev1.elapsed_time(ev2) / 1e3
    if world > 1:
        t = torch.tensor([dt, render_s, gather_s], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, render_s, gather_s = (float(x) for x in t.tolist())

    # every pixel of the gathered image must hold exactly warmup + steps samples
    sample_ok = image is not None and bool(torch.all(image[..., 3] == frames).item())
    # HIP events around the timed dispatches: per step and per launch, gaps included
    fpl = r.frames_per_launch(cam_t)
    launches = -(-args.steps // fpl)
    step_s = ev0.elapsed_time(ev1) / 1e3 / args.steps
    launch_s = ev0.elapsed_time(ev1) / 1e3 / launches
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
               "speedup_of_culled": round(t_exh / step_s, 2)}

    # Presentation kernel on the gathered image: 16 B read + 4 B written per
    # pixel, HBM-bound.
    present = None
    if image is not None:
        out8 = torch.empty((h, w, 4), dtype=torch.uint8, device=image.device)
        pipe.present(image, w, h, "srgb", out8)
        p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        p0.record(stream)
        for _ in range(20):
            pipe.present(image, w, h, "srgb", out8)
        p1.record(stream)
        torch.cuda.synchronize()
        t_p = p0.elapsed_time(p1) / 1e3 / 20
        present = {"kernel": "rt_present_kernel<srgb>", "avg_us": round(t_p * 1e6, 2),
                   "achieved": round(w * h * 20 / t_p / 1e9, 1), "peak": PEAK_HBM_GBS,
                   "unit": "GB/s", "frac": round(w * h * 20 / t_p / 1e9 / PEAK_HBM_GBS, 4),
                   "bytes_per_launch": w * h * 20}

    # The reference's dispatch structure on the same frames: one launch per frame.
    per_frame = None
    if fpl > 1 and args.per_frame_steps > 0:
        pipe.set_frames_per_launch(1)
        q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        q0.record(stream)
        s0 = frames + args.exhaustive_steps
        r.frames(cam_t, spheres, seeds[s0:s0 + args.per_frame_steps])
        q1.record(stream)
        torch.cuda.synchronize()
        pipe.set_frames_per_launch(0)
        t_pf = q0.elapsed_time(q1) / 1e3 / args.per_frame_steps
        per_frame = {"frames_per_launch": 1, "us_per_step": round(t_pf * 1e6, 2),
                     "Mrays_per_s": round(local_px / t_pf / 1e6, 1),
                     "hbm_frac": round(hbm_bytes / t_pf / 1e9 / PEAK_HBM_GBS, 4)}

    avg_frames = args.steps / launches
    if args.scan == "exhaustive" and flops:
        roof = {"bound": "valu", "achieved": round(flops / step_s / 1e12, 3),
                "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(flops / step_s / 1e12 / PEAK_FP32_TFLOPS, 4),
                "traffic": load_pmc(f"{args.config}_exhaustive", fpl),
                "kernel_avg_us": round(launch_s * 1e6, 2), "frames_per_launch": fpl,
                "flop_per_launch": round(flops * avg_frames)}
    else:
        # Culled scan: the redundant ray-sphere tests are gone (exactly), so
        # the algorithm-independent unit left is the progressive update's 32 B/pixel.
        roof = {"bound": "hbm", "achieved": round(hbm_bytes / step_s / 1e9, 1),
                "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(hbm_bytes / step_s / 1e9 / PEAK_HBM_GBS, 4),
                "traffic": load_pmc(f"{args.config}_culled", fpl),
                "kernel_avg_us": round(launch_s * 1e6, 2), "frames_per_launch": fpl,
                "bytes_per_launch": round(hbm_bytes * avg_frames),
                "moved_bytes_per_launch": round(local_px * 16 * (avg_frames + 1)),
                "us_per_step": round(step_s * 1e6, 2)}

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
            "present_rgba8": present,
            "per_frame_dispatch": per_frame,
            "accumulated_spp_ok": sample_ok,
            # max over ranks; value's time includes both (and the barriers)
            "timed_breakdown_ms": {"frames": round(render_s * 1e3, 4),
                                   "gather_and_deinterleave": round(gather_s * 1e3, 4)},
        }
        if world == 1 and args.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(cams[0], spheres, w, h, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    pipe.close()


if __name__ == "__main__":
    main()
