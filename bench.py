"""Benchmark of the per-pixel ray-tracing hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config K3]

Configs (BASELINE.json `configs`):
  K2, K3 (default)  1920x1080, 3 / 500 spheres, max_depth 1.  A step is ONE progressive
                    `update` (wgsl:333-364): one camera sample per pixel of this rank's stripe
                    bands, accumulated into the RGBA32F image.  The whole image (N=1) runs
                    one launch per frame, the reference's dispatch structure (lib.rs:408-417);
                    rank shares of at most CHAIN_MAX_TILES tiles run the steps' frames as
                    frame chains — fused launches that still write every frame's image to the
                    ping-pong buffer its dispatch would write (rt_set_frame_images EVERY), so
                    only the launch boundary between frames goes (--frame-launch).
  K4                1920x1080, 500 spheres, 64 spp anti-aliased accumulate, max_depth 1.  A
                    step is one 64-spp render from a reset accumulator: 64 chained updates
                    issued by one rt_update_frames call (fused launches of up to 64 frames).
  K5                3840x2160, 500 spheres, 64 spp, 8 bounces — the multi-GPU config.  A step
                    is one 64-spp render (one 64-frame launch of the bounce instance).
With N GPUs (one process per GPU, torch.distributed.run) the image is split into 8-row bands
dealt round-robin; the steps have no collective (a rank's bands need nothing from another
rank).  After the K timed steps the finished tiles are gathered to rank 0 with ONE RCCL
gather + the de-interleave kernel (rt_gather_stripes, the ncclGather behind librt_hip.so's C
ABI; RT_GATHER=torch: torch.distributed.gather instead): the job's output collection, timed
on its own between barriers and reported as `gather` next to the job-level rate that includes
it (`job`), not inside the K steps.

value = W*H*spp_per_step*K camera rays / max-over-ranks wall time of the K steps (Mrays/s,
all ranks together).
image_ok: the timed image against committed fixtures (K2/K3: 4096 sampled pixels after W+K
frames, tests/golden/bench_k*.npz; K4: the full-image SHA-256 of tests/golden/k4.npz; K5:
the 512 sampled pixels of k5.npz) — null when no fixture covers the run's frame count.
roofline (the timed trace-kernel launches, HIP events on the stream they run on): the
algorithmic bytes of the reference's progressive update, 32 B per pixel per launch (16 B
load + 16 B store of the accumulator), against 8 TB/s; `traffic` = the PMC
bytes of the same kernel at the same frames per launch (profiles/pmc_r02_<config>.json,
FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM); `valu` = the binding resource: VALU
wave-instructions per launch (same PMC file) x 2 cycles (a wave64 VALU op on a SIMD-32) over
the cycles 1024 SIMDs offer at 2.4 GHz during the measured launch time.
cpu_baseline: the scalar C oracle on the box's host cores over a bounded sample (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
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
from gpu_ray_tracing.distributed import StripeComm, StripeRenderer  # noqa: E402

BASELINE = json.loads((ROOT / "BASELINE.json").read_text())
GOLDEN = ROOT / "tests" / "golden"
PEAK_FP32_TFLOPS = 157.3      # MI355X FP32 vector peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E peak
# Practical floor of one progressive update's memory pattern (read + write 16 B per pixel,
# one dependent launch per frame, no tracing), measured by tools/rmw_floor.hip at 1920x1080:
# 10.18 us per launch = 0.815 of the 8 TB/s peak (profiles/archive/r02_rmw_floor.jsonl)
RMW_FLOOR_GBS = 6518.0
CLOCK_GHZ = 2.4               # MI355X max engine clock
SIMDS = 1024                  # 256 CUs x 4 SIMDs
VALU_ISSUE_CYCLES = 2         # one wave64 VALU instruction on a SIMD-32
FLOP_PER_TEST = 23            # oc 3, a 5, h 5, c 7, D 3 (wgsl:183-187)
BYTES_PER_PIXEL_LAUNCH = 32   # 16 B load + 16 B store of the accumulator (wgsl:339, 363)
FRAME_SEED = 0x5EED
BENCH_SPP = 65536             # the dispatch configs' spp cap (never reached; fixtures agree)

CONFIGS = {
    # name: width, height, scene kind, spheres, max_depth, frames per step, description
    "K2": (1920, 1080, rt.SCENE_THREE, 3, 1, 1,
           "configs[1]: 1920x1080, 3 spheres, 1 spp, one progressive update per step"),
    "K3": (1920, 1080, rt.SCENE_N, 500, 1, 1,
           "configs[2]: 1920x1080, 500 spheres, 1 spp, one progressive update per step"),
    "K4": (1920, 1080, rt.SCENE_N, 500, 1, 64,
           "configs[3]: 1920x1080, 500 spheres, 64 spp accumulate per step (fused launches)"),
    "K5": (3840, 2160, rt.SCENE_N, 500, 8, 64,
           "configs[4]: 3840x2160, 500 spheres, 64 spp, 8 bounces per step"),
}
DEFAULT_STEPS = {"K2": (200, 20), "K3": (200, 20), "K4": (8, 2), "K5": (2, 1)}
# K2/K3 steps of a rank share of at most this many 8x8 tiles run as frame chains (fused
# launches writing every frame's image) under --frame-launch auto; larger shares (the whole
# image: 32 400 tiles) one update launch per frame.  DESIGN.md §6.
CHAIN_MAX_TILES = 20000


def share_tiles(w, rows):
    return ((w + 7) // 8) * ((rows + 7) // 8)


def frame_launch_mode(policy, w, rows):
    """The K2/K3 step structure for a share of `rows` local rows: 'dispatch' or 'chain'."""
    if policy != "auto":
        return policy
    return "chain" if share_tiles(w, rows) <= CHAIN_MAX_TILES else "dispatch"


def set_frame_launch(pipe, mode):
    """dispatch: one `update` launch per frame (rt_set_frames_per_launch(1)); chain: fused
    launches (up to 64 frames) that write every frame's image (rt_set_frame_images EVERY)."""
    pipe.set_frames_per_launch(1 if mode == "dispatch" else 0)
    pipe.set_frame_images("every" if mode == "chain" else "last_two")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="K3", choices=sorted(CONFIGS))
    ap.add_argument("--queues", type=int, default=int(os.environ.get("RT_QUEUES", "0")),
                    help="concurrent parts per one-frame update (rt_set_update_queues; "
                         "0 = the library's choice)")
    ap.add_argument("--submit", default=os.environ.get("RT_SUBMIT", "auto"),
                    choices=["auto", "hip", "aql"],
                    help="how one-frame updates are submitted (rt_set_update_submit): HIP "
                         "launches (auto) or AQL packets on the context's HSA queues")
    ap.add_argument("--warm-ms", type=float, default=float(os.environ.get("RT_WARM_MS", "50")),
                    help="before the warmup steps, render this long with the same update "
                         "frames on scratch images (untimed: a running render's steps, not a "
                         "freshly started process's first launches, are what is timed; 0 = "
                         "off)")
    ap.add_argument("--frame-launch", default=os.environ.get("RT_FRAME_LAUNCH", "auto"),
                    choices=["auto", "dispatch", "chain"],
                    help="K2/K3 steps: one update launch per frame (dispatch, the reference's "
                         "structure), or the rank's consecutive frames in fused launches that "
                         "still write every frame's image to its ping-pong buffer (chain: "
                         "rt_set_frame_images EVERY, only the launch boundary between frames "
                         "removed); auto = dispatch for shares of at least "
                         "CHAIN_MAX_TILES + 1 tiles (whole images), chain below")
    ap.add_argument("--gate", action="store_true",
                    help="diagnostic for profiled runs: hold the stream while the timed steps "
                         "are issued, then release it (StreamGate); the line is then not a "
                         "measurement")
    ap.add_argument("--scan", default="culled", choices=["culled", "exhaustive"],
                    help="sphere-list scan: exact culling (default) or the reference's "
                         "exhaustive linear walk; images are bit-identical")
    ap.add_argument("--side", type=int, default=20,
                    help="frames for each side measurement (exhaustive scan, fused frames, "
                         "moving camera; 0 = none)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU baseline budget in seconds (0 = skip)")
    a = ap.parse_args()
    d_steps, d_warm = DEFAULT_STEPS[a.config]
    a.steps = d_steps if a.steps is None else a.steps
    a.warmup = d_warm if a.warmup is None else a.warmup
    return a


def host_cpus():
    """(nproc, this process's CPU-affinity size): the whole machine and what we may use."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    return nproc, aff


def host_threads():
    """Host cores for the threaded baseline: this process's CPU set, at most 16 (a GPU
    box's per-GPU share of host cores: OMP_NUM_THREADS / MAX_JOBS are 16 there)."""
    return max(1, min(16, host_cpus()[1]))


def cgroup_cpus():
    """The CPU bandwidth limit of this process's cgroup (cgroup v2 cpu.max: quota / period)
    in CPUs, or None when unlimited or unreadable.  (A box may show every host core in nproc
    and the affinity set while its cgroup allows far fewer: the all-cores sample then runs
    more threads than the quota schedules at once.)"""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cam, spheres, w, h, seconds):
    """The scalar C oracle on one update of the same camera and scene, on
    native threads (oracle_update_threads: 8-row bands claimed from a shared counter):
    (i) one thread on a row band (~seconds/5), (ii) host_threads() threads over whole frames
    (~2*seconds/5, at least one frame; the reported value: a GPU's share of the host), (iii)
    every core of the process's affinity set (~seconds/5, 2-row bands)."""
    from oracle import oracle as O
    img = np.zeros((h, w, 4), np.float32)
    O.lib()
    mid = (h // 2) & ~7
    t0 = time.perf_counter()
    O.update(img, cam.blob, spheres.spheres, rows=(mid, mid + 8))
    per_row = (time.perf_counter() - t0) / 8
    rows1 = int(min(h, max(8, seconds / 5 / max(per_row, 1e-9)))) & ~7 or 8
    y0 = max(0, (h - rows1) // 2) & ~7
    t0 = time.perf_counter()
    O.update(img, cam.blob, spheres.spheres, rows=(y0, y0 + rows1))
    single = rows1 * w / (time.perf_counter() - t0) / 1e6

    def threaded(threads, share, band):
        # one frame first (its time sizes the sample), then enough frames for ~share s
        t0 = time.perf_counter()
        O.update_threads(img, cam.blob, spheres.spheres, threads, band)
        one = time.perf_counter() - t0
        frames = max(1, int(round(share / max(one, 1e-6))) - 1)
        t0 = time.perf_counter()
        for _ in range(frames):
            O.update_threads(img, cam.blob, spheres.spheres, threads, band)
        return frames, time.perf_counter() - t0

    T = host_threads()
    frames, dt = threaded(T, 2 * seconds / 5, 8)
    # every CPU the process may run on at once: the affinity set, capped by the cgroup's CPU
    # bandwidth quota (a GPU box shows 256 CPUs in its affinity set while its cgroup
    # schedules 16: 256 threads there time-slice 16 CPUs and measure the oversubscription)
    aff, quota = host_cpus()[1], cgroup_cpus()
    A = max(1, min(aff, int(quota))) if quota else aff
    band = max(1, min(8, h // (2 * A)))        # at least two bands per thread
    fa, dta = threaded(A, seconds / 5, band)
    return {"value": round(w * h * frames / dt / 1e6, 3), "unit": "Mrays/s", "cores": T,
            "kind": "port",
            "sample": f"{frames} full {w}x{h} update(s) on {T} threads (8-row bands from a "
                      f"shared counter), {dt:.1f} s; scalar C oracle (oracle/rt_oracle.c, gcc -O3), "
                      f"max_depth {int(cam.max_depth)}",
            "single_thread": {"value": round(single, 3), "cores": 1,
                              "sample": f"{w}x{rows1} rows of one update"},
            "all_cores": {"value": round(w * h * fa / dta / 1e6, 3), "cores": A,
                          "sample": f"{fa} full {w}x{h} update(s) on {A} threads "
                                    f"({band}-row bands from a shared counter), {dta:.1f} s",
                          "bound": ("cgroup CPU quota" if quota and int(quota) < aff
                                    else "affinity set")},
            "cpu_model": cpu_model(),
            "nproc": host_cpus()[0], "affinity_cpus": aff,
            "cgroup_cpu_quota": quota,
            "cores_rule": "value: min(16, affinity) threads, the per-GPU share of the box's host "
                          "cores; all_cores: min(affinity set, cgroup CPU quota) threads — every "
                          "CPU the process can run on at once"}


def load_pmc(config, kernel, frames_per_launch, queues=1):
    """The newest committed rocprofv3 PMC summary of the timed kernel (tools/pmc_bench.sh),
    if it was taken for the same kernel instance at the same frames per launch and the same
    concurrent parts per update (`queues`: a summary's per-launch counts are one part's), and
    its path."""
    for rnd in ("r05", "r04", "r03", "r02"):
        p = ROOT / "profiles" / f"pmc_{rnd}_{config}.json"
        if not p.exists():
            continue
        d = json.loads(p.read_text())
        if (d.get("kernel") == kernel and d.get("frames_per_launch") == frames_per_launch
                and d.get("queues", 1) == queues):
            return d, p.relative_to(ROOT).as_posix()
    return None, None


def load_weighted(config, kernel, pmc_path=None):
    """The weighted VALU cycles per launch of the timed kernel (tools/valu_weighted.py over
    the PMC instruction classes and the instance's disassembly), if committed — and, when the
    file names the PMC summary it was computed from, only for that summary."""
    for rnd in ("r05", "r04", "r03"):
        p = ROOT / "profiles" / f"valu_weighted_{rnd}_{config}.json"
        if not p.exists():
            continue
        d = json.loads(p.read_text())
        if d.get("kernel") == kernel and (pmc_path is None or d.get("pmc", pmc_path) == pmc_path):
            return d, p.relative_to(ROOT).as_posix()
    return None, None


def image_check(config, image, frames, cam, w, h):
    """The timed image against the committed fixtures (see the module docstring)."""
    if image is None:
        return None, "not the gathering rank"
    img = image.detach().cpu().numpy()
    if config in ("K2", "K3"):
        g = dict(np.load(GOLDEN / f"bench_{config.lower()}.npz"))
        if not np.array_equal(g["camera"].view(np.uint32), cam.blob.view(np.uint32)):
            return False, "camera blob differs from the fixture's"
        counts = [int(c) for c in g["frame_counts"]]
        if frames not in counts:
            return None, f"no fixture for {frames} frames (have {counts})"
        want = g["pixels"][counts.index(frames)]
        got = img[g["py"], g["px"]]
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        return bool(same.all()), f"{want.shape[0]} sampled pixels after {frames} frames"
    g = dict(np.load(GOLDEN / f"{config.lower()}.npz"))
    if "sha256" in g:
        ok = hashlib.sha256(np.ascontiguousarray(img, np.float32).tobytes()).hexdigest() == \
            str(g["sha256"])
        return ok, "full-image SHA-256 of the 64-spp render"
    got = img[g["py"], g["px"]]
    want = g["pixels"]
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    return bool(same.all()), f"{want.shape[0]} sampled pixels of the 64-spp render"


def share_pixels_ok(config, local, frames, world, rank=0):
    """A rank's share (local rows of bands rank, rank + world, ...) against the fixture's
    sampled pixels that fall in those bands (the K2/K3 fixtures after `frames` frames, K5's
    64-spp render)."""
    img = local.detach().cpu().numpy()
    if config in ("K2", "K3"):
        g = dict(np.load(GOLDEN / f"bench_{config.lower()}.npz"))
        counts = [int(c) for c in g["frame_counts"]]
        if frames not in counts:
            return None
        want = g["pixels"][counts.index(frames)]
    else:
        g = dict(np.load(GOLDEN / f"{config.lower()}.npz"))
        want = g["pixels"]
    py, px = g["py"], g["px"]
    mine = (py // 8) % world == rank
    ly = (py[mine] // 8 // world) * 8 + py[mine] % 8
    got, want = img[ly, px[mine]], want[mine]
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    return bool(same.all()) and int(mine.sum()) > 0


def over_ranks(share, world):
    """share(rank) -> {"us_per_step", ...} for every rank of a world-size run, timed one after
    another on this GPU: the job's step is the slowest rank's (bench.py --gpus N takes the
    max over ranks), so `us_per_step` is the max; each rank's own time and pixel check are
    kept (rank_us, image_ok = every rank's share matches the fixture)."""
    per = [share(r) for r in range(world)]
    slow = max(range(world), key=lambda r: per[r]["us_per_step"])
    out = dict(per[slow])
    out.update({"us_per_step": per[slow]["us_per_step"], "max_over_ranks": True,
                "slowest_rank": slow, "rank_us": [d["us_per_step"] for d in per],
                "rank0_us": per[0]["us_per_step"],
                "image_ok": all(d["image_ok"] for d in per) if all(
                    d["image_ok"] is not None for d in per) else None})
    return out


def driver_record_sides(device, stream, main_cfg, main_us):
    """Side measurements for the driver's N=1 record (after the timed region), each with its
    image check: the other per-dispatch config (K2 next to K3), one K5 64-spp step, and every
    rank's 1/2, 1/4, 1/8 share of K3 (one update launch per frame, and frame chains) and K5
    timed alone on this GPU — what each rank of `bench.py --gpus N` computes per step, the
    slowest rank setting the step — so the strong-scaling curve has a per-rank measurement
    behind it (tools/rank_sim.py's method)."""
    out = {}
    pipe = rt.ComputeShaderPipeline(device)
    try:
        def setup(cfg):
            w, h, kind, nsph, depth, spf, _ = CONFIGS[cfg]
            if spf == 1:
                sc = rt.SphereCollection.generate(kind, nsph, 1)
                seeds = rt.frame_seeds(FRAME_SEED, 25)
                st = rt.CameraSettings(max_depth=depth, samples_per_pixel=BENCH_SPP)
                cam = rt.SceneCamera.from_settings(st, w, h, float(seeds[0]))
            else:
                g = dict(np.load(GOLDEN / f"{cfg.lower()}.npz"))
                sc, seeds, cam = rt.SphereCollection(g["spheres"]), g["seeds"], rt.SceneCamera(g["camera"])
            return w, h, sc, seeds, cam

        def dispatch_share(cfg, world, mode, rank=0, reps=5, warm_s=0.05):
            # the driver's structure: 5 frames from a reset, then 20 timed (25-frame fixture),
            # as each rank of bench.py --gpus N runs it after its warm-up: untimed frames on
            # scratch images first (the share's lists, order and code, and warm_s of the same
            # frames — the main line's --warm-ms: the host's image check of the previous side
            # line leaves the GPU idle, and 5 ms of warm-up measured 0.3-0.8 us per step
            # slower), then `reps` timed regions, each from a reset; the median
            w, h, sc, seeds, cam = setup(cfg)
            set_frame_launch(pipe, mode)
            cam_t = cam.with_fields(camera_has_moved=0.0)
            scratch = StripeRenderer(pipe, w, h, rank, world)
            t_w = time.perf_counter()
            while True:
                scratch.frames(cam, sc, seeds[:20])
                torch.cuda.synchronize()
                if time.perf_counter() - t_w >= warm_s:
                    break
            del scratch
            r = StripeRenderer(pipe, w, h, rank, world)
            runs = []
            for _ in range(reps):
                r.frames(cam, sc, seeds[:5])
                runs.append(timed(stream, lambda: r.frames(cam_t, sc, seeds[5:25])) / 20)
            t = sorted(runs)[len(runs) // 2]
            info = pipe.last_launch_info()
            return {"us_per_step": round(t * 1e6, 2), "kernel": info["kernel_name"],
                    "launches_per_step": round(info["launches"] / 20, 3),
                    "runs_us": [round(x * 1e6, 2) for x in runs],
                    "image_ok": share_pixels_ok(cfg, r.local, 25, world, rank)}

        def k5_share(world, rank=0):
            w, h, sc, seeds, cam = setup("K5")
            pipe.set_frames_per_launch(0)
            pipe.set_frame_images("last_two")
            r = StripeRenderer(pipe, w, h, rank, world)
            r.frames(cam, sc, seeds)                   # records the tile costs
            r.frames(cam, sc, seeds)                   # builds the order (and its buffers)
            # (each call restarts from the camera's reset; the median of five launches)
            runs = sorted(timed(stream, lambda: r.frames(cam, sc, seeds)) for _ in range(5))
            t = runs[2]
            info = pipe.last_launch_info()
            return {"us_per_step": round(t * 1e6, 1), "us_per_spp": round(t / 64 * 1e6, 2),
                    "runs_us": [round(x * 1e6, 1) for x in runs],
                    "kernel": info["kernel_name"],
                    "image_ok": share_pixels_ok("K5", r.local, 64, world, rank)}

        other = "K2" if main_cfg == "K3" else "K3"
        d = dispatch_share(other, 1, "dispatch")
        w, h = CONFIGS[other][:2]
        out[other.lower()] = dict(d, Mrays_per_s=round(w * h / d["us_per_step"], 1),
                                  hbm_frac=round(w * h * BYTES_PER_PIXEL_LAUNCH /
                                                 (d["us_per_step"] * 1e3) / PEAK_HBM_GBS, 4),
                                  what=f"{other}: 5 + 20 frames from a reset, one update "
                                       f"launch per frame, µs per update by HIP events")
        # K4: one 64-spp 1920x1080 render from a reset (fused frames), as --config K4 steps,
        # the full-image SHA-256 of k4.npz
        w4, h4, sc4, seeds4, cam4 = setup("K4")
        pipe.set_frames_per_launch(0)
        pipe.set_frame_images("last_two")
        r4 = StripeRenderer(pipe, w4, h4, 0, 1)
        for _ in range(2):
            r4.frames(cam4, sc4, seeds4)               # costs recorded, order built
        runs4 = sorted(timed(stream, lambda: r4.frames(cam4, sc4, seeds4)) for _ in range(5))
        info4 = pipe.last_launch_info()
        ok4, what4 = image_check("K4", r4.local[:h4], 64, cam4, w4, h4)
        out["k4"] = {"us_per_step": round(runs4[2] * 1e6, 1),
                     "us_per_frame": round(runs4[2] / 64 * 1e6, 2),
                     "runs_us": [round(x * 1e6, 1) for x in runs4],
                     "kernel": info4["kernel_name"], "launches_per_step": info4["launches"],
                     "image_ok": ok4, "image_check": what4,
                     "Mrays_per_s": round(w4 * h4 * 64 / (runs4[2] * 1e6), 1),
                     "what": "K4: one 64-spp 1920x1080 render from a reset (fused frames, "
                             "cost-ordered after two untimed renders), the median of five"}
        del r4
        k5 = k5_share(1)
        out["k5"] = dict(k5, Mrays_per_s=round(3840 * 2160 * 64 / k5["us_per_step"], 1),
                         what="one 64-spp 3840x2160 depth-8 step (one 64-frame bounce launch, "
                              "cost-ordered by the steps before; the median of five), 512 "
                              "sampled pixels")
        shares = {"K3": {}, "K5": {}}
        base = {"dispatch": main_us if main_cfg == "K3" else None}
        for mode in ("dispatch", "chain"):
            rows = {}
            for world in (1, 2, 4, 8):
                if world == 1 and mode == "dispatch" and base["dispatch"]:
                    rows["1"] = {"us_per_step": round(base["dispatch"], 2), "kernel": "(the timed steps)"}
                    continue
                rows[str(world)] = over_ranks(
                    lambda rk: dispatch_share("K3", world, mode, rk), world)
            ref = rows["1"]["us_per_step"]
            for k, v in rows.items():
                v["predicted_efficiency"] = round(ref / (int(k) * v["us_per_step"]), 3)
            shares["K3"][mode] = rows
        # efficiency of each share against the 1-GPU step as the line times it
        one = shares["K3"]["dispatch"]["1"]["us_per_step"]
        for mode in ("dispatch", "chain"):
            for k, v in shares["K3"][mode].items():
                v["efficiency_vs_1gpu_step"] = round(one / (int(k) * v["us_per_step"]), 3)
        k5rows = {"1": {"us_per_step": k5["us_per_step"], "us_per_spp": k5["us_per_spp"]}}
        for world in (2, 4, 8):
            k5rows[str(world)] = over_ranks(lambda rk: k5_share(world, rk), world)
        for k, v in k5rows.items():
            v["predicted_efficiency"] = round(k5["us_per_step"] / (int(k) * v["us_per_step"]), 3)
        shares["K5"]["fused_64"] = k5rows
        shares["what"] = ("every rank's stripe share (8-row bands dealt round-robin) timed alone "
                          "on this GPU, i.e. each rank's step of bench.py --gpus N; us_per_step "
                          "= the slowest rank's (max_over_ranks; rank_us lists them all); "
                          "predicted_efficiency = the 1-rank time / (N x that time) in "
                          "the same launch structure; K3 'dispatch' = one update launch per "
                          "frame, 'chain' = fused launches writing every frame's image "
                          "(--frame-launch auto takes chain for shares <= %d tiles)"
                          % CHAIN_MAX_TILES)
        out["rank_shares"] = shares
    finally:
        pipe.close()
    return out


def _unserializable(o):
    """json default: a value the line cannot hold is named, not fatal (the line still
    prints; the bad path shows in its place)."""
    return f"<{type(o).__name__} {getattr(o, '__name__', '')}>"


def timed_steps(run, sync, world, barrier=None, device=None, stamp=None, wait=None):
    """The timed region of the K steps.  Every rank leaves an opening barrier (then
    synchronises), starts its clock, issues the steps (`run`), synchronises, and stops its
    clock: its own wall time of the K steps.  The closing barrier follows outside that time
    and is reported on its own (`barrier_s`), so that at N > 1 the value measures the render,
    not the collective's latency (a 8-rank K3 step is ~3 µs, the same order as one barrier).
    The job's time is the MAX over ranks (all ranks start together after the opening
    barrier).  Returns {"dt": max over ranks, "per_rank": [s...], "issue": this rank's host
    issue time, "barrier_s": max over ranks of the closing barrier}.  `stamp(name)` (optional)
    is called at the start, when the issue returns and after the synchronise.  `wait`
    (default: sync) is the closing wait of the steps; it must end in a synchronise."""
    barrier = barrier or dist.barrier
    wait = wait or sync
    sync()
    if world > 1:
        barrier()
        sync()
    if stamp:
        stamp("t0")
    t0 = time.perf_counter()
    run()
    t_issued = time.perf_counter()
    if stamp:
        stamp("issued")
    wait()
    mine = time.perf_counter() - t0
    if stamp:
        stamp("synced")
    bar = 0.0
    per_rank, bars = [mine], [0.0]
    if world > 1:
        tb = time.perf_counter()
        barrier()
        sync()
        bar = time.perf_counter() - tb
        t = torch.tensor([mine, bar], dtype=torch.float64, device=device)
        got = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(got, t)
        per_rank = [float(g[0]) for g in got]
        bars = [float(g[1]) for g in got]
    return {"dt": max(per_rank), "per_rank": per_rank, "issue": t_issued - t0,
            "barrier_s": max(bars)}


class StreamGate:
    """--gate (diagnostic, never a measurement): the stream waits on a host-memory word
    (hipStreamWaitValue32) while the timed steps are issued, and the host opens it after the
    issue, so that the GPU runs the steps back to back however slowly the host issues them —
    under rocprofv3's kernel trace every dispatch costs the host ~8 µs more, which starves a
    one-launch-per-frame chain and distorts the trace (tools/timeline.py).  Uses the HIP
    runtime torch loaded (same soname)."""

    def __init__(self):
        import ctypes
        self.ct = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        p = ctypes.c_void_p()
        if self.hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(64), 0) != 0:
            raise RuntimeError("hipHostMalloc failed")
        self.ptr = p
        self.word = ctypes.c_uint32.from_address(p.value)
        self.word.value = 0
        self.n = 0

    def hold(self, stream):
        self.n += 1
        rc = self.hip.hipStreamWaitValue32(self.ct.c_void_p(stream.cuda_stream), self.ptr,
                                           self.ct.c_uint32(self.n), 0,        # >= n
                                           self.ct.c_uint32(0xFFFFFFFF))
        if rc != 0:
            raise RuntimeError(f"hipStreamWaitValue32 failed ({rc})")

    def release(self):
        self.word.value = self.n


def timed(stream, fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with "
                         f"torch.distributed.run --nproc-per-node N")
    # RT_BENCH_BACKEND=gloo rehearses the N > 1 path with every rank on the visible GPUs
    # (several ranks per GPU; the gather staged through host memory) — a check of the
    # multi-rank flow and its image on a one-GPU box, never a measurement
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    device = local_rank if backend == "nccl" else local_rank % torch.cuda.device_count()
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    cfg = args.config
    w, h, kind, nsph, depth, spf, desc = CONFIGS[cfg]
    dispatch = spf == 1
    if dispatch:
        # progressive frames: frame 0 resets, one seed per frame
        spheres = rt.SphereCollection.generate(kind, nsph, 1)
        seeds = rt.frame_seeds(FRAME_SEED, args.warmup + args.steps + 5 * args.side)
        settings = rt.CameraSettings(max_depth=depth, samples_per_pixel=BENCH_SPP)
        cam0 = rt.SceneCamera.from_settings(settings, w, h, float(seeds[0]))
        cam_t = cam0.with_fields(camera_has_moved=0.0)
    else:
        # every step renders the golden 64-spp image from a reset accumulator
        g = dict(np.load(GOLDEN / f"{cfg.lower()}.npz"))
        spheres = rt.SphereCollection(g["spheres"])
        seeds = g["seeds"]
        cam0 = cam_t = rt.SceneCamera(g["camera"])
        assert cam0.camera_has_moved > 0.5 and len(seeds) == spf

    pipe = rt.ComputeShaderPipeline(device)
    pipe.set_scan_mode(args.scan)
    pipe.set_spheres(spheres)
    launch_mode = None
    if dispatch:
        # one `update` launch per frame, or (small rank shares) frame chains
        launch_mode = frame_launch_mode(args.frame_launch, w,
                                        rt.stripe_local_rows(h, rank, world))
        set_frame_launch(pipe, launch_mode)
    pipe.set_update_queues(args.queues)
    pipe.set_update_submit(args.submit)
    # the job's one gather: RCCL behind the C ABI (rt_comm_create + rt_gather_stripes)
    use_abi = world > 1 and backend == "nccl" and os.environ.get("RT_GATHER", "abi") == "abi"
    comm = StripeComm.from_process_group(pipe) if use_abi else None
    gather_how = ("rt_gather_stripes: ncclGather + de-interleave in librt_hip.so" if use_abi
                  else "none (one rank)" if world == 1
                  else f"torch.distributed.gather over {backend} + rt_deinterleave_stripes")
    r = StripeRenderer(pipe, w, h, rank, world, comm=comm)
    stream = torch.cuda.current_stream()
    local_px = w * min(r.rows, h)

    def step_block(n, first):
        if dispatch:
            off = 0 if first else args.warmup
            r.frames(cam0 if first else cam_t, spheres, seeds[off:off + n])
        else:
            for _ in range(n):
                r.frames(cam0, spheres, seeds)

    # Cold start (N=1 side line, before anything else ran on the GPU in this process): the
    # same W + K frames on scratch images, timed the same way — what the line's value would
    # be without the warm-up below.
    cold_start = None
    if args.side > 0 and world == 1 and dispatch:
        cr = StripeRenderer(pipe, w, h, rank, world, comm=None)
        torch.cuda.synchronize()
        if args.warmup:
            cr.frames(cam0, spheres, seeds[:args.warmup])
        torch.cuda.synchronize()
        tc0 = time.perf_counter()
        t_cold = timed(torch.cuda.current_stream(), lambda: cr.frames(
            cam0 if args.warmup == 0 else cam_t, spheres,
            seeds[args.warmup:args.warmup + args.steps]))
        dt_cold = time.perf_counter() - tc0
        ok, what = image_check(cfg, cr.local, args.warmup + args.steps, cam0, w, h)
        cold_start = {"us_per_step_events": round(t_cold / args.steps * 1e6, 2),
                "us_per_step_wall": round(dt_cold / args.steps * 1e6, 2),
                "Mrays_per_s": round(w * h * args.steps / dt_cold / 1e6, 1),
                "image_ok": ok, "image_check": what,
                "what": "the same warmup + steps frames on scratch images at process start, "
                        "before the --warm-ms warm-up (wall: synchronize on both sides)"}
        del cr
    # Warm-up (untimed, scratch images): a progressive render's steps run back to back in a
    # process that has long been issuing them; a 20-step timed region (~0.4 ms) right after
    # process start would otherwise time the chip's start from idle (K3: 22.2 against 16.2 µs
    # per update, profiles/r03/r03w_driver_warm.log; not the waves' clock, 1.83 GHz cold and 1.88
    # warm, profiles/r03/r03zb_stamps_single_k3_*.jsonl, nor the host's issue rate,
    # profiles/r03/r03zc_driver_cold_warm_hip_aql.log).  The same frames on
    # separate images: the timed images, their counts and the fixture check are untouched.
    warm_s = 0.0
    if args.warm_ms > 0:
        scratch = StripeRenderer(pipe, w, h, rank, world, comm=None)
        torch.cuda.synchronize()
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < args.warm_ms / 1e3:
            scratch.frames(cam0, spheres, seeds[:20] if dispatch else seeds)
            torch.cuda.synchronize()
        warm_s = time.perf_counter() - t_w
        del scratch
    # warmup (untimed); the dispatch configs' frame 0 resets the accumulator
    if args.warmup:
        step_block(args.warmup, True)
        # one untimed gather + de-interleave: RCCL sets up its point-to-point connections
        # and the de-interleave kernel's code object loads on first use, neither of which
        # belongs to a step (the timed region still ends with the job's own gather)
        r.finish()
    # (HIP events created before the timed region: their creation is host work, not steps)
    ev0, ev1, ev2, ev3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    for e in (ev0, ev1, ev2, ev3):
        e.record(stream)      # (torch creates an event at its first record: not in the region)

    # timed: K steps issued by rt_update_frames (timed_steps: opening barrier, each rank's
    # own clock around its steps and synchronize, the max over ranks; the closing barrier
    # reported apart)
    host_t = {} if os.environ.get("RT_TIMELINE") is not None else None   # tools/timeline.py

    def stamp(name):
        host_t[name] = (time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                        time.clock_gettime_ns(time.CLOCK_BOOTTIME))

    gate = StreamGate() if args.gate else None

    def run():
        if gate:
            gate.hold(stream)
        ev0.record(stream)
        try:
            step_block(args.steps, args.warmup == 0)
        finally:
            if gate:
                gate.release()
        ev1.record(stream)

    red_dev = "cuda" if backend == "nccl" else "cpu"
    ts = timed_steps(run, torch.cuda.synchronize, world, device=red_dev,
                     stamp=stamp if host_t is not None else None)
    dt = ts["dt"]
    info = pipe.last_launch_info()             # the last timed rt_update_frames call
    # the job's one gather of the finished tiles, timed on its own (barrier on both sides)
    t1 = time.perf_counter()
    ev2.record(stream)
    image = r.finish()
    ev3.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt_gather = time.perf_counter() - t1
    render_s, gather_s = ev0.elapsed_time(ev1) / 1e3, ev2.elapsed_time(ev3) / 1e3
    if world > 1:
        t = torch.tensor([dt, render_s, gather_s, dt_gather], dtype=torch.float64,
                         device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, render_s, gather_s, dt_gather = (float(x) for x in t.tolist())
    frames_total = (args.warmup + args.steps) if dispatch else spf
    image_ok, image_what = image_check(cfg, image, frames_total, cam0, w, h)
    # this rank's per-tile candidate lists of the timed camera (a tile with more than
    # kCandMax = 19 candidates has none: its camera rays scan the whole scene, same pixels)
    cand_stats = pipe.candidate_stats()

    # dispatch configs: the timed steps are ONE rt_update_frames call (one launch per
    # frame); 64-spp configs: one call per step, all alike
    total_launches = info["launches"] * (1 if dispatch else args.steps)
    launches_per_step = total_launches / args.steps
    # a one-frame update may run as `queues` concurrent launches (parts of the image on
    # their own streams): the roofline's unit is then the update, all its parts together
    queues = max(1, info.get("queues", 1))
    launch_s = ev0.elapsed_time(ev1) / 1e3 / max(1, total_launches // queues)
    value = w * h * spf * args.steps / dt / 1e6

    # roofline of the timed trace kernel
    kernel = info["kernel_name"]
    fpl = info["max_frames_per_launch"]
    bytes_launch = local_px * BYTES_PER_PIXEL_LAUNCH
    ref_bytes_launch = bytes_launch
    if launch_mode == "chain":
        # a frame chain carries fpl progressive updates but keeps the accumulator in
        # registers between them: it reads the input once (16 B per pixel) and writes every
        # frame's image (16 B per pixel per frame).  The reference's 32 B per pixel per frame
        # (a load and a store per dispatch) is reported beside it, not as `achieved`.
        bytes_launch = local_px * (16 * fpl + 16)
        ref_bytes_launch = local_px * BYTES_PER_PIXEL_LAUNCH * fpl
    pmc, pmc_path = load_pmc(cfg, kernel, fpl, queues) if world == 1 else (None, None)
    wgt, wgt_path = load_weighted(cfg, kernel, pmc_path) if pmc else (None, None)
    # (a summary's counts are per launch, i.e. per concurrent part: times the parts per update)
    pq = pmc.get("queues", 1) if pmc else 1
    roof = {"bound": "hbm", "achieved": round(bytes_launch / launch_s / 1e9, 1),
            "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(bytes_launch / launch_s / 1e9 / PEAK_HBM_GBS, 4),
            "traffic": pmc["hbm_bytes_per_launch"] * pq if pmc and "hbm_bytes_per_launch" in pmc
                       else None,
            "kernel": kernel, "kernel_avg_us": round(launch_s * 1e6, 2),
            "frames_per_launch": fpl, "launches_per_step": launches_per_step,
            "queues": queues, "submit": info.get("submit"),
            "algorithmic_bytes_per_launch": bytes_launch,
            "reference_bytes_per_launch": ref_bytes_launch,
            "binding": "valu",
            # the same bytes against the measured streaming floor of the pattern (no tracing)
            "practical_hbm": {"floor_GBs": RMW_FLOOR_GBS,
                              "frac": round(bytes_launch / launch_s / 1e9 / RMW_FLOOR_GBS, 4),
                              "source": "tools/rmw_floor.hip, profiles/archive/r02_rmw_floor.jsonl"}}
    if pmc and pmc.get("valu_insts_per_launch"):
        insts = pmc["valu_insts_per_launch"] * pq
        avail = SIMDS * CLOCK_GHZ * 1e9 * launch_s
        roof["valu"] = {"insts_per_launch": insts,
                        "issue_cycles": insts * VALU_ISSUE_CYCLES,
                        "available_cycles": round(avail),
                        "frac": round(insts * VALU_ISSUE_CYCLES / avail, 4),
                        "pmc": pmc_path,
                        "rule": "VALU wave-instructions x 2 cycles / (1024 SIMDs x 2.4 GHz x "
                                "kernel_avg_us)"}
        if wgt:
            # each PMC instruction class priced at the measured issue cost of the kernel's
            # own forms of that class (profiles/r0*_valu_rates.txt): the SIMD cycles the
            # VALU work holds, against what 1024 SIMDs offer at the 2.4-GHz peak clock
            wc = wgt["weighted_cycles"] * pq
            roof["valu"].update({
                "weighted_cycles": wc, "weighted_frac": round(wc / avail, 4),
                "weighted_frac_bounds": [round(b * pq / avail, 4)
                                         for b in wgt["weighted_cycles_bounds"]],
                "mean_cycles_per_valu": wgt["mean_cycles_per_valu"], "weighted": wgt_path})
            roof["binding_frac"] = roof["valu"]["weighted_frac"]

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
        "data": "synthetic (seeded scene + per-frame seeds; SURVEY §8d)"
                + ("" if backend == "nccl" else f"; REHEARSAL over {backend}, not a measurement")
                + ("; GATED issue (--gate): a profiling diagnostic, not a measurement"
                   if args.gate else ""),
        "config": {"workload": f"{cfg} {desc}, max_depth {depth}",
                   "width": w, "height": h, "spheres": nsph, "spp_per_step": spf,
                   "max_depth": depth, "parallelism": f"stripes{world}",
                   "scan": args.scan, "kernel": kernel,
                   "frame_launch": launch_mode or "fused_64",
                   "step": ("one progressive update (1 spp) of every pixel of the rank's "
                            "bands; " + {"dispatch": "one update launch per frame",
                                         "chain": "the steps' frames in fused launches, every "
                                                  "frame's image written",
                                         None: "64 frames per step"}[launch_mode])},
        "roofline": roof,
        "image_ok": image_ok,
        "image_check": image_what,
        # max over ranks: the K steps by HIP events; each rank's own wall time of its K steps
        # (value's time is their max); the closing barrier after them, outside value
        "timed_breakdown_ms": {"steps": round(render_s * 1e3, 4),
                               # host time of the steps' issue (this rank): the call returned
                               "host_issue": round(ts["issue"] * 1e3, 4),
                               "per_rank_ms": [round(x * 1e3, 4) for x in ts["per_rank"]],
                               "barrier_ms": round(ts["barrier_s"] * 1e3, 4)},
        # the job's output collection after the timed steps, and the job-level rate with it
        "gather": {"how": gather_how, "wall_ms": round(dt_gather * 1e3, 4),
                   "events_ms": round(gather_s * 1e3, 4),
                   "bytes_to_root": 16 * w * r.rows0 * (world - 1)},   # (padded bands)
        "job": {"wall_ms": round((dt + dt_gather) * 1e3, 4),
                "Mrays_per_s": round(w * h * spf * args.steps / (dt + dt_gather) / 1e6, 2),
                "what": "the K steps plus the one gather of the finished tiles"},
        "candidate_lists": cand_stats,
        "warm_up": {"ms": round(warm_s * 1e3, 2), "steps": args.warmup,
                    "what": "untimed update frames on scratch images before the warmup steps "
                            "(--warm-ms): the timed steps are a running render's, not a "
                            "freshly started process's first launches"},
    }

    if host_t is not None:
        # host clocks (CLOCK_MONOTONIC, CLOCK_BOOTTIME ns) at the timed region's start, when
        # the steps' issue returned, and after the closing synchronize: tools/timeline.py
        # places them on a rocprofv3 trace of the same run
        line["timeline_host"] = host_t

    # ---- side measurements (after the timed region and its image check) -------------
    side = {}
    if args.side > 0 and world == 1:
        base = args.warmup + args.steps
        if dispatch and depth == 1:
            # the reference algorithm (exhaustive scan) on further frames: its FP32 roofline
            pipe.set_scan_mode("exhaustive")
            t_exh = timed(stream, lambda: r.frames(cam_t, spheres, seeds[base:base + args.side]))
            t_exh /= args.side
            pipe.set_scan_mode(args.scan)
            flops = local_px * nsph * FLOP_PER_TEST
            side["fp32_exhaustive_scan"] = {
                "kernel": pipe.last_launch_info()["kernel_name"],
                "us_per_frame": round(t_exh * 1e6, 2),
                "achieved": round(flops / t_exh / 1e12, 3), "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s", "frac": round(flops / t_exh / 1e12 / PEAK_FP32_TFLOPS, 4),
                "flop_per_frame": flops}
            # the same frames fused (up to 64 per launch; K4's launches, the last two
            # frames' images written), after one untimed fused call that records the tile
            # costs the fused instances order by (the dispatch steps record none); then as a
            # frame chain writing every frame's image (what rank shares run)
            set_frame_launch(pipe, "dispatch")
            pipe.set_frames_per_launch(0)
            s1 = base + args.side
            r.frames(cam_t, spheres, seeds[s1:s1 + args.side])
            s1 += args.side
            t_f = timed(stream, lambda: r.frames(cam_t, spheres, seeds[s1:s1 + args.side]))
            fi = pipe.last_launch_info()
            set_frame_launch(pipe, "chain")
            s2 = s1 + args.side
            t_c = timed(stream, lambda: r.frames(cam_t, spheres, seeds[s2:s2 + args.side]))
            ci = pipe.last_launch_info()
            set_frame_launch(pipe, launch_mode)
            side["fused_frames"] = {"kernel": fi["kernel_name"],
                                    "frames_per_launch": fi["max_frames_per_launch"],
                                    "us_per_frame": round(t_f / args.side * 1e6, 2),
                                    "Mrays_per_s": round(local_px * args.side / t_f / 1e6, 1),
                                    "what": "the last two frames' images written per launch"}
            side["chain_frames"] = {"kernel": ci["kernel_name"],
                                    "frames_per_launch": ci["max_frames_per_launch"],
                                    "us_per_frame": round(t_c / args.side * 1e6, 2),
                                    "Mrays_per_s": round(local_px * args.side / t_c / 1e6, 1),
                                    "what": "every frame's image written (rt_set_frame_images "
                                            "EVERY): the structure of the rank shares' steps"}
            # moving camera: every frame a new camera (the reference's WASD movement resets
            # the accumulator, camera.rs:243-252, wgsl:345-350): candidate lists rebuilt
            # every frame, one update dispatch each
            a, b = r.buf[0], r.buf[1]
            cams = []
            for f in range(args.side):
                ang = math.radians(0.05 * (f + 1))
                st = rt.CameraSettings(max_depth=depth, samples_per_pixel=BENCH_SPP,
                                       look_from=(13.0 * math.cos(ang) - 3.0 * math.sin(ang),
                                                  2.0, 13.0 * math.sin(ang) + 3.0 * math.cos(ang)))
                cams.append(rt.SceneCamera.from_settings(st, w, h, float(seeds[f])))

            def cold():
                nonlocal a, b
                for c in cams:
                    pipe.update(a, b, w, h, c, spheres)
                    a, b = b, a
            t_c = timed(stream, cold) / args.side
            side["cold_camera"] = {"us_per_frame": round(t_c * 1e6, 2),
                                   "Mrays_per_s": round(local_px / t_c / 1e6, 1),
                                   "what": "a new camera every frame: candidate-list build "
                                           "(rt_candidates_kernel) + one update, reset "
                                           "accumulator; host issue included"}
        # presentation kernel on the final image: 16 B read + 4 B written/px
        if image is not None:
            out8 = torch.empty((h, w, 4), dtype=torch.uint8, device=image.device)
            pipe.present(image, w, h, "srgb", out8)
            t_p = timed(stream, lambda: [pipe.present(image, w, h, "srgb", out8)
                                         for _ in range(20)]) / 20
            side["present_rgba8"] = {"kernel": "rt_present_kernel<srgb>",
                                     "avg_us": round(t_p * 1e6, 2),
                                     "achieved": round(w * h * 20 / t_p / 1e9, 1),
                                     "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                     "frac": round(w * h * 20 / t_p / 1e9 / PEAK_HBM_GBS, 4)}
        if cold_start is not None:
            side["cold_start"] = cold_start
        if dispatch and depth == 1:
            # K2 / K5 / rank shares: each with its image check
            # (a side measurement that fails is reported in the line, never costs the line)
            try:
                side.update(driver_record_sides(device, stream, cfg,
                                                render_s / args.steps * 1e6))
            except Exception as e:          # noqa: BLE001
                torch.cuda.synchronize()
                side["side_error"] = f"{type(e).__name__}: {e}"[:400]
    line.update(side)

    if rank == 0:
        if world == 1 and args.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(cam0, spheres, w, h, args.cpu_seconds)
        print(json.dumps(line, default=_unserializable), flush=True)
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if world > 1:
        dist.destroy_process_group()
    pipe.close()


if __name__ == "__main__":
    main()
