"""Benchmark of the per-pixel ray-tracing hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config K3]

Configs (BASELINE.json `configs`):
  K2, K3 (default)  1920x1080, 3 / 500 spheres, max_depth 1.  A step is ONE progressive
                    `update` (wgsl:333-364): one camera sample per pixel of this rank's stripe
                    bands, accumulated into the RGBA32F image, the image of every frame written
                    to the ping-pong buffer the reference's dispatch writes (lib.rs:218-227,
                    366-374).  The K steps are one rt_update_frames call; the SAME launch
                    structure runs at every N (--frame-launch chain, default): fused launches
                    of up to 64 frames that write every frame's image (rt_set_frame_images
                    EVERY) — the reference's per-frame loop with only the launch boundary
                    between frames removed.  --frame-launch dispatch: one launch per frame,
                    the reference's own structure (reported as the `dispatch` side line at N=1).
  K4                1920x1080, 500 spheres, 64 spp anti-aliased accumulate, max_depth 1.  A
                    step is one 64-spp render from a reset accumulator (fused launches).
  K5                3840x2160, 500 spheres, 64 spp, 8 bounces — the multi-GPU config.  A step
                    is one 64-spp render (one 64-frame launch of the bounce instance).
With N GPUs (one process per GPU, torch.distributed.run) the image is split into 8-row bands
dealt round-robin; the steps have no collective (a rank's bands need nothing from another
rank).  After the K timed steps the finished tiles are gathered to rank 0 with ONE RCCL
gather + the de-interleave kernel (rt_gather_stripes, the ncclGather behind librt_hip.so's C
ABI; RT_GATHER=torch: torch.distributed.gather instead), timed on its own and reported as
`gather` and in the job-level rate `job`, not inside the K steps.

Timed region (timed_steps): barrier + synchronize, every rank reads CLOCK_MONOTONIC, issues
its K steps, synchronizes and reads it again; the job's time is max(end) - min(start) over
ranks (one host: one clock).  Nothing else runs inside it (no events: HIP event markers cost
~2.5 µs per region on an idle GPU, profiles/r06/r06b/).
value = W*H*spp_per_step*K camera rays / that time (Mrays/s, all ranks together).
segments_per_s: sphere_list_hit calls (SURVEY §8a "seg") per second — the fixture's exact
count for the rendered frames (the oracle counts them over the whole image).
image_ok: the timed image's SHA-256 (NaN canonical) against the fixture's whole-image digest
(tests/golden/*.npz `sha256`, oracle-generated), else its sampled pixels; rank shares are
checked band by band against the fixture's per-band digests (`band_sha`).
roofline: the timed kernel's launch duration over an identical repetition of the timed call
right after the region (the GPU still warm), from timing events its launches' own dispatch
packets carry (rt_set_launch_timing; one launch per frame: HIP events around the
repetition); `bound: "valu"` when a committed PMC
summary of that kernel instance exists (profiles/pmc_<round>_<config>.json): achieved = the
VALU lane-operations per second it issues (SQ_INSTS_VALU x 64 / launch time) against 1024
SIMDs x 32 lanes x 2.4 GHz (a wave64 VALU op holds a SIMD-32 two cycles); `hbm` = the
algorithmic bytes actually moved (chain: 16 B load once + 16 B store per pixel and frame;
dispatch: 16 B load + 16 B store per pixel and frame) against 8 TB/s, `traffic`
= the PMC bytes (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM).
cpu_baseline: the scalar C oracle on the box's host cores over a bounded sample (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import statistics
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
PEAK_VALU_TOPS = SIMDS * 32 * CLOCK_GHZ / 1e3   # 78.64 T lane-ops/s
FLOP_PER_TEST = 23            # oc 3, a 5, h 5, c 7, D 3 (wgsl:183-187)
BYTES_PER_PIXEL_LAUNCH = 32   # 16 B load + 16 B store of the accumulator (wgsl:339, 363)
FRAME_SEED = 0x5EED
BENCH_SPP = 65536             # the dispatch configs' spp cap (never reached; fixtures agree)
ROWS = 8                      # RT_STRIPE_ROWS
CANON_NAN = np.uint32(0x7FC00000)

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


def set_frame_launch(pipe, mode):
    """dispatch: one `update` launch per frame (rt_set_frames_per_launch(1)); chain: fused
    launches (up to 64 frames) that write every frame's image (rt_set_frame_images EVERY)."""
    pipe.set_frames_per_launch(1 if mode == "dispatch" else 0)
    pipe.set_frame_images("every" if mode == "chain" else "last_two")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="K3", choices=sorted(CONFIGS))
    ap.add_argument("--frame-launch", default=os.environ.get("RT_FRAME_LAUNCH", "chain"),
                    choices=["chain", "dispatch"],
                    help="K2/K3 steps at every N: the K frames in fused launches that write "
                         "every frame's image (chain, default), or one update launch per frame "
                         "(dispatch, the reference's structure)")
    ap.add_argument("--queues", type=int, default=int(os.environ.get("RT_QUEUES", "0")),
                    help="dispatch structure: concurrent parts per one-frame update "
                         "(rt_set_update_queues; 0 = the library's choice)")
    ap.add_argument("--submit", default=os.environ.get("RT_SUBMIT", "auto"),
                    choices=["auto", "hip", "aql"],
                    help="dispatch structure: how one-frame updates are submitted "
                         "(rt_set_update_submit)")
    ap.add_argument("--warm-ms", type=float, default=float(os.environ.get("RT_WARM_MS", "50")),
                    help="before the warmup steps, render this long with the same frames on "
                         "scratch images (untimed: a running render's steps, not a freshly "
                         "started process's first launches, are what is timed; 0 = off)")
    ap.add_argument("--gate", action="store_true",
                    help="diagnostic for profiled runs: hold the stream while the timed steps "
                         "are issued, then release it (StreamGate); the line is then not a "
                         "measurement")
    ap.add_argument("--scan", default="culled", choices=["culled", "exhaustive"],
                    help="sphere-list scan: exact culling (default) or the reference's "
                         "exhaustive linear walk; images are bit-identical")
    ap.add_argument("--side", type=int, default=20,
                    help="frames for each side measurement (0 = none)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU baseline budget in seconds (0 = skip)")
    a = ap.parse_args(argv)
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
    in CPUs, or None when unlimited or unreadable."""
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
    every CPU the process can run on at once (~seconds/5, 2-row bands)."""
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
    # schedules 16: 256 threads there would measure the oversubscription)
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
                          "cores; all_cores: min(affinity set, cgroup CPU quota) threads"}


def load_pmc(config, kernel, frames_per_launch, queues=1):
    """The newest committed rocprofv3 PMC summary of the timed kernel (tools/pmc_bench.sh),
    if it was taken for the same kernel instance at the same frames per launch and the same
    concurrent parts per update (a summary's per-launch counts are one part's), and its
    path."""
    for rnd in ("r06", "r05", "r04", "r03", "r02"):
        p = ROOT / "profiles" / f"pmc_{rnd}_{config}.json"
        if not p.exists():
            continue
        d = json.loads(p.read_text())
        if (d.get("kernel") == kernel and d.get("frames_per_launch") == frames_per_launch
                and d.get("queues", 1) == queues):
            return d, p.relative_to(ROOT).as_posix()
    return None, None


def load_weighted(config, kernel, pmc_path):
    """The weighted VALU cycles per launch of the timed kernel (tools/valu_weighted.py: the
    PMC's instruction classes priced at the kernel's own forms' measured issue costs), if
    committed for that kernel and that PMC summary, and its path."""
    for rnd in ("r06",):
        p = ROOT / "profiles" / f"valu_weighted_{rnd}_{config}.json"
        if not p.exists():
            continue
        d = json.loads(p.read_text())
        if d.get("kernel") == kernel and d.get("pmc") == pmc_path:
            return d, p.relative_to(ROOT).as_posix()
    return None, None


# ---- image checks against the committed fixtures ---------------------------------------
def canon_sha(a) -> str:
    """SHA-256 of a float32 image's bytes with every NaN as 0x7FC00000 (the parity tests
    treat any NaN as equal to any NaN; tests/golden/make_band_digests.py digests the same)."""
    a = np.ascontiguousarray(a, np.float32).copy()
    a.view(np.uint32)[np.isnan(a)] = CANON_NAN
    return hashlib.sha256(a.tobytes()).hexdigest()


def _fixture(config):
    name = f"bench_{config.lower()}.npz" if config in ("K2", "K3") else f"{config.lower()}.npz"
    return dict(np.load(GOLDEN / name))


def _fixture_at(g, frames):
    """(whole-image sha, band digests [bands, 32] or None, sampled pixels, segments) of a
    fixture after `frames` frames, or None when it holds no such frame count."""
    if "frame_counts" in g:                       # bench_k2 / bench_k3: several frame counts
        counts = [int(c) for c in g["frame_counts"]]
        if frames not in counts:
            return None
        k = counts.index(frames)
        sha = str(g["sha256"][k]) if "sha256" in g else None
        bands = g["band_sha"][k] if "band_sha" in g else None
        segs = int(g["segments"][k]) if "segments" in g else None
        return sha, bands, g["pixels"][k], segs
    sha = str(g["sha256"]) if "sha256" in g else None
    segs = int(g["segments"]) if "segments" in g else None
    return sha, g.get("band_sha"), g["pixels"], segs


def _pixels_same(got, want):
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    return bool(same.all())


def image_check(config, image, frames, cam):
    """The timed image against the committed fixture: its whole-image digest when the
    fixture has one for this frame count, else its sampled pixels."""
    if image is None:
        return None, "not the gathering rank"
    g = _fixture(config)
    if not np.array_equal(g["camera"].view(np.uint32), cam.blob.view(np.uint32)):
        return False, "camera blob differs from the fixture's"
    at = _fixture_at(g, frames)
    if at is None:
        return None, f"no fixture for {frames} frames"
    sha, _, want, _ = at
    img = image.detach().cpu().numpy()
    if sha is not None:
        return canon_sha(img) == sha, f"whole-image SHA-256 after {frames} frames"
    return _pixels_same(img[g["py"], g["px"]], want), \
        f"{want.shape[0]} sampled pixels after {frames} frames"


def stripe_bands(height, rank, world):
    """The global 8-row bands of `rank` (band b -> rank b % world), in local order."""
    return list(range(rank, (height + ROWS - 1) // ROWS, world))


def share_check(config, local, frames, bands):
    """A rank's share (its local rows: global band bands[j] at local rows 8j..8j+7) against
    the fixture: every band's digest when the fixture has per-band digests, else the sampled
    pixels that fall in those bands.  None when no fixture covers the frame count."""
    g = _fixture(config)
    at = _fixture_at(g, frames)
    if at is None:
        return None
    _, band_sha, want, _ = at
    img = local.detach().cpu().numpy()
    if band_sha is not None:
        for j, b in enumerate(bands):
            d = np.frombuffer(bytes.fromhex(canon_sha(img[ROWS * j:ROWS * (j + 1)])), np.uint8)
            if not np.array_equal(d, band_sha[b]):
                return False
        return True
    py, px = g["py"], g["px"]
    where = {b: j for j, b in enumerate(bands)}
    mine = np.array([int(y) // ROWS in where for y in py])
    if not mine.any():
        return None
    ly = np.array([where[int(y) // ROWS] * ROWS + int(y) % ROWS for y in py[mine]])
    return _pixels_same(img[ly, px[mine]], want[mine])


def fixture_segments(config, frames):
    at = _fixture_at(_fixture(config), frames)
    return at[3] if at else None


# ---- timing --------------------------------------------------------------------------
def over_ranks(share, world):
    """share(rank) -> {"us_per_step", ...} for every rank of a world-size run, timed one after
    another on this GPU: the job's step is the slowest rank's (bench.py --gpus N takes the
    max over ranks), so `us_per_step` is the max; each rank's own time and check are kept."""
    per = [share(r) for r in range(world)]
    slow = max(range(world), key=lambda r: per[r]["us_per_step"])
    out = dict(per[slow])
    us = [d["us_per_step"] for d in per]
    out.update({"us_per_step": per[slow]["us_per_step"], "max_over_ranks": True,
                "slowest_rank": slow, "rank_us": us, "rank0_us": per[0]["us_per_step"],
                "rank_spread": round(max(us) / min(us) - 1.0, 4) if min(us) > 0 else None,
                "image_ok": all(d["image_ok"] for d in per) if all(
                    d["image_ok"] is not None for d in per) else None})
    return out


def timed_steps(run, sync, world, barrier=None, device=None, stamp=None, wait=None):
    """The timed region of the K steps.  Every rank leaves an opening barrier (then
    synchronises), reads CLOCK_MONOTONIC, issues the steps (`run`), synchronises (`wait`,
    default sync) and reads the clock again.  At N > 1 the ranks' start and end stamps are
    all-gathered and the job's time is max(end) - min(start): all ranks run on one host, so
    one clock covers them, and the skew with which they leave the opening barrier stays
    inside the job's time.  The closing barrier follows outside that time and is reported on
    its own (`barrier_s`).  Returns {"dt": the job's time, "per_rank": [each rank's own
    end - start], "max_rank_s": their max, "start_skew_s": max - min start, "issue": this
    rank's host issue time, "barrier_s": max over ranks of the closing barrier}.
    `stamp(name)` (optional) is called at the start, when the issue returns and after the
    synchronise."""
    barrier = barrier or dist.barrier
    wait = wait or sync
    clock = time.clock_gettime_ns
    mono = time.CLOCK_MONOTONIC
    sync()
    if world > 1:
        barrier()
        sync()
    if stamp:
        stamp("t0")
    t0 = clock(mono)
    run()
    t_issued = clock(mono)
    if stamp:
        stamp("issued")
    wait()
    t1 = clock(mono)
    if stamp:
        stamp("synced")
    starts, ends, bars = [t0], [t1], [0]
    if world > 1:
        tb = clock(mono)
        barrier()
        sync()
        bar = clock(mono) - tb
        t = torch.tensor([t0, t1, bar], dtype=torch.int64, device=device)
        got = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(got, t)
        starts = [int(g[0]) for g in got]
        ends = [int(g[1]) for g in got]
        bars = [int(g[2]) for g in got]
    per_rank = [(e - s) / 1e9 for s, e in zip(starts, ends)]
    return {"dt": (max(ends) - min(starts)) / 1e9, "per_rank": per_rank,
            "max_rank_s": max(per_rank), "start_skew_s": (max(starts) - min(starts)) / 1e9,
            "issue": (t_issued - t0) / 1e9, "barrier_s": max(bars) / 1e9}


class StreamGate:
    """--gate (diagnostic, never a measurement): the stream waits on a host-memory word
    (hipStreamWaitValue32) while the timed steps are issued, and the host opens it after the
    issue, so that the GPU runs the steps back to back however slowly the host issues them
    (under rocprofv3's kernel trace every dispatch costs the host ~8 µs more).  Uses the HIP
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
    """HIP events on `stream` around fn(), seconds (the side lines' and the roofline's kernel
    time; never inside the main timed region)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3


def wall(fn):
    """Host wall clock around fn() and a synchronize, seconds (synchronized before)."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def runtime_floor_us(reps=50):
    """The host's round trip to an idle GPU: one 1-element kernel (torch's fill) launched and
    synchronized, median µs — the fixed cost any timed region of one launch pays."""
    x = torch.zeros(1, device="cuda")
    t = []
    for _ in range(reps):
        t.append(wall(lambda: x.fill_(1.0)))
    return round(statistics.median(t) * 1e6, 2)


def roofline(kernel, launch_s, bytes_launch, pmc, pmc_path, parts=1, extra=None,
             ref_bytes=None, weighted=None):
    """The roofline object of the timed kernel: HBM bytes moved against 8 TB/s, and — when a
    PMC summary of that kernel instance is committed — the VALU issue it measured against
    the VALU peak (then the bound: these kernels issue far more VALU than they move bytes).
    ref_bytes: the reference's per-dispatch traffic for the same frames (32 B per pixel and
    frame, SURVEY §8d B_comp), reported beside the bytes actually moved, labelled."""
    gbs = bytes_launch / launch_s / 1e9
    hbm = {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": round(gbs / PEAK_HBM_GBS, 4),
           "algorithmic_bytes_per_launch": int(bytes_launch),
           "practical_floor_frac": round(gbs / RMW_FLOOR_GBS, 4)}
    if ref_bytes and ref_bytes != bytes_launch:
        hbm["reference_semantics"] = {
            "bytes_per_launch": int(ref_bytes),
            "frac": round(ref_bytes / launch_s / 1e9 / PEAK_HBM_GBS, 4),
            "what": "the reference's 32 B per pixel and frame (a load and a store per "
                    "dispatch, SURVEY §8d B_comp progressive) over the same time: traffic "
                    "the fused kernel does not move, an effective-bandwidth figure only"}
    traffic = None
    if pmc and "hbm_bytes_per_launch" in pmc:
        traffic = pmc["hbm_bytes_per_launch"] * parts
        hbm["traffic_GBs"] = round(traffic / launch_s / 1e9, 1)
    roof = {"bound": "hbm", **hbm, "traffic": traffic, "kernel": kernel,
            "kernel_avg_us": round(launch_s * 1e6, 2)}
    if pmc and pmc.get("valu_insts_per_launch"):
        insts = pmc["valu_insts_per_launch"] * parts
        ach = insts * 64 / launch_s / 1e12
        roof = {"bound": "valu", "achieved": round(ach, 3), "peak": round(PEAK_VALU_TOPS, 2),
                "unit": "TOP/s (VALU lane-ops)",
                "frac": round(insts * VALU_ISSUE_CYCLES / (SIMDS * CLOCK_GHZ * 1e9 * launch_s), 4),
                "traffic": traffic, "kernel": kernel, "kernel_avg_us": round(launch_s * 1e6, 2),
                "valu_insts_per_launch": insts, "pmc": pmc_path,
                "rule": "frac = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x "
                        "kernel_avg_us); achieved = SQ_INSTS_VALU x 64 lanes / kernel_avg_us",
                "hbm": hbm}
        if weighted:
            wd, wpath = weighted
            wc = wd["weighted_cycles"] * parts
            roof["weighted"] = {
                "frac": round(wc / (SIMDS * CLOCK_GHZ * 1e9 * launch_s), 4),
                "cycles_per_launch": wc, "mean_cycles_per_valu": wd["mean_cycles_per_valu"],
                "file": wpath,
                "what": "each VALU instruction class priced at the measured issue cost of the "
                        "kernel's own forms (tools/valu_weighted.py): the SIMD cycles the VALU "
                        "work holds, against 1024 SIMDs x 2.4 GHz"}
    if extra:
        roof.update(extra)
    return roof


# ---- side measurements of the N=1 record -----------------------------------------------
def _setup(cfg):
    w, h, kind, nsph, depth, spf, _ = CONFIGS[cfg]
    if spf == 1:
        sc = rt.SphereCollection.generate(kind, nsph, 1)
        seeds = rt.frame_seeds(FRAME_SEED, 220)
        st = rt.CameraSettings(max_depth=depth, samples_per_pixel=BENCH_SPP)
        cam = rt.SceneCamera.from_settings(st, w, h, float(seeds[0]))
    else:
        g = _fixture(cfg)
        sc, seeds, cam = rt.SphereCollection(g["spheres"]), g["seeds"], rt.SceneCamera(g["camera"])
    return w, h, sc, seeds, cam


def driver_record_sides(device, stream, main_cfg):
    """Side measurements for the driver's N=1 record (after the timed region), each with its
    image check:
      dispatch     the main config with one update launch per frame (the reference's own
                   structure), 5 + 20 frames, µs per update by events and wall, HBM fraction;
      k2 / k3      the other per-update config the same way;
      k4, k5       one 64-spp step each (K5: with segments/s);
      rank_shares  every rank's share of K3 (frame chains, the main line's structure) and of
                   K5 at 1 / 2 / 4 / 8 ranks timed alone on this GPU, WALL-CLOCK around the
                   call and a synchronize as timed_steps times a rank, at the driver's 20
                   steps and at bench.py's default 200; the job's step is the slowest rank's
                   (max over ranks); efficiency against the 1-rank share timed the same way."""
    out = {}
    pipe = rt.ComputeShaderPipeline(device)
    try:
        def share_run(cfg, world, mode, rank=0, steps=20, reps=5, warm_s=0.05):
            # reset + warm frames, then `steps` timed frames in one call, as each rank of
            # bench.py --gpus N runs them after its warm-up (untimed frames on scratch images
            # first: the share's lists, order and code, and warm_s of the same frames)
            w, h, sc, seeds, cam = _setup(cfg)
            set_frame_launch(pipe, mode)
            cam_t = cam.with_fields(camera_has_moved=0.0)
            lead = 5 if steps <= 20 else 20
            scratch = StripeRenderer(pipe, w, h, rank, world)
            t_w = time.perf_counter()
            while True:
                scratch.frames(cam, sc, seeds[:20])
                torch.cuda.synchronize()
                if time.perf_counter() - t_w >= warm_s:
                    break
            del scratch
            r = StripeRenderer(pipe, w, h, rank, world)
            walls, evs = [], []
            for k in range(reps):
                r.frames(cam, sc, seeds[:lead])
                walls.append(wall(lambda: r.frames(cam_t, sc, seeds[lead:lead + steps])) / steps)
            ok = share_check(cfg, r.local, lead + steps, stripe_bands(h, rank, world))
            # the kernel time of three more such calls: frame chains from the timing events
            # their launches carry (rt_set_launch_timing — ≈ 9 µs slower per call, so never in
            # the wall-clock calls), one-frame launches (which carry none) by HIP events
            pipe.set_launch_timing(mode == "chain")
            for k in range(3):
                r.frames(cam, sc, seeds[:lead])
                if mode == "chain":
                    wall(lambda: r.frames(cam_t, sc, seeds[lead:lead + steps]))
                    evs.append(pipe.last_call_kernel_time()[0] / steps)
                else:
                    evs.append(timed(stream, lambda: r.frames(cam_t, sc, seeds[lead:lead + steps])) / steps)
            pipe.set_launch_timing(False)
            info = pipe.last_launch_info()
            t = statistics.median(walls)
            return {"us_per_step": round(t * 1e6, 3),
                    "events_us_per_step": round(statistics.median(evs) * 1e6, 3),
                    "kernel": info["kernel_name"],
                    "launches_per_step": round(info["launches"] / steps, 3),
                    "wall_runs_us": [round(x * 1e6, 3) for x in walls],
                    "image_ok": ok}

        def k5_run(world, rank=0, partition=None):
            w, h, sc, seeds, cam = _setup("K5")
            pipe.set_frames_per_launch(0)
            pipe.set_frame_images("last_two")
            r = StripeRenderer(pipe, w, h, rank, world, partition=partition)
            r.frames(cam, sc, seeds)                   # records the tile costs
            r.frames(cam, sc, seeds)                   # builds the order (and its buffers)
            # (each call restarts from the camera's reset; wall-clock, the median of five)
            runs = sorted(wall(lambda: r.frames(cam, sc, seeds)) for _ in range(5))
            info = pipe.last_launch_info()
            return {"us_per_step": round(runs[2] * 1e6, 1),
                    "runs_us": [round(x * 1e6, 1) for x in runs],
                    "kernel": info["kernel_name"],
                    "bands": list(r.bands),
                    "image_ok": share_check("K5", r.local, 64, r.band_list())}

        # the reference's structure (one launch per frame) for the main and the other config
        other = "K2" if main_cfg == "K3" else "K3"
        for cfg, key in ((main_cfg, "dispatch"), (other, other.lower())):
            pipe.set_update_queues(0)
            d = share_run(cfg, 1, "dispatch")
            w, h = CONFIGS[cfg][:2]
            ev = d["events_us_per_step"]
            out[key] = dict(d, config=cfg, Mrays_per_s=round(w * h / d["us_per_step"], 1),
                            hbm_frac_events=round(w * h * BYTES_PER_PIXEL_LAUNCH /
                                                  (ev * 1e3) / PEAK_HBM_GBS, 4),
                            what=f"{cfg}: 5 + 20 frames from a reset, one update launch per "
                                 f"frame (the reference's dispatch structure); us_per_step wall "
                                 f"(synchronize on both sides), events_us_per_step by HIP "
                                 f"events; HBM: 32 B per pixel per update")
        # K4: one 64-spp 1920x1080 render from a reset (fused frames)
        w4, h4, sc4, seeds4, cam4 = _setup("K4")
        pipe.set_frames_per_launch(0)
        pipe.set_frame_images("last_two")
        r4 = StripeRenderer(pipe, w4, h4, 0, 1)
        for _ in range(2):
            r4.frames(cam4, sc4, seeds4)               # costs recorded, order built
        runs4 = sorted(wall(lambda: r4.frames(cam4, sc4, seeds4)) for _ in range(5))
        info4 = pipe.last_launch_info()
        ok4, what4 = image_check("K4", r4.local[:h4], 64, cam4)
        out["k4"] = {"us_per_step": round(runs4[2] * 1e6, 1),
                     "us_per_frame": round(runs4[2] / 64 * 1e6, 2),
                     "runs_us": [round(x * 1e6, 1) for x in runs4],
                     "kernel": info4["kernel_name"], "launches_per_step": info4["launches"],
                     "image_ok": ok4, "image_check": what4,
                     "Mrays_per_s": round(w4 * h4 * 64 / (runs4[2] * 1e6), 1),
                     "what": "K4: one 64-spp 1920x1080 render from a reset (fused frames, "
                             "cost-ordered after two untimed renders), wall, the median of five"}
        del r4
        k5 = k5_run(1)
        # the whole image's per-band costs, as its first (cost-recording) launch measured them
        w5, h5 = CONFIGS["K5"][:2]
        k5_costs = pipe.band_costs(w5, h5, (0, 1, h5 // ROWS))
        segs5 = fixture_segments("K5", 64)
        out["k5"] = dict(k5, Mrays_per_s=round(3840 * 2160 * 64 / k5["us_per_step"], 1),
                         segments_per_s=(round(segs5 / (k5["us_per_step"] / 1e6), 1)
                                         if segs5 else None),
                         what="one 64-spp 3840x2160 depth-8 step (one 64-frame bounce launch, "
                              "cost-ordered by the steps before), wall, the median of five")

        # rank shares: the main line's structure (frame chains) at every N, wall-clock
        shares = {}
        for steps in (20, 200):
            rows = {}
            for world in (1, 2, 4, 8):
                rows[str(world)] = over_ranks(
                    lambda rk: share_run("K3", world, "chain", rk, steps=steps), world)
            one = rows["1"]["us_per_step"]
            for k, v in rows.items():
                v["efficiency"] = round(one / (int(k) * v["us_per_step"]), 4)
                if v.get("events_us_per_step"):
                    v["events_efficiency"] = round(rows["1"]["events_us_per_step"] /
                                                   (int(k) * v["events_us_per_step"]), 4)
            shares[f"K3_chain_{steps}_steps"] = rows
        # the fixed cost of one call: wall(steps) = fixed + steps * per_step, from the two
        # step counts of the slowest rank
        fixed = {}
        for k in ("1", "2", "4", "8"):
            a, b = (shares[f"K3_chain_{s}_steps"][k]["us_per_step"] for s in (20, 200))
            per = (200 * b - 20 * a) / 180
            fixed[k] = {"fixed_us": round(20 * a - 20 * per, 2), "per_step_us": round(per, 3)}
        shares["K3_call_model"] = fixed
        shares["runtime_floor_us"] = runtime_floor_us()
        k5rows = {"1": {"us_per_step": k5["us_per_step"], "image_ok": k5["image_ok"]}}
        for world in (2, 4, 8):
            k5rows[str(world)] = over_ranks(lambda rk: k5_run(world, rk), world)
        for k, v in k5rows.items():
            v["efficiency"] = round(k5["us_per_step"] / (int(k) * v["us_per_step"]), 4)
        # the 8-rank shares once more: how far a rank's own time moves between two timings
        # of the same share (run-to-run noise against the spread between ranks)
        k5rows["8"]["rank_us_repeat"] = [k5_run(8, rk)["us_per_step"] for rk in range(8)]
        shares["K5_fused_64"] = k5rows
        # cost-balanced contiguous ranges: rt_partition_bands over the whole image's band
        # costs, then two calibration rounds — each range's band costs rescaled by the time
        # its share took over the cost it was given (a share's time is not its tiles' costs
        # in the whole image: placement, tails), re-cut — and the final partition timed
        # afresh like the round-robin shares
        brows = {"1": k5rows["1"]}
        for world in (2, 4, 8):
            adj = np.array(k5_costs, np.float64)
            hist = []
            for it in range(3):
                part = rt.partition_bands(adj, world)
                if it == 2:
                    break
                t = [k5_run(world, rk, part)["us_per_step"] for rk in range(world)]
                hist.append({"partition": [list(b) for b in part], "rank_us": t})
                for (f, _, c), tr in zip(part, t):
                    cs = adj[f:f + c].sum()
                    if c and cs > 0:
                        adj[f:f + c] *= tr / cs
            brows[str(world)] = over_ranks(lambda rk: k5_run(world, rk, part), world)
            brows[str(world)]["partition"] = [list(b) for b in part]
            brows[str(world)]["calibration"] = hist
        for k, v in brows.items():
            v["efficiency"] = round(k5["us_per_step"] / (int(k) * v["us_per_step"]), 4)
        shares["K5_balanced_64"] = brows
        shares["what"] = (
            "every rank's stripe share (8-row bands dealt round-robin) timed alone on this GPU "
            "in the main line's structure, each rank's step of bench.py --gpus N: us_per_step = "
            "the slowest rank's (max_over_ranks; rank_us lists them all) wall-clock per step "
            "(host clock around one call of the steps and a synchronize, the median of five "
            "calls; events_us_per_step: the kernel time of three more calls, from the timing "
            "events their launches carry, rt_set_launch_timing); efficiency = the 1-rank "
            "time / (N x that time) in the same structure and step count; K3 at the driver's 20 "
            "steps and at the default 200; K3_call_model: fixed_us + steps x per_step_us fitted "
            "to the two; runtime_floor_us: one 1-element kernel launched and synchronized on "
            "the idle GPU (the floor of any call's fixed cost); K5: one 64-spp step per call, "
            "K5_balanced_64 with contiguous band ranges cut by rt_partition_bands from the "
            "whole image's per-band costs (rt_band_costs), calibrated twice by the ranges' "
            "measured times, instead of round-robin bands")
        out["rank_shares"] = shares
    finally:
        pipe.close()
    return out


def _unserializable(o):
    """json default: a value the line cannot hold is named, not fatal."""
    return f"<{type(o).__name__} {getattr(o, '__name__', '')}>"


def main(argv=None):
    args = parse(argv)
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
        seeds = rt.frame_seeds(FRAME_SEED, args.warmup + args.steps + 3 * args.side)
        settings = rt.CameraSettings(max_depth=depth, samples_per_pixel=BENCH_SPP)
        cam0 = rt.SceneCamera.from_settings(settings, w, h, float(seeds[0]))
        cam_t = cam0.with_fields(camera_has_moved=0.0)
    else:
        # every step renders the golden 64-spp image from a reset accumulator
        g = _fixture(cfg)
        spheres = rt.SphereCollection(g["spheres"])
        seeds = g["seeds"]
        cam0 = cam_t = rt.SceneCamera(g["camera"])
        assert cam0.camera_has_moved > 0.5 and len(seeds) == spf

    pipe = rt.ComputeShaderPipeline(device)
    pipe.set_scan_mode(args.scan)
    pipe.set_spheres(spheres)
    launch_mode = None
    if dispatch:
        launch_mode = args.frame_launch
        set_frame_launch(pipe, launch_mode)
    pipe.set_update_queues(args.queues)
    pipe.set_update_submit(args.submit)
    # the job's one gather: RCCL behind the C ABI (rt_comm_create + rt_gather_stripes)
    use_abi = world > 1 and backend == "nccl" and os.environ.get("RT_GATHER", "abi") == "abi"
    comm, comm_error = None, None
    if use_abi:
        # the gather runs after the timed region: should librt_hip.so's communicator fail to
        # come up on every rank (e.g. no loadable librccl), the job gathers through
        # torch.distributed's RCCL group instead and says so in `gather.how`
        try:
            comm = StripeComm.from_process_group(pipe)
        except Exception as e:              # noqa: BLE001
            comm_error = f"{type(e).__name__}: {e}"[:200]
        ok = torch.tensor([0 if comm_error else 1], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0 and comm is not None:
            comm.close()
            comm, comm_error = None, comm_error or "another rank's rt_comm_create failed"
        use_abi = comm is not None
    gather_how = ("rt_gather_stripes: ncclGather + de-interleave in librt_hip.so" if use_abi
                  else "none (one rank)" if world == 1
                  else f"torch.distributed.gather over {backend} + rt_deinterleave_stripes"
                  + (f" (rt_comm_create failed: {comm_error})" if comm_error else ""))
    r = StripeRenderer(pipe, w, h, rank, world, comm=comm)
    stream = torch.cuda.current_stream()
    local_px = w * min(r.rows, h)

    def step_block(rend, n, first):
        if dispatch:
            off = 0 if first else args.warmup
            rend.frames(cam0 if first else cam_t, spheres, seeds[off:off + n])
        else:
            for _ in range(n):
                rend.frames(cam0, spheres, seeds)

    # Warm-up (untimed, scratch images): a progressive render's steps run back to back in a
    # process that has long been issuing them; a 20-step timed region (~0.3 ms) right after
    # process start would otherwise time the chip's start from idle.  The same
    # frames on separate images: the timed images, their counts and the fixture check are
    # untouched.
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
        step_block(r, args.warmup, True)
        # one untimed gather + de-interleave: RCCL sets up its point-to-point connections
        # and the de-interleave kernel's code object loads on first use, neither of which
        # belongs to a step (the job's own gather follows the timed steps)
        r.finish()

    host_t = {} if os.environ.get("RT_TIMELINE") is not None else None   # tools/timeline.py

    def stamp(name):
        host_t[name] = (time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                        time.clock_gettime_ns(time.CLOCK_BOOTTIME))

    gate = StreamGate() if args.gate else None
    # the roofline's kernel time: an identical repetition of the timed call right after the
    # region (the GPU still warm) on a scratch renderer allocated here — its fused launches
    # carrying timing events in their own dispatch packets (rt_set_launch_timing; that launch
    # path costs ≈ 9 µs more per call, so it never runs inside the region), one-launch-per-
    # frame steps (which carry none) between HIP events
    launch_timing = launch_mode != "dispatch"
    rep = StripeRenderer(pipe, w, h, rank, world, comm=None)

    def run():
        if gate:
            gate.hold(stream)
        try:
            step_block(r, args.steps, args.warmup == 0)
        finally:
            if gate:
                gate.release()

    # timed: the K steps (timed_steps: opening barrier, CLOCK_MONOTONIC around each rank's
    # steps and synchronize, the job's time max(end) - min(start); the closing barrier apart)
    red_dev = "cuda" if backend == "nccl" else "cpu"
    ts = timed_steps(run, torch.cuda.synchronize, world, device=red_dev,
                     stamp=stamp if host_t is not None else None)
    dt = ts["dt"]
    info = pipe.last_launch_info()             # the last timed rt_update_frames call
    if launch_timing:
        # the repetition's last call: all K steps (K2/K3 chains) or one 64-spp step
        if dispatch:
            step_block(rep, args.warmup, True)
            pipe.set_launch_timing(True)
            step_block(rep, args.steps, args.warmup == 0)
        else:
            pipe.set_launch_timing(True)
            step_block(rep, 1, False)
        k_s, k_launches = pipe.last_call_kernel_time()
        pipe.set_launch_timing(False)
        torch.cuda.synchronize()
        del rep
        kernel_how = {"how": "an identical repetition of the timed call right after the "
                             "region, timing events carried by its launches' dispatch "
                             "packets (rt_set_launch_timing)", "launches": k_launches,
                      "us": round(k_s * 1e6, 3)}
    else:
        # HIP events over an identical repetition of the timed call (the same reset and
        # frames on the scratch renderer), issued at once while the GPU is as warm as in the
        # region (a host-side check first would let its clock drop)
        if dispatch:
            step_block(rep, args.warmup, True)
        rep_s = timed(stream, lambda: step_block(rep, args.steps, args.warmup == 0))
        del rep
        kernel_how = {"how": "HIP events over an identical repetition of the timed call",
                      "us_per_step": round(rep_s / args.steps * 1e6, 3)}
    # the job's one gather of the finished tiles, timed on its own (barrier on both sides)
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t1 = time.perf_counter()
    e2.record(stream)
    image = r.finish()
    e3.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt_gather = time.perf_counter() - t1
    gather_s = e2.elapsed_time(e3) / 1e3
    if world > 1:
        t = torch.tensor([gather_s, dt_gather], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gather_s, dt_gather = (float(x) for x in t.tolist())
    frames_total = (args.warmup + args.steps) if dispatch else spf
    image_ok, image_what = image_check(cfg, image, frames_total, cam0)
    share_ok = share_check(cfg, r.local, frames_total, stripe_bands(h, rank, world))
    if world > 1:
        flag = torch.tensor([{True: 1, False: 0, None: 2}[share_ok]], dtype=torch.int32,
                            device=red_dev)
        got = [torch.zeros_like(flag) for _ in range(world)]
        dist.all_gather(got, flag)
        vals = [int(g[0]) for g in got]
        share_ok = None if 2 in vals else all(v == 1 for v in vals)
    cand_stats = pipe.candidate_stats()

    total_launches = info["launches"] * (1 if dispatch else args.steps)
    launches_per_step = total_launches / args.steps
    queues = max(1, info.get("queues", 1))
    if launch_timing:
        launch_s = k_s / max(1, k_launches)
    else:
        launch_s = rep_s / max(1, total_launches // queues)
    value = w * h * spf * args.steps / dt / 1e6

    kernel = info["kernel_name"]
    fpl = info["max_frames_per_launch"]
    if launch_mode == "chain":
        # a frame chain carries fpl progressive updates, the accumulator in registers between
        # them: it reads the input once (16 B per pixel) and writes every frame's image (16 B
        # per pixel per frame)
        bytes_launch = local_px * (16 * fpl + 16)
    elif dispatch:
        bytes_launch = local_px * BYTES_PER_PIXEL_LAUNCH
    else:
        # 64-spp steps: one read and the last two frames' images per launch
        bytes_launch = local_px * 16 * 3
    pmc, pmc_path = load_pmc(cfg, kernel, fpl, queues) if world == 1 else (None, None)
    pq = pmc.get("queues", 1) if pmc else 1
    ref_bytes = local_px * BYTES_PER_PIXEL_LAUNCH * fpl   # the reference: one dispatch per frame
    wgt = load_weighted(cfg, kernel, pmc_path) if pmc else (None, None)
    roof = roofline(kernel, launch_s, bytes_launch, pmc, pmc_path, pq, ref_bytes=ref_bytes,
                    weighted=wgt if wgt[0] else None,
                    extra={"frames_per_launch": fpl, "launches_per_step": launches_per_step,
                           "queues": queues, "submit": info.get("submit"),
                           "kernel_time": kernel_how})

    segs = fixture_segments(cfg, frames_total)
    if dispatch and depth == 1:
        seg_step = w * h            # one sphere_list_hit per camera ray at max_depth 1
    elif segs:
        seg_step = segs             # one step = the fixture's 64-spp render
    else:
        seg_step = None
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
                                         "chain": "the K steps' frames in fused launches, every "
                                                  "frame's image written",
                                         None: "64 frames per step"}[launch_mode])},
        "roofline": roof,
        "segments_per_s": (round(seg_step * args.steps / dt, 1) if seg_step else None),
        "image_ok": image_ok,
        "image_check": image_what,
        "share_ok": share_ok,
        "timed_breakdown_ms": {"job": round(dt * 1e3, 4),
                               "max_rank": round(ts["max_rank_s"] * 1e3, 4),
                               "per_rank_ms": [round(x * 1e3, 4) for x in ts["per_rank"]],
                               "start_skew": round(ts["start_skew_s"] * 1e3, 4),
                               "host_issue": round(ts["issue"] * 1e3, 4),
                               "barrier_ms": round(ts["barrier_s"] * 1e3, 4)},
        "gather": {"how": gather_how, "wall_ms": round(dt_gather * 1e3, 4),
                   "events_ms": round(gather_s * 1e3, 4),
                   "bytes_to_root": 16 * w * r.rows0 * (world - 1)},   # (padded bands)
        "job": {"wall_ms": round((dt + dt_gather) * 1e3, 4),
                "Mrays_per_s": round(w * h * spf * args.steps / (dt + dt_gather) / 1e6, 2),
                "what": "the K steps plus the one gather of the finished tiles"},
        "candidate_lists": cand_stats,
        "warm_up": {"ms": round(warm_s * 1e3, 2), "steps": args.warmup},
    }
    if host_t is not None:
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
        if dispatch and depth == 1:
            # the dispatch structure, K2 / K4 / K5, rank shares: each with its image check
            # (a side measurement that fails is reported in the line, never costs the line)
            try:
                side.update(driver_record_sides(device, stream, cfg))
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
