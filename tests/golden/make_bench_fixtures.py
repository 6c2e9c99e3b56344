"""Generates tests/golden/bench_k2.npz and bench_k3.npz: what bench.py's timed image must hold.

bench.py --config K2/K3 runs W warmup + K timed progressive `update` dispatches (frame 0
resets the accumulator) with the per-frame seeds rt_frame_seeds(0x5EED) and the
CameraSettings::default geometry at 1920x1080, max_depth 1, samples_per_pixel 65536 (never
capped).  After the timed frames it compares 4096 sampled pixels of the image with these
fixtures, for the frame counts W + K listed here (the driver's --warmup 5 --steps 20 and
bench.py's defaults).  The values come from the CPU oracle (test infrastructure), through
the rt_render contract (oracle.render_pixels: frames chained updates of the given pixels).
K4 and K5 need no extra fixture: bench.py checks them against k4.npz / k5.npz.

    python tests/golden/make_bench_fixtures.py        # ~2 min on 8 cores (with the digests)
"""
from __future__ import annotations

import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import host_ref as H  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent
BENCH_SEED = 0x5EED
BENCH_SPP = 65536
FRAME_COUNTS = (25, 220)          # (--warmup 5 --steps 20), (bench.py defaults 20 + 200)
SAMPLES = 4096


def sample_coords(w, h, n, seed):
    rng = np.random.default_rng(seed)
    xs = rng.integers(0, w, n, dtype=np.uint32)
    ys = rng.integers(0, h, n, dtype=np.uint32)
    xs[:5] = [0, w - 1, 0, w - 1, w // 2]
    ys[:5] = [0, 0, h - 1, h - 1, h // 2]
    return xs, ys


def fixture(name, kind, n):
    w, h = 1920, 1080
    spheres = H.generate_scene(kind, n, 1)
    seeds = H.frame_seeds(BENCH_SEED, max(FRAME_COUNTS))
    cam = H.scene_camera_from(spp=BENCH_SPP, max_depth=1, width=w, height=h,
                              random_seed=float(seeds[0]), moved=True)
    xs, ys = sample_coords(w, h, SAMPLES, 4321)
    parts = np.array_split(np.arange(SAMPLES), 32)

    def run(frames):
        def work(idx):
            st, _ = O.render_pixels(np.zeros((idx.size, 4), np.float32), xs[idx], ys[idx], cam,
                                    spheres, seeds[:frames])
            return idx, st
        out = np.empty((SAMPLES, 4), np.float32)
        with ThreadPoolExecutor() as ex:
            for idx, st in ex.map(work, parts):
                out[idx] = st
        return out

    pixels = np.stack([run(f) for f in FRAME_COUNTS])
    np.savez_compressed(OUT / name, camera=cam, spheres=spheres, seeds=seeds,
                        width=np.array(w), height=np.array(h), px=xs, py=ys,
                        frame_counts=np.array(FRAME_COUNTS, np.uint32), pixels=pixels)
    print("wrote", name, pixels.shape)


def main():
    fixture("bench_k2.npz", 0, 0)
    fixture("bench_k3.npz", 2, 500)
    # whole-image and per-band digests at both frame counts (make_band_digests.py)
    sys.path.insert(0, str(OUT))
    import make_band_digests
    make_band_digests.main(["bench"])


if __name__ == "__main__":
    main()
