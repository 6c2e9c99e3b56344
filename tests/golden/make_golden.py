"""Generates the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no fixtures and cannot run here, so every fixture is
oracle-generated ("parity unpinned" w.r.t. the reference itself).  Inputs are built by the
Python restatements in oracle/host_ref.py (camera.rs / sphere.rs), and every fixture
stores the exact 176-byte camera blob, the sphere bytes and the per-frame seeds, so the
fixtures do not depend on any product code.

    python tests/golden/make_golden.py            # all fixtures (K4 full hash: ~1 min, 8 cores)

The whole-image and per-band digests of K4 / K5 (and K5's 16 384 sampled pixels and exact
segment count) are added by make_band_digests.py, which main() runs last (K5: ~12 min).
"""
from __future__ import annotations

import hashlib
import json
import os
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
THREADS = os.cpu_count() or 1


def camera(w, h, spp, depth, seed, moved=True, defocus=0.6):
    return H.scene_camera_from(spp=spp, max_depth=depth, width=w, height=h,
                               random_seed=float(seed), moved=moved, defocus_angle=defocus)


def render_full(w, h, cam, spheres, seeds, inp=None):
    """rt_render contract on the full image, parallel over row chunks (ctypes drops the GIL)."""
    inp = np.zeros((h, w, 4), np.float32) if inp is None else inp
    chunks = [(y0, min(h, y0 + 8)) for y0 in range(0, h, 8)]

    def work(c):
        y0, y1 = c
        yy, xx = np.mgrid[y0:y1, 0:w]
        st, segs = O.render_pixels(inp[y0:y1].reshape(-1, 4), xx.ravel(), yy.ravel(), cam,
                                   spheres, seeds)
        return y0, y1, st.reshape(y1 - y0, w, 4), segs

    out = np.empty_like(inp)
    segs = 0
    with ThreadPoolExecutor(THREADS) as ex:
        for y0, y1, st, s in ex.map(work, chunks):
            out[y0:y1] = st
            segs += s
    return out, segs


def sample_coords(w, h, n, seed):
    rng = np.random.default_rng(seed)
    xs = rng.integers(0, w, n, dtype=np.uint32)
    ys = rng.integers(0, h, n, dtype=np.uint32)
    # always include the four corners and the centre
    xs[:5] = [0, w - 1, 0, w - 1, w // 2]
    ys[:5] = [0, 0, h - 1, h - 1, h // 2]
    return xs, ys


def digest(img: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(img, np.float32).tobytes()).hexdigest()


def save(name, **arrays):
    np.savez_compressed(OUT / name, **arrays)
    print("wrote", name, {k: getattr(v, "shape", v) for k, v in arrays.items()})


def full_config(name, w, h, scene, spp, depth, frames, full_hash=True, n_samples=4096):
    spheres = scene
    seeds = H.frame_seeds(BENCH_SEED, frames)
    cam = camera(w, h, spp, depth, seeds[0])
    xs, ys = sample_coords(w, h, n_samples, 1234)
    st, _ = O.render_pixels(np.zeros((xs.size, 4), np.float32), xs, ys, cam, spheres, seeds)
    extra = {}
    if full_hash:
        img, segs = render_full(w, h, cam, spheres, seeds)
        extra = dict(sha256=np.array(digest(img)), channel_sums=img.astype(np.float64).sum((0, 1)),
                     segments=np.array(segs, np.uint64))
        assert np.array_equal(img[ys, xs].view(np.uint32), st.view(np.uint32))
    save(name, camera=cam, spheres=spheres, seeds=seeds, width=np.array(w), height=np.array(h),
         px=xs, py=ys, pixels=st, **extra)


def main():
    three = H.generate_scene(0)
    n500 = H.generate_scene(2, 500, 1)
    default = H.generate_scene(1, 0, 1)

    # K1: 256x256, 3 spheres, 1 spp, 1 bounce — full golden image.
    seeds = H.frame_seeds(BENCH_SEED, 1)
    cam = camera(256, 256, 1, 1, seeds[0])
    img, segs = O.update(np.zeros((256, 256, 4), np.float32), cam, three)
    save("k1.npz", camera=cam, spheres=three, seeds=seeds, image=img,
         segments=np.array(segs, np.uint64))

    # Accumulator fixture: default-like scene, depth 8, three chained updates (frame 0
    # resets), from a non-zero input state.
    w, h = 96, 64
    seeds = H.frame_seeds(7, 3)
    rng = np.random.default_rng(5)
    state0 = np.concatenate([rng.random((h, w, 3), np.float32),
                             np.full((h, w, 1), 3.0, np.float32)], axis=2)
    frames = []
    cur = state0
    for f in range(3):
        c = camera(w, h, 500, 8, seeds[f], moved=(f == 0))
        cur, _ = O.update(cur, c, default)
        frames.append(cur)
    cams = np.stack([camera(w, h, 500, 8, seeds[f], moved=(f == 0)) for f in range(3)])
    save("accum_default.npz", cameras=cams, spheres=default, seeds=seeds, state0=state0,
         frames=np.stack(frames))

    # Full-size configs (BASELINE.json configs[1..4]).
    full_config("k2.npz", 1920, 1080, three, 1, 1, 1)
    full_config("k3.npz", 1920, 1080, n500, 1, 1, 1)
    full_config("k4.npz", 1920, 1080, n500, 64, 1, 64)
    full_config("k5.npz", 3840, 2160, n500, 64, 8, 64, full_hash=False, n_samples=512)

    # Known-answer tests for the integer RNG and the canonical sin/cos.
    vals = [0, 1, 2, 73, 51, 1000, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF, 123456789]
    kat = {
        "hash": {str(v): O.hash_u32(v) for v in vals},
        "random_float_bits": {str(v): int(np.float32(O.random_float(v)).view(np.uint32))
                              for v in vals},
        "sincos_bits": {repr(x): [int(np.float32(c).view(np.uint32)) for c in O.sincos(x)]
                        for x in [0.0, 0.5, 1.0, 1.5707964, 3.1415927, 4.0, 6.2831855]},
    }
    (OUT / "kat.json").write_text(json.dumps(kat, indent=1))
    print("wrote kat.json")

    import make_band_digests
    make_band_digests.main(["k5", "k4"])


if __name__ == "__main__":
    main()
