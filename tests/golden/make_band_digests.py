"""Adds exact whole-image and per-band digests to the full-size fixtures (round 6).

For every fixture below, the CPU oracle renders the WHOLE image (oracle.render_pixels over
8-row bands on native threads) and the fixture gets:
  sha256        SHA-256 of the float32 image bytes (row-major H x W x 4, NaN canonical)
  band_sha      uint8 [H / 8, 32]: SHA-256 of each 8-row band's bytes (RT_STRIPE_ROWS), so
                that any rank's share under any band -> rank map can be checked exactly,
                band by band, without the 132-MB image
  segments      sphere_list_hit calls of the whole render (one "segment" each),
                the numerator of bench.py's segments/s
  channel_sums  float64 sums of the four channels (diagnostic)
K5 (3840x2160, 500 spheres, 64 spp, depth 8) also gets 16384 random sampled pixels (plus the
corners and the centre) replacing round 5's 512, for locating a mismatch.  The camera,
spheres and seeds of each fixture are kept byte for byte (the fixture's own inputs).
bench_k2/k3 get one digest set per frame count they hold (band_sha [counts, H/8, 32]).

    python tests/golden/make_band_digests.py [k5|k4|bench]...   # K5 ~12 min on 8 cores
"""
from __future__ import annotations

import hashlib
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden as G  # noqa: E402
from make_golden import O  # noqa: E402

ROWS = 8
CANON_NAN = np.uint32(0x7FC00000)


def canon(img: np.ndarray) -> np.ndarray:
    """NaN channels (a degenerate refraction, SURVEY §8b "Errors") as one bit pattern: the
    parity tests compare NaN == NaN whatever its payload or sign (conftest.bits_equal), and
    the digests must say the same.  Every digest of this script and of the checkers that
    read it (bench.py, tests) is taken over canon(image)."""
    a = np.ascontiguousarray(img, np.float32).copy()
    a.view(np.uint32)[np.isnan(a)] = CANON_NAN
    return a


def band_digests(img: np.ndarray) -> np.ndarray:
    img = canon(img)
    h = img.shape[0]
    out = np.zeros((h // ROWS, 32), np.uint8)
    for b in range(h // ROWS):
        out[b] = np.frombuffer(hashlib.sha256(img[b * ROWS:(b + 1) * ROWS].tobytes()).digest(),
                               np.uint8)
    return out


def full_image(name):
    g = dict(np.load(HERE / name))
    w, h = int(g["width"]), int(g["height"])
    img, segs = G.render_full(w, h, g["camera"], g["spheres"], g["seeds"])
    return g, img, segs


def add_full(name, n_samples=None, sample_seed=1234):
    g, img, segs = full_image(name)
    w, h = int(g["width"]), int(g["height"])
    if n_samples:
        xs, ys = G.sample_coords(w, h, n_samples, sample_seed)
        g["px"], g["py"] = xs, ys
    # the sampled pixels must be the full render's
    got = img[g["py"], g["px"]]
    if "pixels" in g and not n_samples:
        assert np.array_equal(got.view(np.uint32), g["pixels"].view(np.uint32)), name
    g["pixels"] = got
    print(name, "NaN channels:", int(np.isnan(img).sum()))
    g.update(sha256=np.array(G.digest(canon(img))), band_sha=band_digests(img),
             segments=np.array(segs, np.uint64),
             channel_sums=img.astype(np.float64).sum((0, 1)))
    G.save(name, **g)


def add_bench(name):
    g = dict(np.load(HERE / name))
    w, h = int(g["width"]), int(g["height"])
    shas, bands, segs_all = [], [], []
    for k, frames in enumerate(int(c) for c in g["frame_counts"]):
        img, segs = G.render_full(w, h, g["camera"], g["spheres"], g["seeds"][:frames])
        want = g["pixels"][k]
        assert np.array_equal(img[g["py"], g["px"]].view(np.uint32), want.view(np.uint32)), name
        print(name, frames, "NaN channels:", int(np.isnan(img).sum()))
        shas.append(G.digest(canon(img)))
        bands.append(band_digests(img))
        segs_all.append(segs)
    g.update(sha256=np.array(shas), band_sha=np.stack(bands),
             segments=np.array(segs_all, np.uint64))
    G.save(name, **g)


def main(which):
    O.lib()
    if "k5" in which:
        add_full("k5.npz", n_samples=16384)
    if "k4" in which:
        add_full("k4.npz")
    if "bench" in which:
        add_bench("bench_k3.npz")
        add_bench("bench_k2.npz")


if __name__ == "__main__":
    main(sys.argv[1:] or ["k5", "k4", "bench"])
