"""CPU tests of the oracle itself (no GPU): known-answer RNG values, canonical sin/cos
accuracy, analytic ray/sphere cases, a float64 restatement of the whole per-pixel
pipeline, and the committed golden fixtures."""
import json
import math

import numpy as np
import pytest

from conftest import GOLDEN, bits_equal, load_golden

M32 = 0xFFFFFFFF


def py_hash(v):
    """wgsl:50-59 in Python integers (independent of the C oracle)."""
    s = v & M32
    s ^= 2747636419
    s = (s * 2654435769) & M32
    s ^= s >> 16
    s = (s * 2654435769) & M32
    s ^= s >> 16
    s = (s * 2654435769) & M32
    return s


def py_rf(v):
    return float(np.float32(py_hash(v))) / 2.0 ** 32


# Hand-checked anchors (python integer arithmetic): hash(0), hash(1).
def test_hash_known_answers(oracle):
    assert py_hash(0) == oracle.hash_u32(0)
    rng = np.random.default_rng(0)
    vals = [0, 1, 2, 3, 73, 51, 1000, 0x7FFFFFFF, 0x80000000, M32] + \
        [int(v) for v in rng.integers(0, 2 ** 32, 2000, dtype=np.uint64)]
    for v in vals:
        assert oracle.hash_u32(v) == py_hash(v), v
    kat = json.loads((GOLDEN / "kat.json").read_text())
    for k, v in kat["hash"].items():
        assert py_hash(int(k)) == v


def test_random_float_semantics(oracle):
    # f32(hash)/4294967295.0 where the literal is 2^32 in f32: exact scaling.
    assert float(np.float32(4294967295.0)) == 2.0 ** 32
    rng = np.random.default_rng(1)
    for v in [int(x) for x in rng.integers(0, 2 ** 32, 2000, dtype=np.uint64)]:
        assert oracle.random_float(v) == py_rf(v)
    # f32(u32) rounds to nearest, so rf reaches exactly 1.0 for hash >= 0xFFFFFF80
    assert float(np.float32(0xFFFFFF80)) == 2.0 ** 32
    kat = json.loads((GOLDEN / "kat.json").read_text())
    for k, bits in kat["random_float_bits"].items():
        assert int(np.float32(oracle.random_float(int(k))).view(np.uint32)) == bits


def _ulp_err(got, want):
    want32 = np.float32(want)
    spacing = np.spacing(np.float32(abs(want32))) if want32 != 0 else np.float32(1e-45)
    return abs(float(got) - want) / float(spacing)


def test_canonical_sincos_accuracy(oracle):
    """The fixed sin/cos polynomial stays within 2 ulp (abs err <= 6e-8 near zeros) of the
    true functions over the reference's argument range [0, 2*pi] (wgsl:237, 328)."""
    xs = np.linspace(0.0, 6.2831855, 20001, dtype=np.float32)
    worst = 0.0
    for x in xs:
        s, c = oracle.sincos(float(x))
        for got, want in ((s, math.sin(float(x))), (c, math.cos(float(x)))):
            if abs(want) < 1e-3:
                assert abs(got - want) < 6e-8
            else:
                worst = max(worst, _ulp_err(got, want))
    assert worst <= 2.0, worst
    kat = json.loads((GOLDEN / "kat.json").read_text())
    for x, bits in kat["sincos_bits"].items():
        s, c = oracle.sincos(float(x))
        assert [int(np.float32(s).view(np.uint32)), int(np.float32(c).view(np.uint32))] == bits


SPH = [0.0, 1.0, 0.0, 1.0, 0.5, 0.5, 0.5, -2.0]


def test_sphere_hit_through_centre(oracle):
    t, p, n, front = oracle.sphere_hit(SPH, (0, 1, -5), (0, 0, 1), 0.001, 3.4e35)
    assert t == 4.0 and list(p) == [0, 1, -1] and list(n) == [0, 0, -1] and front


def test_sphere_hit_tangent_is_back_face(oracle):
    # D == 0 exactly; dot(d, outward) == 0 is not < 0, so front_face = false and the
    # normal is flipped (wgsl:159-160).
    t, p, n, front = oracle.sphere_hit(SPH, (-5, 0, 0), (1, 0, 0), 0.001, 3.4e35)
    assert t == 5.0 and list(p) == [0, 0, 0] and not front and list(n) == [0, 1, 0]


def test_sphere_hit_from_inside(oracle):
    t, p, n, front = oracle.sphere_hit(SPH, (0, 1, 0), (0, 0, 2), 0.001, 3.4e35)
    assert t == 0.5 and list(p) == [0, 1, 1] and not front and list(n) == [0, 0, -1]


def test_sphere_hit_rejections(oracle):
    assert oracle.sphere_hit(SPH, (0, 1, -5), (0, 0, -1), 0.001, 3.4e35) is None  # behind
    assert oracle.sphere_hit(SPH, (0, 3, -5), (0, 0, 1), 0.001, 3.4e35) is None   # miss
    # tmax <= root is a miss (strict), so an equal-t later sphere never wins
    assert oracle.sphere_hit(SPH, (0, 1, -5), (0, 0, 1), 0.001, 4.0) is None
    # root <= tmin falls through to the far root
    t, *_ = oracle.sphere_hit(SPH, (0, 1, -5), (0, 0, 1), 4.0, 3.4e35)
    assert t == 6.0


# ---- float64 restatement of the pipeline (independent math: libm sin/cos/pow) --------

def _f64_pixel(cam, spheres, x, y, inp):
    c = cam
    center = np.array(c[0:3], float)
    vul, pdu, pdv = np.array(c[4:7], float), np.array(c[8:11], float), np.array(c[12:15], float)
    ddu, ddv = np.array(c[16:19], float), np.array(c[24:27], float)
    defocus, depth, spp, moved, rseed = c[11], int(c[27]), int(c[31]), c[35], c[39]
    col, n = np.array(inp[:3], float), int(inp[3])
    if moved > 0.5:
        col, n = np.zeros(3), 0
    if n >= spp:
        return np.array([*col, n])
    B = int(np.float32(rseed) * np.float32(2.0 ** 32)) & M32
    s = (1 + n + B) & M32
    g = py_hash(py_hash((x * 73) & M32) ^ py_hash((y * 51) & M32) ^ ((s * 25 + B) & M32))
    off = (py_rf(g) - 0.5, py_rf((g * g) & M32) - 0.5)
    pc = vul + pdu * (x + 0.5 + off[0]) + pdv * (y + 0.5 + off[1])
    if defocus > 0:
        ang = float(np.float32(2.0 * 3.1415926)) * py_rf(g + 1)
        p = np.array([math.cos(ang), math.sin(ang)])
        p /= np.linalg.norm(p)
        o = center + p[0] * ddu + p[1] * ddv
    else:
        o = center
    d = pc - o
    seed = (s + 1) & M32
    cf = np.ones(3)
    for i in range(depth):
        best, bt = -1, 3.4e35
        for k, sp in enumerate(spheres):
            C, R = np.array(sp[0:3], float), float(sp[3])
            oc = C - o
            a, h, cc = d @ d, oc @ d, oc @ oc - R * R
            D = h * h - a * cc
            if D < 0:
                continue
            q = math.sqrt(D)
            r = (h - q) / a
            if r <= 0.001 or bt <= r:
                r = (h + q) / a
                if r <= 0.001 or bt <= r:
                    continue
            best, bt = k, r
        if best < 0:
            break
        sp = spheres[best]
        C, R, mat = np.array(sp[0:3], float), float(sp[3]), np.array(sp[4:8], float)
        p = o + bt * d
        nrm = (p - C) / R
        front = d @ nrm < 0
        nrm = nrm if front else -nrm
        sb = py_hash((seed + i * 1000) & M32)

        def ruv(sd):
            z = 2 * py_rf(sd) - 1
            aa = py_rf(sd + 1) * float(np.float32(6.283185307))
            r_ = math.sqrt(max(0.0, 1 - z * z))
            return np.array([r_ * math.cos(aa), r_ * math.sin(aa), z])

        if mat[3] < -1:
            nd = nrm + ruv(sb)
            if nd @ nd < 1e-6:
                nd = nrm
            att = mat[:3]
        elif mat[3] <= 1:
            rf_ = d - 2 * (nrm @ d) * nrm
            refl = rf_ / np.linalg.norm(rf_) + mat[3] * ruv(sb)
            if not refl @ nrm > 0:
                return None  # absorbed: colour 0 (handled by caller)
            nd = refl / np.linalg.norm(refl)
            att = mat[:3]
        else:
            att = np.ones(3)
            ratio = 1 / mat[0] if front else mat[0]
            u = d / np.linalg.norm(d)
            cos_t = min(-(u @ nrm), 1.0)
            sin_t = math.sqrt(max(0.0, 1 - cos_t * cos_t))
            r0 = ((1 - ratio) / (1 + ratio)) ** 2
            refl_p = ratio * sin_t > 1 or r0 + (1 - r0) * math.pow(1 - cos_t, 5) > py_rf(sb)
            if refl_p:
                nd = u - 2 * (nrm @ u) * nrm
            else:
                dd = nrm @ u
                k = 1 - ratio * ratio * (1 - dd * dd)
                nd = np.zeros(3) if k < 0 else ratio * u - (ratio * dd + math.sqrt(k)) * nrm
            nd = nd / np.linalg.norm(nd)
        cf = cf * att
        o, d = p, nd
    uy = d[1] / np.linalg.norm(d)
    a = 0.5 * (uy + 1)
    sky = (1 - a) * np.ones(3) + a * np.array([0.5, 0.7, 1.0])
    res = cf * sky
    col = col + (res - col) / (n + 1)
    return np.array([*col, n + 1])


@pytest.mark.parametrize("scene_kind,depth,defocus", [(0, 1, 0.6), (1, 3, 0.6), (0, 8, 0.0)])
def test_oracle_matches_float64_restatement(oracle, scene_kind, depth, defocus):
    """The f32 canonical oracle agrees with an independent float64/libm evaluation: all but a
    handful of pixels (near discrete decision boundaries) within 1e-4 per channel."""
    from oracle import host_ref as H
    w, h = 24, 16
    spheres = H.generate_scene(scene_kind, 0, 3)
    cam = H.scene_camera_from(max_depth=depth, width=w, height=h, random_seed=0.375,
                              defocus_angle=defocus)
    inp = np.zeros((h, w, 4), np.float32)
    out, _ = oracle.update(inp, cam, spheres)
    close = 0
    for y in range(h):
        for x in range(w):
            ref = _f64_pixel(cam, spheres, x, y, inp[y, x])
            if ref is None:
                ref = np.array([0, 0, 0, 1.0])
            if np.all(np.abs(out[y, x] - ref) <= 1e-4):
                close += 1
    assert close >= w * h - 3, f"{w * h - close} pixels differ from the float64 restatement"


def test_golden_k1(oracle):
    g = load_golden("k1.npz")
    out, segs = oracle.update(np.zeros((256, 256, 4), np.float32), g["camera"], g["spheres"])
    ok, bad = bits_equal(out, g["image"])
    assert ok, bad
    assert segs == int(g["segments"]) == 256 * 256


def test_parallel_update_is_the_same_image(oracle):
    """The threaded CPU baseline (row bands from a queue) computes the same bits."""
    g = load_golden("k1.npz")
    out, segs = oracle.update_parallel(np.zeros((256, 256, 4), np.float32), g["camera"],
                                       g["spheres"], threads=3)
    ok, bad = bits_equal(out, g["image"])
    assert ok, bad
    assert segs == 256 * 256


@pytest.mark.parametrize("threads,band", [(1, 8), (5, 2), (64, 1)])
def test_native_threaded_update_is_the_same_image(oracle, threads, band):
    """bench.py's CPU baseline (oracle_update_threads: pthreads claiming row bands from a
    shared counter, more threads than bands included) computes the golden image's bits."""
    g = load_golden("k1.npz")
    out, segs = oracle.update_threads(np.zeros((256, 256, 4), np.float32), g["camera"],
                                      g["spheres"], threads, band)
    ok, bad = bits_equal(out, g["image"])
    assert ok, bad
    assert segs == 256 * 256


def test_golden_accumulator(oracle):
    g = load_golden("accum_default.npz")
    cur = g["state0"]
    for f in range(3):
        cur, _ = oracle.update(cur, g["cameras"][f], g["spheres"])
        ok, bad = bits_equal(cur, g["frames"][f])
        assert ok, (f, bad)


@pytest.mark.parametrize("name", ["k2.npz", "k3.npz", "k4.npz", "k5.npz"])
def test_golden_sampled_pixels(oracle, name):
    g = load_golden(name)
    n = 256 if name in ("k4.npz", "k5.npz") else g["px"].size
    st, _ = oracle.render_pixels(np.zeros((n, 4), np.float32), g["px"][:n], g["py"][:n],
                                 g["camera"], g["spheres"], g["seeds"])
    ok, bad = bits_equal(st, g["pixels"][:n])
    assert ok, bad
