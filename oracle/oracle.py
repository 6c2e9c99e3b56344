"""TEST INFRASTRUCTURE ONLY — Python handle on the CPU oracle (oracle/rt_oracle.c).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker /
CPU baseline.  The product (librt_hip.so, gpu_ray_tracing) never imports this module.
Parity with the reference is UNPINNED (no reference fixtures exist; see rt_oracle.c).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "_build" / "librt_oracle.so"

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        h = ctypes.CDLL(str(LIB_PATH))
        h.oracle_hash.restype = _U32
        h.oracle_hash.argtypes = [_U32]
        h.oracle_random_float.restype = ctypes.c_float
        h.oracle_random_float.argtypes = [_U32]
        h.oracle_sincos.restype = None
        h.oracle_sincos.argtypes = [ctypes.c_float, _P, _P]
        h.oracle_update_rows.restype = ctypes.c_uint64
        h.oracle_update_rows.argtypes = [_P, _P, _U32, _U32, _U32, _U32, _P, _P, _U32]
        h.oracle_update.restype = ctypes.c_uint64
        h.oracle_update.argtypes = [_P, _P, _U32, _U32, _P, _P, _U32]
        h.oracle_update_threads.restype = ctypes.c_uint64
        h.oracle_update_threads.argtypes = [_P, _P, _U32, _U32, _P, _P, _U32, _U32, _U32]
        h.oracle_render_pixels.restype = ctypes.c_uint64
        h.oracle_render_pixels.argtypes = [_P, _P, _P, ctypes.c_uint64, _P, _P, _U32, _U32, _P]
        h.oracle_init.restype = None
        h.oracle_init.argtypes = [_P, _U32, _U32]
        h.oracle_sphere_hit.restype = ctypes.c_int
        h.oracle_sphere_hit.argtypes = [_P, _P, ctypes.c_float, ctypes.c_float, _P]
        _lib = h
    return _lib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def hash_u32(v: int) -> int:
    return int(lib().oracle_hash(v & 0xFFFFFFFF))


def random_float(v: int) -> float:
    return float(np.float32(lib().oracle_random_float(v & 0xFFFFFFFF)))


def sincos(x: float) -> tuple[float, float]:
    s = np.zeros(1, np.float32)
    c = np.zeros(1, np.float32)
    lib().oracle_sincos(ctypes.c_float(x), _p(s), _p(c))
    return float(s[0]), float(c[0])


def sphere_hit(sphere, ray_o, ray_d, tmin: float, tmax: float):
    """wgsl:182-221 for one sphere: returns None or (t, p, n, front)."""
    s = _f32(sphere).reshape(8)
    r = _f32(list(ray_o) + list(ray_d))
    out = np.zeros(8, np.float32)
    hit = lib().oracle_sphere_hit(_p(s), _p(r), ctypes.c_float(tmin), ctypes.c_float(tmax),
                                  _p(out))
    if not hit:
        return None
    return float(out[0]), out[1:4].copy(), out[4:7].copy(), bool(out[7])


def update(inp: np.ndarray, camera: np.ndarray, spheres: np.ndarray,
           rows: tuple[int, int] | None = None) -> tuple[np.ndarray, int]:
    """One `update` over a (H, W, 4) image.  Returns (out, segments traced)."""
    inp = _f32(inp)
    h, w, _ = inp.shape
    out = inp.copy()
    cam = _f32(camera).reshape(44)
    sph = _f32(spheres).reshape(-1, 8)
    y0, y1 = rows if rows else (0, h)
    segs = lib().oracle_update_rows(_p(inp), _p(out), w, h, y0, y1, _p(cam), _p(sph),
                                    sph.shape[0])
    return out, int(segs)


def update_threads(inp: np.ndarray, camera: np.ndarray, spheres: np.ndarray, threads: int,
                   band: int = 8) -> tuple[np.ndarray, int]:
    """`update` over the whole image on `threads` native threads (oracle_update_threads:
    bands claimed from a shared counter, no Python between them).  Same image as update()."""
    inp = _f32(inp)
    h, w, _ = inp.shape
    out = inp.copy()
    cam = _f32(camera).reshape(44)
    sph = _f32(spheres).reshape(-1, 8)
    segs = lib().oracle_update_threads(_p(inp), _p(out), w, h, _p(cam), _p(sph), sph.shape[0],
                                       max(1, threads), max(1, band))
    return out, int(segs)


def update_parallel(inp: np.ndarray, camera: np.ndarray, spheres: np.ndarray, threads: int,
                    rows: tuple[int, int] | None = None, band: int = 8) -> tuple[np.ndarray, int]:
    """`update` over rows [y0, y1) with `threads` host threads pulling 8-row bands from a
    shared queue (ctypes releases the GIL during each C call).  Same image as update()."""
    from concurrent.futures import ThreadPoolExecutor
    inp = _f32(inp)
    h, w, _ = inp.shape
    out = inp.copy()
    cam = _f32(camera).reshape(44)
    sph = _f32(spheres).reshape(-1, 8)
    y0, y1 = rows if rows else (0, h)
    L = lib()

    def run(b0):
        return int(L.oracle_update_rows(_p(inp), _p(out), w, h, b0, min(b0 + band, y1),
                                        _p(cam), _p(sph), sph.shape[0]))

    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        segs = sum(ex.map(run, range(y0, y1, band)))
    return out, segs


def render_pixels(state: np.ndarray, px, py, camera: np.ndarray, spheres: np.ndarray,
                  seeds) -> tuple[np.ndarray, int]:
    """`frames` chained updates for a list of pixels (contract of rt_render)."""
    st = _f32(state).reshape(-1, 4).copy()
    px = np.ascontiguousarray(px, np.uint32)
    py = np.ascontiguousarray(py, np.uint32)
    cam = _f32(camera).reshape(44)
    sph = _f32(spheres).reshape(-1, 8)
    sd = _f32(seeds).reshape(-1)
    segs = lib().oracle_render_pixels(_p(st), _p(px), _p(py), px.size, _p(cam), _p(sph),
                                      sph.shape[0], sd.size, _p(sd))
    return st, int(segs)


def render(inp: np.ndarray, camera: np.ndarray, spheres: np.ndarray, seeds) -> tuple[np.ndarray, int]:
    """Full-image rt_render contract: chained updates with per-frame seeds."""
    inp = _f32(inp)
    h, w, _ = inp.shape
    yy, xx = np.mgrid[0:h, 0:w]
    st, segs = render_pixels(inp.reshape(-1, 4), xx.ravel(), yy.ravel(), camera, spheres, seeds)
    return st.reshape(h, w, 4), segs
