"""Scene: mirror of src/scene/sphere.rs.

``SphereCollection`` holds GpuSphere records (sphere.rs:20-33) as an (N, 8) float32
array: position xyz, radius, material color rgba (color.w encodes the material,
wgsl:272-284).  Generators call the seeded C++ implementation of
``create_default_spheres`` (sphere.rs:45-153) in librt_hip.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

SCENE_THREE = 0      # the three large spheres (sphere.rs:114-136)
SCENE_DEFAULT = 1    # ground + 14x14 jittered grid + 3 large (sphere.rs:45-153)
SCENE_N = 2          # ground + grid in [-12,12)^2 truncated to N-4 + 3 large


@dataclass
class SphereCollection:
    spheres: np.ndarray  # (count, 8) float32

    @property
    def count(self) -> int:
        return int(self.spheres.shape[0])

    def as_bytes(self) -> bytes:
        return np.ascontiguousarray(self.spheres, np.float32).tobytes()

    def ctypes_ptr(self):
        self._keep = np.ascontiguousarray(self.spheres, np.float32)
        return self._keep.ctypes.data_as(ctypes.c_void_p)

    @staticmethod
    def generate(kind: int, n_spheres: int = 0, seed: int = 1) -> "SphereCollection":
        count = _lib.U32(0)
        _lib.call("rt_scene_generate", kind, n_spheres, seed, None, 0, ctypes.byref(count))
        buf = np.zeros((count.value, 8), np.float32)
        _lib.call("rt_scene_generate", kind, n_spheres, seed,
                  buf.ctypes.data_as(ctypes.c_void_p), count.value, ctypes.byref(count))
        return SphereCollection(buf)


def three_spheres() -> SphereCollection:
    return SphereCollection.generate(SCENE_THREE)


def create_default_spheres(seed: int = 1) -> SphereCollection:
    return SphereCollection.generate(SCENE_DEFAULT, 0, seed)


def synthetic_scene(n: int, seed: int = 1) -> SphereCollection:
    return SphereCollection.generate(SCENE_N, n, seed)


def frame_seeds(seed: int, frames: int) -> np.ndarray:
    """Per-frame random_seed values k/2^24 (stand-in for rand::random(), camera.rs:346)."""
    out = np.zeros(frames, np.float32)
    _lib.lib().rt_frame_seeds(seed, frames, out.ctypes.data_as(ctypes.c_void_p))
    return out
