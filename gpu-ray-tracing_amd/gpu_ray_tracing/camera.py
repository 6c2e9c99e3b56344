"""Camera: mirror of src/camera.rs.

``CameraSettings`` is camera.rs:9-46 (main-world settings, Default at 30-46);
``SceneCamera`` is the 176-byte GPU struct (camera.rs:256-291) and
``SceneCamera.from_settings`` is ``impl From<&CameraSettings> for SceneCamera``
(camera.rs:293-351), evaluated by the C++ host code in librt_hip.so with the image size
as an argument and the per-frame ``random_seed`` supplied by the caller.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib


@dataclass
class CameraSettings:
    """camera.rs:9-28; defaults from camera.rs:30-46."""

    field_of_view: float = 20.0
    samples_per_pixel: int = 500
    camera_has_moved: bool = True
    max_depth: int = 30
    vup: tuple = (0.0, 1.0, 0.0)
    look_from: tuple = (13.0, 2.0, 3.0)
    look_at: tuple = (0.0, 0.0, 0.0)
    defocus_angle: float = 0.6
    focus_distance: float = 10.0

    def to_c(self) -> _lib.CameraSettingsC:
        c = _lib.CameraSettingsC()
        c.field_of_view = self.field_of_view
        c.samples_per_pixel = int(self.samples_per_pixel)
        c.camera_has_moved = 1 if self.camera_has_moved else 0
        c.max_depth = int(self.max_depth)
        c.vup[:] = [float(v) for v in self.vup]
        c.look_from[:] = [float(v) for v in self.look_from]
        c.look_at[:] = [float(v) for v in self.look_at]
        c.defocus_angle = self.defocus_angle
        c.focus_distance = self.focus_distance
        return c

    @staticmethod
    def default_from_library() -> "CameraSettings":
        c = _lib.CameraSettingsC()
        _lib.lib().rt_camera_settings_default(ctypes.byref(c))
        return CameraSettings(c.field_of_view, c.samples_per_pixel, bool(c.camera_has_moved),
                              c.max_depth, tuple(c.vup), tuple(c.look_from), tuple(c.look_at),
                              c.defocus_angle, c.focus_distance)


@dataclass
class SceneCamera:
    """The 176-byte SceneCamera blob (44 little-endian f32)."""

    blob: np.ndarray = field(default_factory=lambda: np.zeros(44, np.float32))

    @staticmethod
    def from_settings(settings: CameraSettings, width: int, height: int,
                      random_seed: float) -> "SceneCamera":
        out = _lib.SceneCameraC()
        s = settings.to_c()
        _lib.call("rt_camera_from_settings", ctypes.byref(s), width, height,
                  ctypes.c_float(random_seed), ctypes.byref(out))
        return SceneCamera(np.frombuffer(bytes(out), np.float32).copy())

    @staticmethod
    def from_bytes(b: bytes) -> "SceneCamera":
        a = np.frombuffer(b, np.float32).copy()
        assert a.size == 44, "SceneCamera is 176 bytes"
        return SceneCamera(a)

    def to_c(self) -> _lib.SceneCameraC:
        return _lib.SceneCameraC.from_buffer_copy(np.ascontiguousarray(self.blob, np.float32))

    def with_fields(self, **kw) -> "SceneCamera":
        c = self.to_c()
        for k, v in kw.items():
            setattr(c, k, v)
        return SceneCamera(np.frombuffer(bytes(c), np.float32).copy())

    def __getattr__(self, name):
        if name == "blob":
            raise AttributeError(name)
        c = self.to_c()
        v = getattr(c, name)
        return tuple(v) if isinstance(v, ctypes.Array) else v
