"""ctypes binding of librt_hip.so (include/rt_abi.h).

The library must be built in-tree (``make -C gpu-ray-tracing_amd`` or
``__graft_entry__.build()``).  There is no fallback: if the HIP library is missing or
fails to load, every entry point raises.

``torch`` is imported before the library is opened so that the HIP runtime torch ships
(soname libamdhip64.so.7) is the one librt_hip.so binds to; streams and device pointers
from torch are then valid inside the library.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (load order: torch's HIP runtime first)

PKG_ROOT = Path(__file__).resolve().parent.parent          # gpu-ray-tracing_amd/
LIB_PATH = PKG_ROOT / "build" / "librt_hip.so"

F = ctypes.c_float
U32 = ctypes.c_uint32


class RtError(RuntimeError):
    """A librt_hip.so entry point returned a non-zero rt_status."""

    def __init__(self, status: int, func: str, message: str):
        super().__init__(f"{func} failed with status {status} ({STATUS_NAMES.get(status, '?')}): "
                         f"{message}")
        self.status = status


STATUS_NAMES = {
    0: "RT_OK",
    1: "RT_ERR_INVALID_ARGUMENT",
    2: "RT_ERR_INVALID_SIZE",
    3: "RT_ERR_INVALID_DEVICE",
    4: "RT_ERR_HIP",
    5: "RT_ERR_NO_MEMORY",
    6: "RT_ERR_INVALID_CONTEXT",
    7: "RT_ERR_COMM",
}
RT_COMM_ID_BYTES = 128
RT_STRIPE_ROWS = 8
RT_SCAN_EXHAUSTIVE = 0
RT_SCAN_CULLED = 1
RT_ENCODE_LINEAR = 0
RT_ENCODE_SRGB = 1


class SceneCameraC(ctypes.Structure):
    """rt_scene_camera == SceneCamera (camera.rs:256-291), 176 bytes."""

    _fields_ = [
        ("center", F * 3), ("viewport_height", F),
        ("viewport_upper_left", F * 3), ("viewport_width", F),
        ("pixel_delta_u", F * 3), ("defocus_angle", F),
        ("pixel_delta_v", F * 3), ("aspect_ratio", F),
        ("defocus_disk_u", F * 3), ("_padding0", F),
        ("viewport_u", F * 3), ("_padding1", F),
        ("defocus_disk_v", F * 3), ("max_depth", F),
        ("look_from", F * 3), ("samples_per_pixel", F),
        ("look_at", F * 3), ("camera_has_moved", F),
        ("vup", F * 3), ("random_seed", F),
        ("viewport_v", F * 3), ("defocus_radius", F),
    ]


class SphereC(ctypes.Structure):
    """rt_sphere == GpuSphere (sphere.rs:20-26), 32 bytes."""

    _fields_ = [("position", F * 3), ("radius", F), ("color", F * 4)]


class CameraSettingsC(ctypes.Structure):
    """rt_camera_settings == CameraSettings (camera.rs:9-28)."""

    _fields_ = [
        ("field_of_view", F), ("samples_per_pixel", U32), ("camera_has_moved", U32),
        ("max_depth", U32), ("vup", F * 3), ("look_from", F * 3), ("look_at", F * 3),
        ("defocus_angle", F), ("focus_distance", F),
    ]


assert ctypes.sizeof(SceneCameraC) == 176
assert ctypes.sizeof(SphereC) == 32

P = ctypes.c_void_p
_SIGS = {
    "rt_abi_version": (U32, []),
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_kernel_name": (ctypes.c_char_p, [ctypes.c_int]),
    "rt_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(P)]),
    "rt_destroy": (ctypes.c_int, [P]),
    "rt_set_scan_mode": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_set_spheres": (ctypes.c_int, [P, P, U32, P]),
    "rt_init_image": (ctypes.c_int, [P, P, U32, U32, P]),
    "rt_update": (ctypes.c_int, [P, P, P, U32, U32, P, P, U32, P]),
    "rt_render": (ctypes.c_int, [P, P, P, U32, U32, P, P, U32, U32, P, P]),
    "rt_render_stripes": (ctypes.c_int, [P, P, P, U32, U32, U32, U32, P, P, U32, U32, P, P]),
    "rt_update_frames": (ctypes.c_int, [P, P, P, U32, U32, U32, U32, P, P, U32, U32, P, P,
                                        ctypes.POINTER(ctypes.c_int)]),
    "rt_stripe_local_rows": (U32, [U32, U32, U32]),
    "rt_deinterleave_stripes": (ctypes.c_int, [P, P, P, U32, U32, U32, P]),
    "rt_camera_settings_default": (None, [P]),
    "rt_camera_from_settings": (ctypes.c_int, [P, U32, U32, F, P]),
    "rt_scene_generate": (ctypes.c_int, [U32, U32, ctypes.c_uint64, P, U32, ctypes.POINTER(U32)]),
    "rt_frame_seeds": (None, [ctypes.c_uint64, U32, P]),
    "rt_driver_create": (ctypes.c_int, [P, P, P, U32, U32, ctypes.POINTER(P)]),
    "rt_driver_destroy": (ctypes.c_int, [P]),
    "rt_driver_frame": (ctypes.c_int, [P, P, P, U32, P, ctypes.POINTER(ctypes.c_int)]),
    "rt_driver_state": (ctypes.c_int, [P]),
    "rt_present_rgba8": (ctypes.c_int, [P, P, P, U32, U32, ctypes.c_int, P]),
    "rt_srgb_thresholds": (None, [P]),
    "rt_selftest_fastmath": (ctypes.c_int, [P, ctypes.c_uint64, P]),
    "rt_set_frames_per_launch": (ctypes.c_int, [P, U32]),
    "rt_get_frames_per_launch": (ctypes.c_int, [P, P, ctypes.POINTER(U32)]),
    "rt_set_frame_pairs": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_set_tile_order": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_set_update_queues": (ctypes.c_int, [P, U32]),
    "rt_set_update_submit": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_set_frame_images": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_update_submit_status": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(U32),
                                               ctypes.POINTER(ctypes.c_uint64)]),
    "rt_last_launch_info": (ctypes.c_int, [P, P]),
    "rt_set_path_compaction": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_set_single_kernel": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_candidate_stats": (ctypes.c_int, [P, P]),
    "rt_comm_unique_id": (ctypes.c_int, [P]),
    "rt_comm_create": (ctypes.c_int, [P, P, U32, U32, ctypes.POINTER(P)]),
    "rt_comm_create_all": (ctypes.c_int, [U32, P, P]),
    "rt_comm_destroy": (ctypes.c_int, [P]),
    "rt_comm_info": (ctypes.c_int, [P, ctypes.POINTER(U32), ctypes.POINTER(U32),
                                    ctypes.POINTER(ctypes.c_int)]),
    "rt_comm_group_start": (ctypes.c_int, []),
    "rt_comm_group_end": (ctypes.c_int, []),
    "rt_gather_stripes": (ctypes.c_int, [P, P, P, P, P, U32, U32, U32, P]),
    "rt_update_frames_bands": (ctypes.c_int, [P, P, P, U32, U32, P, P, P, U32, U32, P, P,
                                              ctypes.POINTER(ctypes.c_int)]),
    "rt_band_costs": (ctypes.c_int, [P, U32, U32, P, P]),
    "rt_partition_bands": (ctypes.c_int, [P, U32, U32, P]),
    "rt_deinterleave_bands": (ctypes.c_int, [P, P, P, U32, U32, U32, P, U32, P]),
    "rt_gather_bands": (ctypes.c_int, [P, P, P, P, P, U32, U32, P, U32, P]),
    "rt_set_launch_timing": (ctypes.c_int, [P, ctypes.c_int]),
    "rt_last_call_kernel_time": (ctypes.c_int, [P, ctypes.POINTER(F), ctypes.POINTER(U32)]),
}


class BandSetC(ctypes.Structure):
    """rt_band_set (rt_abi.h, ABI 7): global bands first + j * step, j < count."""
    _fields_ = [("first", U32), ("step", U32), ("count", U32)]


def band_sets(sets) -> ctypes.Array:
    """A ctypes array of rt_band_set from (first, step, count) triples."""
    arr = (BandSetC * len(sets))()
    for i, (f, st, c) in enumerate(sets):
        arr[i].first, arr[i].step, arr[i].count = int(f), int(st), int(c)
    return arr


class LaunchInfoC(ctypes.Structure):
    """rt_launch_info (rt_abi.h)."""
    _fields_ = [("launches", U32), ("frames", U32), ("max_frames_per_launch", U32),
                ("kernel", ctypes.c_int32), ("queues", U32), ("submit", U32),
                ("normal_rn", U32)]

_lib = None


def lib() -> ctypes.CDLL:
    """Open librt_hip.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        path = Path(os.environ.get("RT_HIP_LIB", LIB_PATH))
        if not path.exists():
            raise RuntimeError(f"librt_hip.so not found at {path}: build it with "
                               f"`make -C {PKG_ROOT}` (no CPU fallback exists)")
        handle = ctypes.CDLL(str(path))
        for name, (res, args) in _SIGS.items():
            if "RT_HIP_LIB" in os.environ and not hasattr(handle, name):
                continue  # an older experiment build (tools/ab_variants.py)
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


_fast = False


def fastcall():
    """The CPython binding of rt_update_frames (build/_rt_fastcall*.so, csrc/host/rt_fastcall.c:
    the same library entry point without ctypes' per-call conversion), or None when it has
    not been built or an experiment build of the library is selected (RT_HIP_LIB: the binding
    links the in-tree librt_hip.so)."""
    global _fast
    if _fast is False:
        _fast = None
        if "RT_HIP_LIB" not in os.environ:
            import importlib.machinery
            import importlib.util
            import sysconfig
            path = PKG_ROOT / "build" / ("_rt_fastcall" + sysconfig.get_config_var("EXT_SUFFIX"))
            if path.exists():
                lib()                      # (the library first: the same mapping)
                loader = importlib.machinery.ExtensionFileLoader("_rt_fastcall", str(path))
                spec = importlib.util.spec_from_file_location("_rt_fastcall", path,
                                                              loader=loader)
                mod = importlib.util.module_from_spec(spec)
                loader.exec_module(mod)
                _fast = mod
    return _fast


def exported_symbols() -> list[str]:
    return list(_SIGS)


def check(status: int, func: str) -> None:
    if status != 0:
        msg = lib().rt_last_error()
        raise RtError(status, func, msg.decode() if msg else "")


def call(func: str, *args) -> None:
    check(getattr(lib(), func)(*args), func)
