"""The compute-shader plugin surface (src/lib.rs), bound to the HIP kernels.

Reference -> here:
  ComputeShaderPipeline::from_world (lib.rs:240-324)   -> ComputeShaderPipeline(device)
  ComputeShaderImages {texture_a, texture_b} (138-142)  -> ComputeShaderImages
  `init` dispatch (lib.rs:398-407, wgsl:65-70)          -> ComputeShaderPipeline.init_image
  `update` dispatch (lib.rs:408-417, wgsl:333-364)      -> ComputeShaderPipeline.update
  ComputeShaderNode state machine (lib.rs:326-421)      -> ComputeShaderNode (C++ driver)
Extensions the reference lacks: fused multi-frame accumulation (``render``), the stripe
partition for multi-GPU (``render_stripes`` / ``deinterleave``).

Images are torch float32 tensors of shape (H, W, 4) on the pipeline's device (RGBA32F,
row-major, alpha = sample count).  Every call is enqueued on torch's current stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .camera import SceneCamera
from .scene import SphereCollection

RT_STRIPE_ROWS = _lib.RT_STRIPE_ROWS


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def _np_ptr(a: np.ndarray) -> ctypes.c_void_p:
    # (the array interface's address: ndarray.ctypes builds a helper object per access,
    # several microseconds of host time on every call)
    return ctypes.c_void_p(a.__array_interface__["data"][0])


# torch's current stream as a raw handle without building a Stream object per call
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _is_f32c(a) -> bool:
    return isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous


def _cam_blob(camera: SceneCamera) -> np.ndarray:
    """The camera's 44 f32 as one contiguous array: the rt_scene_camera layout itself."""
    blob = camera.blob
    if not _is_f32c(blob) or blob.size != 44:
        blob = np.ascontiguousarray(blob, np.float32)
        if blob.size != 44:
            raise ValueError("a SceneCamera blob holds 44 f32 (176 bytes)")
    return blob


def _check_image(t: torch.Tensor, width: int, height: int, name: str) -> None:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise ValueError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous float32")
    if t.numel() < width * height * 4:
        raise ValueError(f"{name} holds {t.numel()} floats, need {width * height * 4}")


def stripe_local_rows(height: int, rank: int, nranks: int) -> int:
    return int(_lib.lib().rt_stripe_local_rows(height, rank, nranks))


def stripe_band_set(height: int, rank: int, nranks: int) -> tuple[int, int, int]:
    """The round-robin stripes of rank / nranks as a band set (first, step, count)."""
    bands = (height + RT_STRIPE_ROWS - 1) // RT_STRIPE_ROWS
    return (rank, nranks, (bands - rank + nranks - 1) // nranks if bands > rank else 0)


def partition_bands(band_cost, nranks: int) -> list[tuple[int, int, int]]:
    """rt_partition_bands: the bands cut into nranks contiguous ranges (first, 1, count)
    whose largest cost is the smallest possible (host-only, exact)."""
    c = np.ascontiguousarray(band_cost, np.float64)
    out = (_lib.BandSetC * nranks)()
    _lib.call("rt_partition_bands", _np_ptr(c), c.size, nranks, out)
    return [(b.first, b.step, b.count) for b in out]


class ComputeShaderPipeline:
    """One librt_hip.so context on one HIP device (lib.rs:231-324)."""

    def __init__(self, device: int | torch.device = 0):
        if isinstance(device, torch.device):
            device = device.index if device.index is not None else torch.cuda.current_device()
        self.device = int(device)
        self.torch_device = torch.device("cuda", self.device)
        ctx = ctypes.c_void_p()
        _lib.call("rt_create", self.device, ctypes.byref(ctx))
        self._ctx = ctx
        self._sphere_keep = None
        self.scan_mode = "culled"

    # ---- lifetime ---------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_ctx", None) and self._ctx.value:
            _lib.call("rt_destroy", self._ctx)
            self._ctx = ctypes.c_void_p()

    def set_frames_per_launch(self, n: int) -> None:
        """rt_set_frames_per_launch: update_frames' frames per launch (0 = automatic,
        1 = one `update` dispatch per frame, n = up to n)."""
        _lib.call("rt_set_frames_per_launch", self._ctx, int(n))

    def set_frame_pairs(self, mode: str) -> None:
        """rt_set_frame_pairs: 'auto' | 'off' | 'on' (two waves per tile, alternate frames)
        | 'quad' (four waves per tile) | 'on2' / 'quad2' (two / four waves per pair of tiles,
        two pixels per lane)."""
        _lib.call("rt_set_frame_pairs", self._ctx,
                  {"auto": 0, "off": 1, "on": 2, "quad": 3, "on2": 4, "quad2": 5}[mode])

    def set_frame_images(self, mode: str) -> None:
        """rt_set_frame_images: the images a fused multi-frame launch writes — "last_two"
        (default: the two that survive the call) or "every" (every frame's image to the
        ping-pong buffer its chained update writes, as the reference's dispatches do);
        identical pixels."""
        _lib.call("rt_set_frame_images", self._ctx, {"last_two": 0, "every": 1}[mode])

    def set_tile_order(self, mode: str) -> None:
        """rt_set_tile_order: "auto" (costliest tiles first, from the first launch's
        per-tile durations) or "off" (raster order)."""
        _lib.call("rt_set_tile_order", self._ctx, {"auto": 0, "off": 1}[mode])

    def set_update_queues(self, queues: int) -> None:
        """rt_set_update_queues: one-frame updates of update_frames as `queues` concurrent
        parts on their own streams (0 = automatic, 1 = one launch per update)."""
        _lib.call("rt_set_update_queues", self._ctx, int(queues))

    def set_update_submit(self, mode: str) -> None:
        """rt_set_update_submit: how update_frames submits one-frame updates — "auto" (HIP
        launches; AQL is opt-in), "hip" or "aql" (AQL packets on the context's own HSA
        queues, an error if unavailable; after a failed AQL segment, reported once as an
        error, the context runs HIP launches); identical pixels."""
        _lib.call("rt_set_update_submit", self._ctx, {"auto": 0, "hip": 1, "aql": 2}[mode])

    def submit_status(self) -> dict:
        """rt_update_submit_status: whether AQL submission is available (and why not), the go
        waits that gave up (0 in a correct run) and the AQL packets submitted so far."""
        avail, give_ups, packets = ctypes.c_int(0), _lib.U32(0), ctypes.c_uint64(0)
        _lib.call("rt_update_submit_status", self._ctx, ctypes.byref(avail),
                  ctypes.byref(give_ups), ctypes.byref(packets))
        why = "" if avail.value else _lib.lib().rt_last_error().decode()
        return {"aql_available": bool(avail.value), "go_give_ups": int(give_ups.value),
                "packets": int(packets.value), "why": why}

    def set_path_compaction(self, mode: str) -> None:
        """rt_set_path_compaction for bounce launches: "auto" (default: "split" with four
        chunks for launches of at most 20 000 tiles once their tile costs are measured, else
        "per_wave"), "per_wave", "compact" (paths repacked across four waves after every
        bounce), "pair" (two waves per tile on alternate frames) or "split" (a tile's frames in
        chunks on separate waves, the last finisher accumulating; with measured costs only
        the costliest tiles split, every unit dispatched by its own cost)."""
        _lib.call("rt_set_path_compaction", self._ctx,
                  {"auto": 0, "per_wave": 1, "compact": 2, "pair": 3, "split": 4}[mode])

    def set_single_kernel(self, mode: str) -> None:
        """rt_set_single_kernel: "auto" (one-frame launches of the camera-ray-only case run
        rt_single_kernel: two tiles per wave, one for small launches), "pair", "one" (force
        either) or "off" (the general rt_trace_kernel<2>); identical pixels."""
        _lib.call("rt_set_single_kernel", self._ctx,
                  {"auto": 0, "off": 1, "pair": 2, "one": 3}[mode])

    def frames_per_launch(self, camera) -> int:
        """rt_get_frames_per_launch: frames update_frames fuses per launch for `camera`."""
        out = _lib.U32(0)
        cam = camera.to_c()
        _lib.call("rt_get_frames_per_launch", self._ctx, ctypes.byref(cam), ctypes.byref(out))
        return int(out.value)

    def last_launch_info(self) -> dict:
        """rt_last_launch_info: what the last trace call launched — launches, frames,
        max_frames_per_launch, kernel (RT_KERNEL_* id) and its rocprofv3 name, the parts
        (queues) and the submission ("hip" or "aql")."""
        info = _lib.LaunchInfoC()
        _lib.call("rt_last_launch_info", self._ctx, ctypes.byref(info))
        d = {k: int(getattr(info, k)) for k, _ in info._fields_}
        d["kernel_name"] = _lib.lib().rt_kernel_name(d["kernel"]).decode()
        d["submit"] = {1: "hip", 2: "aql"}.get(d["submit"], "none")
        if d["submit"] == "aql" and d["kernel_name"].startswith("rt_single_kernel"):
            # the AQL path dispatches the chain instances of the same kernel
            d["kernel_name"] = d["kernel_name"].replace("rt_single_kernel", "rt_chain_kernel")
        return d

    def set_launch_timing(self, enable: bool) -> None:
        """rt_set_launch_timing: the fused launches of each update_frames call carry timing
        events in their own dispatch packets (no marker packets on the stream)."""
        _lib.call("rt_set_launch_timing", self._ctx, 1 if enable else 0)

    def last_call_kernel_time(self) -> tuple[float, int]:
        """rt_last_call_kernel_time: (seconds from the start of the last call's first timed
        launch to the end of its last, launches timed); waits for that launch."""
        ms, n = ctypes.c_float(0.0), _lib.U32(0)
        _lib.call("rt_last_call_kernel_time", self._ctx, ctypes.byref(ms), ctypes.byref(n))
        return ms.value / 1e3, int(n.value)

    def candidate_stats(self) -> dict:
        """rt_candidate_stats: the camera rays' per-tile candidate lists built last."""
        out = (ctypes.c_uint64 * 5)()
        _lib.call("rt_candidate_stats", self._ctx, out)
        t, none, entries, mx, cap = (int(v) for v in out)
        listed = t - none
        return {"tiles": t, "tiles_without_list": none,
                "no_list_frac": round(none / t, 6) if t else 0.0,
                "mean_entries": round(entries / listed, 3) if listed else 0.0,
                "max_entries": mx, "capacity": cap}

    def selftest_fastmath(self, n_random: int = 1 << 26) -> list[int]:
        """rt_selftest_fastmath: [defocus, division, sqrt, root-selection mismatches,
        cases run]."""
        out = (ctypes.c_uint64 * 5)()
        _lib.call("rt_selftest_fastmath", self._ctx, n_random, out)
        return list(out)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- helpers ----------------------------------------------------------------------
    def _stream(self) -> ctypes.c_void_p:
        if _raw_stream is not None:
            return ctypes.c_void_p(_raw_stream(self.device))
        return ctypes.c_void_p(torch.cuda.current_stream(self.torch_device).cuda_stream)

    def _spheres(self, spheres: SphereCollection):
        arr = np.ascontiguousarray(spheres.spheres, np.float32)
        self._sphere_keep = arr
        return _np_ptr(arr), arr.shape[0]

    def new_image(self, width: int, height: int) -> torch.Tensor:
        return torch.zeros((height, width, 4), dtype=torch.float32, device=self.torch_device)

    # ---- the plugin operations --------------------------------------------------------
    def set_scan_mode(self, mode: str) -> None:
        """"culled" (default, exact wave-level culling) or "exhaustive" (linear walk)."""
        code = {"exhaustive": _lib.RT_SCAN_EXHAUSTIVE, "culled": _lib.RT_SCAN_CULLED}[mode]
        _lib.call("rt_set_scan_mode", self._ctx, code)
        self.scan_mode = mode

    def set_spheres(self, spheres: SphereCollection) -> None:
        p, n = self._spheres(spheres)
        _lib.call("rt_set_spheres", self._ctx, p, n, self._stream())

    def init_image(self, out: torch.Tensor, width: int, height: int) -> None:
        _check_image(out, width, height, "out")
        _lib.call("rt_init_image", self._ctx, _ptr(out), width, height, self._stream())

    def update(self, inp: torch.Tensor, out: torch.Tensor, width: int, height: int,
               camera: SceneCamera, spheres: SphereCollection) -> None:
        _check_image(inp, width, height, "in")
        _check_image(out, width, height, "out")
        cam = camera.to_c()
        p, n = self._spheres(spheres)
        _lib.call("rt_update", self._ctx, _ptr(inp), _ptr(out), width, height,
                  ctypes.byref(cam), p, n, self._stream())

    def render(self, inp: torch.Tensor, out: torch.Tensor, width: int, height: int,
               camera: SceneCamera, spheres: SphereCollection, seeds) -> None:
        _check_image(inp, width, height, "in")
        _check_image(out, width, height, "out")
        cam = camera.to_c()
        p, n = self._spheres(spheres)
        s = np.ascontiguousarray(seeds, np.float32)
        _lib.call("rt_render", self._ctx, _ptr(inp), _ptr(out), width, height,
                  ctypes.byref(cam), p, n, s.size, _np_ptr(s),
                  self._stream())

    def render_stripes(self, inp: torch.Tensor, out: torch.Tensor, width: int, height: int,
                       rank: int, nranks: int, camera: SceneCamera,
                       spheres: SphereCollection, seeds) -> None:
        rows = stripe_local_rows(height, rank, nranks)
        _check_image(inp, width, rows, "in")
        _check_image(out, width, rows, "out")
        cam = camera.to_c()
        p, n = self._spheres(spheres)
        s = np.ascontiguousarray(seeds, np.float32)
        _lib.call("rt_render_stripes", self._ctx, _ptr(inp), _ptr(out), width, height, rank,
                  nranks, ctypes.byref(cam), p, n, s.size, _np_ptr(s),
                  self._stream())

    def update_frames(self, image_a: torch.Tensor, image_b: torch.Tensor, width: int,
                      height: int, camera: SceneCamera, spheres: SphereCollection, seeds,
                      rank: int = 0, nranks: int = 1) -> int:
        """len(seeds) progressive `update` dispatches ping-ponging a -> b -> a ... (the
        reference's per-frame loop, lib.rs:366-417); returns 0 if image_a holds the
        result, 1 for image_b.  Frame 0 honours camera.camera_has_moved."""
        rows = stripe_local_rows(height, rank, nranks) if nranks > 1 else height
        _check_image(image_a, width, rows, "image_a")
        _check_image(image_b, width, rows, "image_b")
        cam = camera.to_c()
        p, n = self._spheres(spheres)
        s = np.ascontiguousarray(seeds, np.float32)
        newest = ctypes.c_int(-1)
        _lib.call("rt_update_frames", self._ctx, _ptr(image_a), _ptr(image_b), width, height,
                  rank, nranks, ctypes.byref(cam), p, n, s.size, _np_ptr(s), self._stream(),
                  ctypes.byref(newest))
        return newest.value

    def bind_update_frames(self, image_a: torch.Tensor, image_b: torch.Tensor, width: int,
                           height: int, rank: int = 0, nranks: int = 1):
        """update_frames with the images, size and stripe fixed: the images are checked once
        here, and the returned run(camera, spheres, seeds) -> newest issues the call with no
        per-call validation or lookups (the host time before a call's first launch is part of
        a short timed region).  The images must stay allocated while run is used."""
        rows = stripe_local_rows(height, rank, nranks) if nranks > 1 else height
        _check_image(image_a, width, rows, "image_a")
        _check_image(image_b, width, rows, "image_b")
        fn = _lib.lib().rt_update_frames
        ctx, pa, pb = self._ctx, _ptr(image_a), _ptr(image_b)
        newest = ctypes.c_int(-1)
        pnew = ctypes.byref(newest)
        stream = self._stream
        # the CPython binding (rt_fastcall.c) when built: the same call with plain ints and
        # the arrays' buffers, ≈ 1 µs of host time against ≈ 8 µs through ctypes
        fast = _lib.fastcall()
        ictx, ia, ib = ctx.value, pa.value, pb.value
        dev = self.device if fast is not None else None
        raw = _raw_stream
        # the caller's spheres array when it can be passed as it is (contiguous float32
        # (N, 8)), its data pointer and count; `held` keeps the array the pointer points into
        # alive until the next call replaces it (a converted copy included)
        last = {"arr": None, "ptr": None, "n": 0, "held": None}

        # arrays the binding refused (by identity): they take the converting path below from
        # then on instead of raising and catching on every call
        refused = {"arr": None, "seeds": None}

        def run(camera: SceneCamera, spheres: SphereCollection, seeds) -> int:
            arr = spheres.spheres
            # the binding takes exactly what the ctypes path passes unconverted: contiguous
            # float32 (N, 8) spheres (an (N, 16) array would otherwise be read as N records of
            # a 32-byte stride) and contiguous float32 seeds
            if (fast is not None and arr is not refused["arr"] and seeds is not refused["seeds"]
                    and _is_f32c(arr) and arr.ndim == 2 and arr.shape[1] == 8
                    and _is_f32c(seeds)):
                try:
                    r = fast.update_frames(ictx, ia, ib, width, height, rank, nranks,
                                           camera.blob, arr, len(arr), seeds,
                                           raw(dev) if raw else stream().value)
                except (TypeError, ValueError, BufferError):
                    refused.update(arr=arr, seeds=seeds)
                    r = None
                if r is not None:
                    if r < 0:
                        _lib.check(-r, "rt_update_frames")
                    return r
            # the camera blob itself is the 176-byte rt_scene_camera (no struct copy).  A
            # spheres array that is contiguous float32 (N, 8) is passed as it is, its pointer
            # re-read only when the array object or its length changes; any other array is
            # converted on every call.  (The library compares the contents on every call, so
            # an array edited in place is still uploaded.)
            blob = _cam_blob(camera)
            arr = spheres.spheres
            if arr is not last["arr"] or arr.shape[0] != last["n"]:
                direct = _is_f32c(arr) and arr.ndim == 2 and arr.shape[1] == 8
                held = arr if direct else np.ascontiguousarray(arr, np.float32).reshape(-1, 8)
                last.update(arr=arr if direct else None, held=held, n=held.shape[0],
                            ptr=held.__array_interface__["data"][0])
            s = seeds if _is_f32c(seeds) else np.ascontiguousarray(seeds, np.float32)
            rc = fn(ctx, pa, pb, width, height, rank, nranks, blob.__array_interface__["data"][0],
                    last["ptr"], last["n"], s.size, s.__array_interface__["data"][0], stream(),
                    pnew)
            if rc:
                _lib.check(rc, "rt_update_frames")
            return newest.value

        run.images = (image_a, image_b)
        return run

    def update_frames_bands(self, image_a: torch.Tensor, image_b: torch.Tensor, width: int,
                            height: int, bands, camera: SceneCamera,
                            spheres: SphereCollection, seeds) -> int:
        """rt_update_frames_bands: update_frames over the band set bands = (first, step,
        count) — local band j is global band first + j * step; the images hold count * 8
        rows.  Returns 0 if image_a holds the result, 1 for image_b."""
        rows = int(bands[2]) * RT_STRIPE_ROWS
        _check_image(image_a, width, rows, "image_a")
        _check_image(image_b, width, rows, "image_b")
        bs = _lib.band_sets([bands])
        cam = camera.to_c()
        p, n = self._spheres(spheres)
        sd = np.ascontiguousarray(seeds, np.float32)
        newest = ctypes.c_int(-1)
        _lib.call("rt_update_frames_bands", self._ctx, _ptr(image_a), _ptr(image_b), width,
                  height, bs, ctypes.byref(cam), p, n, sd.size, _np_ptr(sd), self._stream(),
                  ctypes.byref(newest))
        return newest.value

    def band_costs(self, width: int, height: int, bands) -> np.ndarray:
        """rt_band_costs: per local band of `bands` the tile costs (device clock ticks) the
        context's last cost-recording launch measured for that share."""
        out = np.zeros(int(bands[2]), np.float64)
        _lib.call("rt_band_costs", self._ctx, width, height, _lib.band_sets([bands]),
                  _np_ptr(out))
        return out

    def deinterleave_bands(self, gathered: torch.Tensor, out: torch.Tensor, width: int,
                           height: int, sets, rows_per_rank: int) -> None:
        """rt_deinterleave_bands: nranks = len(sets) compact buffers of rows_per_rank rows
        each (rank order) scattered into the width x height image."""
        _check_image(gathered, width, rows_per_rank * len(sets), "gathered")
        _check_image(out, width, height, "out")
        _lib.call("rt_deinterleave_bands", self._ctx, _ptr(gathered), _ptr(out), width,
                  height, len(sets), _lib.band_sets(sets), rows_per_rank, self._stream())

    def deinterleave(self, gathered: torch.Tensor, out: torch.Tensor, width: int, height: int,
                     nranks: int) -> None:
        rows = stripe_local_rows(height, 0, nranks)
        _check_image(gathered, width, rows * nranks, "gathered")
        _check_image(out, width, height, "out")
        _lib.call("rt_deinterleave_stripes", self._ctx, _ptr(gathered), _ptr(out), width,
                  height, nranks, self._stream())


    def present(self, image: torch.Tensor, width: int, height: int,
                encoding: str = "srgb", out: torch.Tensor | None = None) -> torch.Tensor:
        """8-bit RGBA of a float image (rt_present_rgba8), a (H, W, 4) uint8 device tensor:
        what the reference's sprite shows (lib.rs:79-102), ready for a PNG."""
        _check_image(image, width, height, "image")
        code = {"linear": _lib.RT_ENCODE_LINEAR, "srgb": _lib.RT_ENCODE_SRGB}[encoding]
        if out is None:
            out = torch.empty((height, width, 4), dtype=torch.uint8, device=self.torch_device)
        if out.dtype != torch.uint8 or not out.is_contiguous() or out.numel() < width * height * 4:
            raise ValueError("out must be contiguous uint8 with width*height*4 elements")
        _lib.call("rt_present_rgba8", self._ctx, _ptr(image), _ptr(out), width, height, code,
                  self._stream())
        return out


def srgb_thresholds() -> np.ndarray:
    """The 256-entry f32 boundary table of the sRGB encoding (rt_srgb_thresholds)."""
    t = np.zeros(256, np.float32)
    _lib.lib().rt_srgb_thresholds(t.ctypes.data_as(ctypes.c_void_p))
    return t


class ComputeShaderImages:
    """texture_a / texture_b (lib.rs:60-93, 138-142): two zero-filled RGBA32F images."""

    def __init__(self, pipeline: ComputeShaderPipeline, width: int, height: int):
        self.width, self.height = width, height
        self.texture_a = pipeline.new_image(width, height)
        self.texture_b = pipeline.new_image(width, height)


class ComputeShaderNode:
    """Render-graph node (lib.rs:326-421) driving init + ping-pong updates per frame."""

    STATES = {0: "Loading", 1: "Init", 2: "Update(0)", 3: "Update(1)"}

    def __init__(self, pipeline: ComputeShaderPipeline, images: ComputeShaderImages):
        self.pipeline = pipeline
        self.images = images
        drv = ctypes.c_void_p()
        _lib.call("rt_driver_create", pipeline._ctx, _ptr(images.texture_a),
                  _ptr(images.texture_b), images.width, images.height, ctypes.byref(drv))
        self._drv = drv

    @property
    def state(self) -> str:
        return self.STATES[_lib.lib().rt_driver_state(self._drv)]

    def frame(self, camera: SceneCamera, spheres: SphereCollection) -> torch.Tensor:
        """One frame (node.update() + node.run()); returns the image written last."""
        cam = camera.to_c()
        p, n = self.pipeline._spheres(spheres)
        newest = ctypes.c_int(-1)
        _lib.call("rt_driver_frame", self._drv, ctypes.byref(cam), p, n,
                  self.pipeline._stream(), ctypes.byref(newest))
        return self.images.texture_a if newest.value == 0 else self.images.texture_b

    def close(self) -> None:
        if getattr(self, "_drv", None) and self._drv.value:
            _lib.call("rt_driver_destroy", self._drv)
            self._drv = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
