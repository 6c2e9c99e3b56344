"""MI355X-native per-pixel ray tracer (Sur091/GPU-Ray-Tracing hot path, rebuilt for gfx950).

Python surface over librt_hip.so (include/rt_abi.h).  Names follow the reference crate
``gpu_ray_tracing`` (Cargo.toml:2): camera (src/camera.rs), scene (src/scene/sphere.rs),
compute_shader (the plugin in src/lib.rs).  The HIP library is the only compute path:
importing this package does not load it; the first call does, and raises if it is absent.
"""
from . import _lib
from .camera import CameraSettings, SceneCamera
from . import image_io
from .compute_shader import (RT_STRIPE_ROWS, ComputeShaderImages, ComputeShaderNode,
                             ComputeShaderPipeline, partition_bands, srgb_thresholds,
                             stripe_band_set, stripe_local_rows)
from .scene import (SCENE_DEFAULT, SCENE_N, SCENE_THREE, SphereCollection,
                    create_default_spheres, frame_seeds, synthetic_scene, three_spheres)

RtError = _lib.RtError

__all__ = [
    "CameraSettings", "SceneCamera", "ComputeShaderPipeline", "ComputeShaderImages",
    "ComputeShaderNode", "SphereCollection", "create_default_spheres", "synthetic_scene",
    "three_spheres", "frame_seeds", "stripe_local_rows", "RT_STRIPE_ROWS", "RtError",
    "SCENE_THREE", "SCENE_DEFAULT", "SCENE_N", "srgb_thresholds", "image_io",
    "partition_bands", "stripe_band_set",
]
