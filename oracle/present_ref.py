"""TEST INFRASTRUCTURE ONLY — numpy restatement of the presentation step,
the checker for rt_present_rgba8 / rt_srgb_thresholds (include/rt_abi.h).

The reference shows the newest Rgba32Float image as a sprite (src/lib.rs:79-102) on an
sRGB surface, i.e. the linear colour is sRGB-encoded for display; it has no file output.
The 8-bit conversion restated here is this repo's definition: "parity
unpinned" against the reference, which has no such output to compare with.
"""
from __future__ import annotations

import numpy as np


def srgb_thresholds() -> np.ndarray:
    """T[0] = 0; T[j] = the smallest f32 >= the linear value whose sRGB code is j - 0.5."""
    t = np.zeros(256, np.float32)
    for j in range(1, 256):
        v = (j - 0.5) / 255.0
        lin = v / 12.92 if v <= 0.04045 else ((v + 0.055) / 1.055) ** 2.4
        f = np.float32(lin)
        if float(f) < lin:
            f = np.nextafter(f, np.float32(2.0))
        t[j] = f
    return t


def present(image: np.ndarray, encoding: str) -> np.ndarray:
    """(H, W, 4) float32 -> (H, W, 4) uint8, alpha 255."""
    rgb = np.asarray(image, np.float32)[..., :3]
    if encoding == "linear":
        v = np.minimum(np.maximum(np.nan_to_num(rgb, nan=0.0, posinf=np.inf, neginf=-np.inf),
                                  np.float32(0)), np.float32(1))
        code = np.floor(v * np.float32(255.0) + np.float32(0.5))   # f32 mul, then f32 add
    elif encoding == "srgb":
        t = srgb_thresholds()[1:]
        code = np.searchsorted(t, rgb, side="right").astype(np.float32)  # #{j: c >= T[j]}
        code[np.isnan(rgb)] = 0
    else:
        raise ValueError(encoding)
    out = np.empty(rgb.shape[:-1] + (4,), np.uint8)
    out[..., :3] = code.astype(np.uint8)
    out[..., 3] = 255
    return out
