"""Image output: file formats for the accumulator the reference only shows
on screen (the sprite of lib.rs:79-102).

* ``.npy``  — the RGBA32F accumulator as is (H, W, 4) float32: mean colour + sample count.
* ``.pfm``  — Portable Float Map, RGB float32, exact linear colour (bottom-to-top rows as
  the format requires).
* ``.png``  — 8-bit RGBA from ``ComputeShaderPipeline.present`` (sRGB or linear encoding
  on the GPU); written here with zlib, no imaging library needed.

The files are written on the host; the conversion to 8 bits runs on the device.
"""
from __future__ import annotations

import struct
import zlib
from pathlib import Path

import numpy as np


def save_npy(path, image) -> None:
    """The float accumulator, bit for bit (torch tensor or ndarray, (H, W, 4) float32)."""
    np.save(path, _host(image).astype(np.float32, copy=False), allow_pickle=False)


def save_pfm(path, image) -> None:
    """RGB float32 PFM ("PF", little-endian scale -1.0), rows bottom to top."""
    a = _host(image).astype(np.float32, copy=False)
    h, w = a.shape[:2]
    rgb = np.ascontiguousarray(a[::-1, :, :3], dtype="<f4")
    with open(path, "wb") as f:
        f.write(b"PF\n%d %d\n-1.0\n" % (w, h))
        f.write(rgb.tobytes())


def load_pfm(path) -> np.ndarray:
    """(H, W, 3) float32 from a PFM written by save_pfm (either endianness)."""
    data = Path(path).read_bytes()
    parts = data.split(b"\n", 3)
    if parts[0] != b"PF":
        raise ValueError("not an RGB PFM file")
    w, h = (int(v) for v in parts[1].split())
    scale = float(parts[2])
    dt = "<f4" if scale < 0 else ">f4"
    a = np.frombuffer(parts[3], dtype=dt, count=w * h * 3).reshape(h, w, 3)
    return a[::-1].astype(np.float32)


def _chunk(tag: bytes, body: bytes) -> bytes:
    return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body))


def save_png(path, rgba8) -> None:
    """8-bit RGBA PNG (colour type 6, filter 0 on every row) of an (H, W, 4) uint8 image."""
    a = _host(rgba8)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("save_png needs an (H, W, 4) uint8 image")
    h, w = a.shape[:2]
    raw = np.concatenate([np.zeros((h, 1), np.uint8), a.reshape(h, w * 4)], axis=1)
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(_chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)))
        f.write(_chunk(b"IDAT", zlib.compress(raw.tobytes(), 6)))
        f.write(_chunk(b"IEND", b""))


def load_png(path) -> np.ndarray:
    """(H, W, 4) uint8 from an 8-bit RGBA, non-interlaced PNG (all five row filters)."""
    data = Path(path).read_bytes()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG file")
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n, tag = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    if depth != 8 or ctype != 6 or interlace != 0:
        raise ValueError("only 8-bit RGBA non-interlaced PNG is supported")
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * 4)
    out = np.zeros((h, w * 4), np.int32)
    prev = np.zeros(w * 4, np.int32)
    for y in range(h):
        ft, row = raw[y, 0], raw[y, 1:].astype(np.int32)
        cur = np.zeros(w * 4, np.int32)
        for i in range(w * 4):
            a_ = cur[i - 4] if i >= 4 else 0
            b_ = prev[i]
            c_ = prev[i - 4] if i >= 4 else 0
            if ft == 0:
                p = 0
            elif ft == 1:
                p = a_
            elif ft == 2:
                p = b_
            elif ft == 3:
                p = (a_ + b_) // 2
            else:
                pa, pb, pc = abs(b_ - c_), abs(a_ - c_), abs(a_ + b_ - 2 * c_)
                p = a_ if pa <= pb and pa <= pc else (b_ if pb <= pc else c_)
            cur[i] = (row[i] + p) & 0xFF
        out[y], prev = cur, cur
    return out.reshape(h, w, 4).astype(np.uint8)


def _host(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach()
        if x.device.type != "cpu":
            x = x.cpu()
        x = x.numpy()
    return np.ascontiguousarray(x)
