"""Image output files: host-side writers/readers round-trip exactly."""
import numpy as np

from conftest import PKG_DIR  # noqa: F401  (puts the package on sys.path)


def test_png_round_trip(tmp_path, rt):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (13, 17, 4), dtype=np.uint8)
    p = tmp_path / "a.png"
    rt.image_io.save_png(p, img)
    assert p.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
    np.testing.assert_array_equal(rt.image_io.load_png(p), img)


def test_png_reader_handles_all_row_filters(tmp_path, rt):
    """load_png undoes filters 1-4 (other writers use them); checked against a hand-filtered
    stream of a known image."""
    import struct
    import zlib
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (5, 6, 4), dtype=np.uint8)
    h, w = img.shape[:2]
    rows = []
    prev = np.zeros(w * 4, np.int32)
    for y in range(h):
        cur = img[y].reshape(-1).astype(np.int32)
        ft = y % 5
        a = np.concatenate([np.zeros(4, np.int32), cur[:-4]])
        c = np.concatenate([np.zeros(4, np.int32), prev[:-4]])
        b = prev
        if ft == 0:
            pred = np.zeros_like(cur)
        elif ft == 1:
            pred = a
        elif ft == 2:
            pred = b
        elif ft == 3:
            pred = (a + b) // 2
        else:
            pa, pb, pc = np.abs(b - c), np.abs(a - c), np.abs(a + b - 2 * c)
            pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))
        rows.append(bytes([ft]) + ((cur - pred) & 0xFF).astype(np.uint8).tobytes())
        prev = cur

    def chunk(tag, body):
        return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body))
    data = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(b"".join(rows))) + chunk(b"IEND", b""))
    p = tmp_path / "f.png"
    p.write_bytes(data)
    np.testing.assert_array_equal(rt.image_io.load_png(p), img)


def test_pfm_and_npy_round_trip(tmp_path, rt):
    rng = np.random.default_rng(5)
    img = rng.random((7, 9, 4), dtype=np.float32)
    img[0, 0, 0] = np.nan
    rt.image_io.save_pfm(tmp_path / "a.pfm", img)
    back = rt.image_io.load_pfm(tmp_path / "a.pfm")
    assert back.tobytes() == np.ascontiguousarray(img[..., :3]).tobytes()
    head = (tmp_path / "a.pfm").read_bytes()[:12]
    assert head.startswith(b"PF\n9 7\n-1.0\n")
    rt.image_io.save_npy(tmp_path / "a.npy", img)
    assert np.load(tmp_path / "a.npy").tobytes() == img.tobytes()


def test_present_restatement_edges():
    from oracle import present_ref as P
    x = np.array([[[0.0, 1.0, 0.5, 7.0], [np.nan, -0.0, np.inf, 0.0],
                   [-np.inf, 1e-30, 0.99999994, 0.0]]], np.float32)
    lin = P.present(x, "linear")
    assert lin[0, 0, :3].tolist() == [0, 255, 128] and lin[0, 1, :3].tolist() == [0, 0, 255]
    assert lin[0, 2, :3].tolist() == [0, 0, 255] and np.all(lin[..., 3] == 255)
    s = P.present(x, "srgb")
    assert s[0, 0, :3].tolist() == [0, 255, 188] and s[0, 1, :3].tolist() == [0, 0, 255]
    assert s[0, 2, :3].tolist() == [0, 0, 255]
