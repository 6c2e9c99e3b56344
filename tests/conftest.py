import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "gpu-ray-tracing_amd"
for p in (str(PKG_DIR), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds on CPU")


def _make(path: Path) -> None:
    # Incremental: a no-op when the in-tree artefacts are up to date (they travel with the
    # snapshot to the GPU box, where /opt/rocm is the same image).
    subprocess.run(["make", "-s", "-C", str(path)], check=True)


@pytest.fixture(scope="session", autouse=True)
def built_artifacts():
    if not (PKG_DIR / "build" / "librt_hip.so").exists():
        _make(PKG_DIR)
    if not (ROOT / "oracle" / "_build" / "librt_oracle.so").exists():
        _make(ROOT / "oracle")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def rt():
    import gpu_ray_tracing
    gpu_ray_tracing._lib.lib()
    return gpu_ray_tracing


def load_golden(name):
    import numpy as np
    return dict(np.load(GOLDEN / name, allow_pickle=False))


def bits_equal(a, b):
    """Bit-exact comparison treating any NaN as equal to any NaN."""
    import numpy as np
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return bool(same.all()), int((~same).sum())


CANON_NAN = 0x7FC00000


def canon_sha(img) -> str:
    """SHA-256 of a float32 image's bytes with every NaN as 0x7FC00000: the digest the
    fixtures' `sha256` / `band_sha` hold (tests/golden/make_band_digests.py), so NaN == NaN
    whatever its payload, as bits_equal compares."""
    import hashlib
    import numpy as np
    a = np.ascontiguousarray(img, np.float32).copy()
    a.view(np.uint32)[np.isnan(a)] = CANON_NAN
    return hashlib.sha256(a.tobytes()).hexdigest()


def bands_match(local, bands, band_sha, rows=8):
    """A rank's compact local image (global band bands[j] at local rows rows*j ...) against
    the fixture's per-band digests: the list of global bands that differ."""
    bad = []
    for j, b in enumerate(bands):
        if canon_sha(local[rows * j:rows * (j + 1)]) != bytes(band_sha[b]).hex():
            bad.append(int(b))
    return bad
