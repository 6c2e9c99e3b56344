"""CPU tests of the C-ABI library's host side: it loads, exports every symbol the header
declares, has the reference's struct layouts, and its C++ host mirror (camera builder,
scene generator, seeds, frame driver argument checks) matches the oracle restatements."""
import ctypes
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT

HEADER = ROOT / "include" / "rt_abi.h"
LIB = PKG_DIR / "build" / "librt_hip.so"


def header_functions():
    text = HEADER.read_text()
    return re.findall(r"^RT_API [^(]*?\b(rt_\w+)\(", text, flags=re.M)


def test_library_exports_every_declared_symbol(rt):
    declared = header_functions()
    assert len(declared) == 52
    nm = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r" T (rt_\w+)$", nm, flags=re.M))
    assert set(declared) <= exported, set(declared) - exported
    # the ctypes binding covers exactly the header
    assert set(rt._lib.exported_symbols()) == set(declared)
    assert rt._lib.lib().rt_abi_version() == 7


def test_scene_camera_layout_matches_reference(rt):
    """camera.rs:256-291 / wgsl:7-40 byte offsets."""
    C = rt._lib.SceneCameraC
    want = dict(center=0, viewport_height=12, viewport_upper_left=16, viewport_width=28,
                pixel_delta_u=32, defocus_angle=44, pixel_delta_v=48, aspect_ratio=60,
                defocus_disk_u=64, _padding0=76, viewport_u=80, _padding1=92,
                defocus_disk_v=96, max_depth=108, look_from=112, samples_per_pixel=124,
                look_at=128, camera_has_moved=140, vup=144, random_seed=156, viewport_v=160,
                defocus_radius=172)
    for name, off in want.items():
        assert getattr(C, name).offset == off, name
    assert ctypes.sizeof(C) == 176
    S = rt._lib.SphereC
    assert (S.position.offset, S.radius.offset, S.color.offset, ctypes.sizeof(S)) == (0, 12, 16, 32)


def test_camera_defaults(rt):
    d = rt.CameraSettings.default_from_library()
    ref = rt.CameraSettings()  # camera.rs:30-46
    assert bytes(d.to_c()) == bytes(ref.to_c())


@pytest.mark.parametrize("w,h,fov,defocus,seed", [
    (1280, 720, 20.0, 0.6, 0.0), (1920, 1080, 20.0, 0.6, 0.5), (256, 256, 45.0, 0.0, 0.25),
    (3840, 2160, 20.0, 0.6, 0.75), (333, 77, 90.0, 2.5, 0.125)])
def test_camera_builder_matches_restatement(rt, w, h, fov, defocus, seed):
    from oracle import host_ref as H
    got = rt.SceneCamera.from_settings(
        rt.CameraSettings(field_of_view=fov, defocus_angle=defocus), w, h, seed).blob
    want = H.scene_camera_from(fov=fov, defocus_angle=defocus, width=w, height=h,
                               random_seed=seed)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_camera_builder_hand_values(rt):
    """Spot values by hand (camera.rs:293-351) at 1280x720 (the reference's SIZE)."""
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(), 1280, 720, 0.0)
    assert cam.aspect_ratio == pytest.approx(16 / 9, rel=1e-7)
    vh = 2 * np.tan(np.radians(10.0)) * 10
    assert cam.viewport_height == pytest.approx(vh, rel=1e-6)
    assert cam.viewport_width == pytest.approx(vh * 16 / 9, rel=1e-6)
    assert cam.defocus_radius == pytest.approx(10 * np.tan(np.radians(0.3)), rel=1e-6)
    w = np.array([13, 2, 3.0]) / np.linalg.norm([13, 2, 3])
    ul = np.array(cam.viewport_upper_left)
    center = np.array(cam.center) - 10 * w
    assert np.linalg.norm(ul - center) == pytest.approx(
        0.5 * np.hypot(cam.viewport_width, cam.viewport_height), rel=1e-5)
    assert cam.max_depth == 30 and cam.samples_per_pixel == 500 and cam.camera_has_moved == 1


@pytest.mark.parametrize("kind,n,seed", [(0, 0, 1), (1, 0, 1), (1, 0, 99), (2, 500, 1),
                                         (2, 4, 1), (2, 64, 3), (2, 1500, 2)])
def test_scene_generator_matches_restatement(rt, kind, n, seed):
    from oracle import host_ref as H
    got = rt.SphereCollection.generate(kind, n, seed).spheres
    want = H.generate_scene(kind, n, seed)
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_scene_contents(rt):
    """sphere.rs:49-136: ground first, three large last, materials encoded in color.w."""
    s = rt.synthetic_scene(500).spheres
    assert s.shape == (500, 8)
    assert list(s[0]) == [0, -1000, 0, 1000, 0.5, 0.5, 0.5, -2]
    assert [list(r) for r in s[-3:]] == [[0, 1, 0, 1, 1.5, 0, 0, 2],
                                         [-4, 1, 0, 1, 0.4, 0.2, 0.1, -2],
                                         [4, 1, 0, 1, 0.7, 0.6, 0.5, 0]]
    small = s[1:-3]
    assert np.all(small[:, 1] == np.float32(0.2)) and np.all(small[:, 3] == np.float32(0.2))
    assert np.all(np.linalg.norm(small[:, :3] - np.array([4, 0.2, 0], np.float32), axis=1) > 0.9)
    kinds = np.where(small[:, 7] < -1, 0, np.where(small[:, 7] <= 1, 1, 2))
    frac = np.bincount(kinds, minlength=3) / len(kinds)
    assert 0.7 < frac[0] < 0.9 and 0.08 < frac[1] < 0.22 and frac[2] < 0.1
    d = rt.create_default_spheres(1)
    assert 190 <= d.count <= 200  # 196 - skipped + 4


def test_frame_seeds(rt):
    from oracle import host_ref as H
    s = rt.frame_seeds(0x5EED, 1000)
    assert np.array_equal(s, H.frame_seeds(0x5EED, 1000))
    assert np.all((s >= 0) & (s < 1)) and np.all(s * 2 ** 24 == np.round(s * 2 ** 24))


def test_stripe_local_rows(rt):
    for h in (1, 7, 8, 9, 64, 1080, 2160, 2161):
        for n in (1, 2, 3, 4, 8):
            rows = [rt.stripe_local_rows(h, r, n) for r in range(n)]
            bands = (h + 7) // 8
            assert sum(rows) // 8 == bands
            assert max(rows) == rows[0]
            assert max(rows) - min(rows) <= 8


def test_argument_errors_without_device(rt):
    """Argument checks that fail before touching a device."""
    L = rt._lib.lib()
    assert L.rt_create(0, None) == 1                         # NULL out pointer
    assert L.rt_update(None, None, None, 8, 8, None, None, 0, None) == 1
    assert L.rt_destroy(None) == 6
    cnt = rt._lib.U32(0)
    assert L.rt_scene_generate(2, 3, 1, None, 0, ctypes.byref(cnt)) == 2  # N < 4
    assert L.rt_scene_generate(9, 0, 1, None, 0, ctypes.byref(cnt)) == 1
    s = rt._lib.CameraSettingsC()
    out = rt._lib.SceneCameraC()
    assert L.rt_camera_from_settings(ctypes.byref(s), 0, 10, ctypes.c_float(0), ctypes.byref(out)) == 2
    assert L.rt_driver_create(None, None, None, 8, 8, None) == 1
    assert L.rt_driver_state(None) == -1
    assert L.rt_stripe_local_rows(100, 3, 2) == 0
    assert L.rt_present_rgba8(None, None, None, 8, 8, 0, None) == 6
    assert L.rt_set_frames_per_launch(None, 4) == 6
    assert L.rt_set_frame_pairs(None, 0) == 6
    assert L.rt_set_tile_order(None, 0) == 6
    assert L.rt_set_update_queues(None, 1) == 6
    assert L.rt_get_frames_per_launch(None, None, None) == 6
    assert L.rt_selftest_fastmath(None, 0, None) == 6
    assert L.rt_last_launch_info(None, None) == 6
    # instance names are the ones rocprofv3 lists (rt_kernels.h asserts the ids)
    assert [L.rt_kernel_name(k).decode() for k in range(8)] == [
        f"rt_trace_kernel<{k}>" for k in range(5)] + [f"rt_bounce_kernel<{m}>" for m in range(3)]
    assert L.rt_set_path_compaction(None, 0) == 6
    assert L.rt_set_single_kernel(None, 0) == 6
    assert L.rt_kernel_name(8).decode() == "rt_single_kernel<2>"
    assert L.rt_kernel_name(9).decode() == "rt_single_kernel<1>"
    assert L.rt_kernel_name(99).decode() == "rt_trace_kernel"
    # the RCCL gather behind the ABI (rt_comm.cpp)
    assert L.rt_comm_unique_id(None) == 1
    assert L.rt_comm_create(None, None, 1, 0, None) == 6
    assert L.rt_comm_create_all(0, None, None) == 1
    assert L.rt_comm_destroy(None) == 1
    assert L.rt_comm_info(None, None, None, None) == 1
    assert L.rt_gather_stripes(None, None, None, None, None, 8, 8, 0, None) == 6
    assert L.rt_candidate_stats(None, None) == 6


def test_comm_unique_id_without_device(rt):
    """rt_comm_unique_id (ncclGetUniqueId) needs no GPU: 128 bytes, fresh on every call."""
    from gpu_ray_tracing.distributed import StripeComm
    a, b = StripeComm.unique_id(), StripeComm.unique_id()
    assert len(a) == len(b) == rt._lib.RT_COMM_ID_BYTES == 128
    assert a != b


def test_srgb_thresholds_match_restatement(rt):
    """The sRGB boundary table the present kernel uses (computed in C++ double) equals the
    numpy float64 restatement, bit for bit, and is strictly increasing."""
    from oracle import present_ref
    t = rt.srgb_thresholds()
    want = present_ref.srgb_thresholds()
    assert t.tobytes() == want.tobytes()
    assert np.all(np.diff(t[1:]) > 0) and t[255] < 1.0
    # j is the nearest code: the encoded value of T[j] rounds up to j, of its predecessor
    # down to j - 1
    v = t[1:].astype(np.float64)
    enc = np.where(v <= 0.0031308, v * 12.92, 1.055 * v ** (1 / 2.4) - 0.055) * 255
    assert np.all(enc >= np.arange(1, 256) - 0.5 - 1e-9)


def test_header_layout_locks_compile_in_c(tmp_path):
    """include/rt_abi.h carries _Static_assert layout locks (camera.rs:256-291,
    sphere.rs:20-26): a C translation unit compiles against it with gcc, and one that
    breaks a lock (a field inserted in a copy of the header) does not."""
    src = tmp_path / "abi_check.c"
    src.write_text('#include "rt_abi.h"\nint main(void) { return (int)sizeof(rt_scene_camera) - 176; }\n')
    ok = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", str(HEADER.parent), "-c",
                         str(src), "-o", str(tmp_path / "a.o")], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr
    broken = tmp_path / "broken"
    broken.mkdir()
    text = HEADER.read_text().replace("    float viewport_height;", "    float inserted;\n    float viewport_height;", 1)
    assert "float inserted;" in text
    (broken / "rt_abi.h").write_text(text)
    bad = subprocess.run(["gcc", "-std=c11", "-I", str(broken), "-c", str(src), "-o",
                          str(tmp_path / "b.o")], capture_output=True, text=True)
    assert bad.returncode != 0 and "static assert" in bad.stderr.lower()
    # C++ (the library's own translation units) sees the same locks
    cpp = tmp_path / "abi_check.cpp"
    cpp.write_text('#include "rt_abi.h"\nint main() { return 0; }\n')
    ok = subprocess.run(["g++", "-std=c++17", "-I", str(HEADER.parent), "-c", str(cpp), "-o",
                         str(tmp_path / "c.o")], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr


def test_ctypes_mirrors_match_the_c_layouts(rt, tmp_path):
    """Every struct the Python mirror passes through the C ABI (gpu_ray_tracing/_lib.py) has
    the size and field offsets gcc gives the header's declaration — rt_scene_camera,
    rt_sphere, rt_camera_settings and rt_launch_info (ABI 5 appended normal_rn)."""
    L = rt._lib
    mirrors = {"rt_scene_camera": L.SceneCameraC, "rt_sphere": L.SphereC,
               "rt_camera_settings": L.CameraSettingsC, "rt_launch_info": L.LaunchInfoC}
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "rt_abi.h"',
             'int main(void) {']
    for cname, py in mirrors.items():
        lines.append(f'    printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'    printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ['    return 0;', '}']
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    cc = subprocess.run(["gcc", "-std=c11", "-I", str(HEADER.parent), str(src), "-o", str(exe)],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        cname, key, val = line.split()
        got[(cname, key)] = int(val)
    for cname, py in mirrors.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


def test_bound_update_frames_passes_the_same_arguments(rt, monkeypatch):
    """bind_update_frames (what StripeRenderer.frames issues) hands rt_update_frames the
    same arguments as ComputeShaderPipeline.update_frames, reports the newest image the same
    way, and raises on a failing status — checked without a device against a stand-in for
    the library function (the GPU tests run both through the real one)."""
    import gpu_ray_tracing.compute_shader as cs

    calls = []

    def fake_update_frames(*args):
        flat = []
        for i, a in enumerate(args):
            if i == 7:                                       # the camera: its 176 bytes
                if type(a).__name__ == "CArgObject":
                    flat.append(("cam", bytes(a._obj)))
                else:
                    flat.append(("cam", ctypes.string_at(a, 176)))
            elif isinstance(a, ctypes.c_void_p):
                flat.append(("ptr", a.value))
            elif i in (8, 11) and isinstance(a, int):        # spheres / seeds addresses
                flat.append(("ptr", a))
            elif type(a).__name__ == "CArgObject":          # ctypes.byref(...)
                obj = a._obj
                flat.append(("ref", bytes(obj) if not isinstance(obj, ctypes.c_int) else "int"))
                if isinstance(obj, ctypes.c_int):
                    obj.value = 1
            else:
                flat.append(a)
        calls.append(flat)
        return fake_update_frames.status

    fake_update_frames.status = 0

    class FakeLib:
        rt_update_frames = staticmethod(fake_update_frames)

        @staticmethod
        def rt_last_error():
            return b"stand-in failure"

    class FakeImage:
        def __init__(self, addr):
            self.addr = addr

        def data_ptr(self):
            return self.addr

    sc = rt.SphereCollection.generate(rt.SCENE_DEFAULT, 0, 1)
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(), 64, 48, 0.25)
    seeds = np.array([0.25, 0.5, 0.75], np.float32)
    monkeypatch.setattr(cs._lib, "lib", lambda: FakeLib)
    monkeypatch.setattr(cs._lib, "fastcall", lambda: None)   # (the ctypes path under test)
    monkeypatch.setattr(cs, "_check_image", lambda *a: None)
    pipe = object.__new__(cs.ComputeShaderPipeline)
    pipe._ctx = ctypes.c_void_p(0x1234)
    pipe._sphere_keep = None
    monkeypatch.setattr(pipe, "_stream", lambda: ctypes.c_void_p(0x77))
    monkeypatch.setattr(cs, "stripe_local_rows", lambda h, r, n: (h + n - 1) // n)
    a, b = FakeImage(0x1000), FakeImage(0x2000)
    newest_plain = pipe.update_frames(a, b, 64, 48, cam, sc, seeds, 1, 3)
    run = pipe.bind_update_frames(a, b, 64, 48, 1, 3)
    newest_bound = run(cam, sc, seeds)
    assert newest_plain == newest_bound == 1
    assert len(calls) == 2
    # (contiguous float32 spheres and seeds are passed without copies: the same addresses)
    plain, bound = calls
    assert len(plain) == len(bound) == 14
    assert plain == bound
    fake_update_frames.status = 3
    try:
        with pytest.raises(Exception, match="stand-in failure"):
            run(cam, sc, seeds)
    finally:
        pipe._ctx = ctypes.c_void_p()   # (no context to destroy: close() skips a null one)


def test_bound_run_keeps_converted_spheres_alive(rt, monkeypatch):
    """A spheres array that is not contiguous float32 (here float64) is converted on every
    bound call, and the converted copy stays alive while the library may read it — even when
    StripeRenderer's two bound directions alternate and each converts its own copy (round-4
    ADVICE: a cached pointer into a copy freed by the other direction).  The stand-in library
    reads the sphere bytes at the pointer it is given, after freed small blocks have been
    reused."""
    import gpu_ray_tracing.compute_shader as cs
    seen = []

    def fake_update_frames(*args):
        ptr, n = args[8], args[9]
        seen.append(np.frombuffer(ctypes.string_at(ptr, n * 32), np.float32).reshape(n, 8).copy())
        return 0

    class FakeLib:
        rt_update_frames = staticmethod(fake_update_frames)

    class FakeImage:
        def __init__(self, addr):
            self.addr = addr

        def data_ptr(self):
            return self.addr

    cam = rt.SceneCamera.from_settings(rt.CameraSettings(), 16, 16, 0.25)
    monkeypatch.setattr(cs._lib, "lib", lambda: FakeLib)
    monkeypatch.setattr(cs._lib, "fastcall", lambda: None)   # (the ctypes path under test)
    monkeypatch.setattr(cs, "_check_image", lambda *a: None)
    pipe = object.__new__(cs.ComputeShaderPipeline)
    pipe._ctx = ctypes.c_void_p(0x1234)
    pipe._sphere_keep = None
    monkeypatch.setattr(pipe, "_stream", lambda: ctypes.c_void_p(0x77))
    a, b = FakeImage(0x1000), FakeImage(0x2000)
    runs = [pipe.bind_update_frames(a, b, 16, 16), pipe.bind_update_frames(b, a, 16, 16)]
    seeds = np.array([0.25], np.float32)
    rng = np.random.default_rng(3)
    sc64 = rt.SphereCollection(rng.random((5, 8)))                 # float64: converted
    sc32 = rt.SphereCollection(rng.random((5, 8)).astype(np.float32))
    want = []
    junk = []
    for k in range(8):
        sc = sc64 if k % 3 else sc32
        runs[k % 2](cam, sc, seeds)
        want.append(np.array(sc.spheres, np.float32))       # (a copy: sc32 is edited below)
        # reuse freed blocks of the converted copies' size
        junk += [np.full((5, 8), -7.0, np.float32) for _ in range(4)]
        # an in-place edit of the float32 array is still seen (no stale copy)
        sc32.spheres[0, 0] += 1.0
    assert len(seen) == len(want)
    for got, exp in zip(seen, want):
        assert np.array_equal(got, exp)
    # the direct (float32) array is passed without a copy
    runs[0](cam, sc32, seeds)
    assert np.array_equal(seen[-1], sc32.spheres)
    pipe._ctx = ctypes.c_void_p()


def test_fastcall_binding_checks_arguments_without_device(rt):
    """The CPython binding of rt_update_frames (build/_rt_fastcall*.so) reaches the library's
    own argument checks (a NULL context: -RT_ERR_INVALID_CONTEXT, no HIP call) and refuses
    buffers that are not C-contiguous float32 (the bound call then converts them)."""
    fast = rt._lib.fastcall()
    assert fast is not None, "build/_rt_fastcall*.so was not built (make -C gpu-ray-tracing_amd)"
    blob = np.zeros(44, np.float32)
    sph = np.zeros((500, 8), np.float32)
    seeds = np.zeros(20, np.float32)
    assert fast.update_frames(0, 0x1000, 0x2000, 64, 48, 0, 1, blob, sph, 500, seeds, None) == -6
    with pytest.raises(TypeError):
        fast.update_frames(0, 0x1000, 0x2000, 64, 48, 0, 1, blob, sph.astype(np.float64), 500,
                           seeds, None)
    with pytest.raises((TypeError, ValueError, BufferError)):
        fast.update_frames(0, 0x1000, 0x2000, 64, 48, 0, 1, blob, sph[:, :4], 500, seeds, None)
    with pytest.raises(ValueError):        # fewer records than the count claims
        fast.update_frames(0, 0x1000, 0x2000, 64, 48, 0, 1, blob, sph[:10], 500, seeds, None)
    with pytest.raises(TypeError):         # the camera is the 176-byte blob
        fast.update_frames(0, 0x1000, 0x2000, 64, 48, 0, 1, blob[:40], sph, 500, seeds, None)
