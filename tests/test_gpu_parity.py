"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle and the
committed golden fixtures, bit for bit (NaN == NaN).  Run on a real MI355X with -m gpu."""
import hashlib
import os

import numpy as np
import pytest
import torch

from conftest import bands_match, bits_equal, canon_sha, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["culled", "culled_one", "culled_general", "exhaustive"])
def pipe(rt, request):
    """Every parity test runs against both sphere-scan strategies, and the culled one with
    each one-frame kernel (rt_set_single_kernel: two tiles per wave, one, the general
    instance)."""
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    p = rt.ComputeShaderPipeline(0)
    p.set_scan_mode(request.param.split("_")[0])
    if request.param == "culled_general":
        p.set_single_kernel("off")
    elif request.param == "culled_one":
        p.set_single_kernel("one")
    yield p
    p.close()


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def assert_same(got, want):
    ok, bad = bits_equal(got, want)
    assert ok, f"{bad} channels differ"


def camera(rt, w, h, depth=1, spp=500, seed=0.5, moved=True, defocus=0.6, fov=20.0):
    s = rt.CameraSettings(max_depth=depth, samples_per_pixel=spp, camera_has_moved=moved,
                          defocus_angle=defocus, field_of_view=fov)
    return rt.SceneCamera.from_settings(s, w, h, seed)


SCENES = {
    "three": lambda rt: rt.three_spheres(),
    "default": lambda rt: rt.create_default_spheres(1),
    "n500": lambda rt: rt.synthetic_scene(500),
}


@pytest.mark.parametrize("scene", ["three", "default", "n500"])
@pytest.mark.parametrize("w,h,depth,defocus", [(64, 48, 1, 0.6), (67, 45, 3, 0.6),
                                               (40, 24, 8, 0.0), (16, 8, 0, 0.6),
                                               (1, 1, 2, 0.6), (129, 7, 5, 1.5)])
def test_update_matches_oracle(rt, oracle, pipe, scene, w, h, depth, defocus):
    sc = SCENES[scene](rt)
    cam = camera(rt, w, h, depth=depth, defocus=defocus, seed=0.3125)
    inp = np.zeros((h, w, 4), np.float32)
    a, b = to_dev(inp), pipe.new_image(w, h)
    pipe.update(a, b, w, h, cam, sc)
    want, _ = oracle.update(inp, cam.blob, sc.spheres)
    assert_same(host(b), want)


@pytest.mark.parametrize("seed", [3, 4])
def test_random_radii_normal_paths_match_oracle(rt, oracle, pipe, seed):
    """The hit normal's division on scenes of random radii (the seeded scene's records with
    every radius drawn from [0.05, 4) bits at random): whether or not the upload's device
    check finds every radius's refined reciprocal correctly rounded (last_launch_info's
    normal_rn, one Markstein step per component, or div_core's two), the frames match the
    oracle; depth 1 (the camera-ray-only instances) and 3."""
    base = np.array(rt.create_default_spheres(seed).spheres, np.float32).reshape(-1, 8)
    rng = np.random.default_rng(seed)
    base[:, 3] = rng.uniform(0.05, 4.0, len(base)).astype(np.float32)
    sc = rt.SphereCollection(base)
    w, h = 72, 40
    seen = set()
    for depth in (1, 3):
        cam = camera(rt, w, h, depth=depth, seed=0.40625)
        inp = np.zeros((h, w, 4), np.float32)
        a, b = to_dev(inp), pipe.new_image(w, h)
        pipe.update(a, b, w, h, cam, sc)
        seen.add(pipe.last_launch_info()["normal_rn"])
        want, _ = oracle.update(inp, cam.blob, sc.spheres)
        assert_same(host(b), want)
    assert seen <= {0, 1}


def test_update_accumulates_from_state(rt, oracle, pipe):
    """Non-zero input accumulator, no reset; samples capped at spp; reset on move."""
    w, h = 48, 40
    sc = rt.create_default_spheres(2)
    rng = np.random.default_rng(0)
    state = np.concatenate([rng.random((h, w, 3), np.float32),
                            rng.integers(0, 8, (h, w, 1)).astype(np.float32)], axis=2)
    for moved, spp in [(False, 500), (False, 4), (True, 500), (False, 0)]:
        cam = camera(rt, w, h, depth=4, spp=spp, moved=moved, seed=0.71875)
        a, b = to_dev(state), pipe.new_image(w, h)
        pipe.update(a, b, w, h, cam, sc)
        want, _ = oracle.update(state, cam.blob, sc.spheres)
        assert_same(host(b), want)


def test_golden_k1_and_accumulator(rt, pipe):
    g = load_golden("k1.npz")
    cam = rt.SceneCamera(g["camera"])
    sc = rt.SphereCollection(g["spheres"])
    a, b = pipe.new_image(256, 256), pipe.new_image(256, 256)
    pipe.update(a, b, 256, 256, cam, sc)
    assert_same(host(b), g["image"])

    g = load_golden("accum_default.npz")
    h, w = g["state0"].shape[:2]
    sc = rt.SphereCollection(g["spheres"])
    cur = to_dev(g["state0"])
    for f in range(3):
        nxt = pipe.new_image(w, h)
        pipe.update(cur, nxt, w, h, rt.SceneCamera(g["cameras"][f]), sc)
        assert_same(host(nxt), g["frames"][f])
        cur = nxt


@pytest.mark.parametrize("name", ["k2.npz", "k3.npz"])
def test_golden_full_hd_single_frame(rt, pipe, name):
    """BASELINE configs[1], [2] at full size: the whole image hashes to the oracle's."""
    g = load_golden(name)
    w, h = int(g["width"]), int(g["height"])
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.update(a, b, w, h, rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]))
    img = host(b)
    assert_same(img[g["py"], g["px"]], g["pixels"])
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["sha256"])
    assert np.array_equal(img.astype(np.float64).sum((0, 1)), g["channel_sums"])


def test_golden_k4_fused_64spp(rt, pipe):
    """configs[3]: 1920x1080, 500 spheres, 64 spp fused accumulate — full-image hash."""
    g = load_golden("k4.npz")
    w, h = int(g["width"]), int(g["height"])
    a = pipe.new_image(w, h)
    pipe.render(a, a, w, h, rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]),
                g["seeds"])
    img = host(a)
    assert_same(img[g["py"], g["px"]], g["pixels"])
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["sha256"])


@pytest.mark.parametrize("pairs", ["auto", "on", "quad", "quad2"])
def test_bench_k4_launches_match_golden(rt, pairs):
    """The kernel bench.py --config K4 times, at the timed size: rt_update_frames of 64
    frames from a reset at 1920x1080 / 500 spheres (AUTO: frame pairs over tile pairs,
    kTraceListPair2; the
    first launch records tile costs, the second runs cost-ordered tiles).  Both launches'
    newest image hashes to k4.npz's, the other buffer holds frame 63."""
    g = load_golden("k4.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    p = rt.ComputeShaderPipeline(0)
    p.set_frame_pairs(pairs)
    try:
        a, b = p.new_image(w, h), p.new_image(w, h)
        for launch in range(2):
            newest = p.update_frames(a, b, w, h, cam, sc, g["seeds"])
            info = p.last_launch_info()
            assert info["launches"] == 1 and info["max_frames_per_launch"] == 64
            assert info["kernel_name"] == {"auto": "rt_tpair_kernel<2>",
                                           "on": "rt_trace_kernel<3>",
                                           "quad": "rt_trace_kernel<4>",
                                           "quad2": "rt_tpair_kernel<4>"}[pairs]
            img = host(b if newest == 1 else a)
            assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["sha256"]), launch
            other = host(a if newest == 1 else b)
            assert np.all(other[..., 3] == 63)
    finally:
        p.close()


@pytest.mark.parametrize("single", ["auto", "one", "off"])
@pytest.mark.parametrize("cfg", ["k2", "k3"])
@pytest.mark.parametrize("submit", ["auto", "aql"])
def test_bench_dispatch_chain_matches_fixture(rt, cfg, single, submit):
    """bench.py --config K2/K3's timed structure: one update launch per frame
    (rt_set_frames_per_launch(1)), 5 + 20 frames from a reset at 1920x1080 (the driver's
    --warmup 5 --steps 20), submitted as HIP launches (auto) or AQL packets, checked against
    the oracle's sampled pixels (tests/golden/bench_k*.npz)."""
    g = load_golden(f"bench_{cfg}.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    p = rt.ComputeShaderPipeline(0)
    p.set_frames_per_launch(1)
    p.set_single_kernel(single)
    p.set_update_submit(submit)
    aql = submit == "aql" and single != "off"
    try:
        a, b = p.new_image(w, h), p.new_image(w, h)
        n0 = p.update_frames(a, b, w, h, cam, sc, g["seeds"][:5])
        if n0 == 1:
            a, b = b, a
        newest = p.update_frames(a, b, w, h, cam.with_fields(camera_has_moved=0.0), sc,
                                 g["seeds"][5:25])
        info = p.last_launch_info()
        # (the library's choice of concurrent parts per update at this size: 2 streams or
        # queues)
        assert info["launches"] == 20 * info["queues"] and info["max_frames_per_launch"] == 1
        assert info["queues"] == (1 if single == "off" else 2)
        assert info["submit"] == ("aql" if aql else "hip")
        name = {"off": "rt_trace_kernel<2>", "one": "rt_single_kernel<1>",
                "auto": "rt_single_kernel<2>"}[single]
        assert info["kernel_name"] == (name.replace("single", "chain") if aql else name)
        img = host(b if newest == 1 else a)
        k = list(g["frame_counts"]).index(25)
        assert_same(img[g["py"], g["px"]], g["pixels"][k])
        assert canon_sha(img) == str(g["sha256"][k])
    finally:
        p.close()


@pytest.mark.parametrize("cfg", ["k2", "k3"])
@pytest.mark.parametrize("normal_rn", ["on", "off"])
def test_normal_markstein_matches_fixture(rt, cfg, normal_rn, monkeypatch):
    """The hit normal's (p - C) / R (wgsl:209) as one Markstein step per component when the
    device's refined reciprocal of every radius is the correctly rounded 1 / R (checked at
    upload: TraceParams::normal_rn, reported as last_launch_info()["normal_rn"]), or with
    div_core's two correction steps (RT_NORMAL_RN=0): the 5 + 20 frames of the bench fixture
    as one-frame launches and as one frame chain, against the oracle's sampled pixels."""
    if normal_rn == "off":
        monkeypatch.setenv("RT_NORMAL_RN", "0")
    g = load_golden(f"bench_{cfg}.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    k = list(g["frame_counts"]).index(25)
    for fpl in (1, 0):
        p = rt.ComputeShaderPipeline(0)
        p.set_frames_per_launch(fpl)
        try:
            a, b = p.new_image(w, h), p.new_image(w, h)
            if p.update_frames(a, b, w, h, cam, sc, g["seeds"][:5]) == 1:
                a, b = b, a
            newest = p.update_frames(a, b, w, h, cam.with_fields(camera_has_moved=0.0), sc,
                                     g["seeds"][5:25])
            info = p.last_launch_info()
            assert info["normal_rn"] == (1 if normal_rn == "on" else 0), info
            img = host(b if newest == 1 else a)
            assert_same(img[g["py"], g["px"]], g["pixels"][k])
            assert canon_sha(img) == str(g["sha256"][k])
        finally:
            p.close()


@pytest.mark.parametrize("order", ["auto", "off"])
@pytest.mark.parametrize("single", ["auto", "one"])
@pytest.mark.parametrize("submit", ["auto", "aql"])
def test_update_queues_match_one_launch(rt, single, order, submit):
    """rt_set_update_queues: one-frame updates as 2-4 concurrent parts on their own streams
    or HSA queues (rt_set_update_submit; each part every queues-th workgroup of the cost
    order, or every queues-th band when the order is off) leave both ping-pong images
    bit-identical to one launch per update — whole image and a rank share, across the reset
    frame, the order's first build and a second call — and match the oracle's sampled pixels
    (tests/golden/bench_k3.npz).  Every part count runs on a fresh context, so the cost
    order is first built inside a call that already has parts in flight (frame 1 in raster
    bands, frame 2 in the new order: the parts are joined before the order is built)."""
    g = load_golden("bench_k3.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    cam_t = cam.with_fields(camera_has_moved=0.0)
    for rank, nranks in ((0, 1), (3, 8)):
        rows = rt.stripe_local_rows(h, rank, nranks)
        ref = None
        for q in (1, 2, 3, 4):
            p = rt.ComputeShaderPipeline(0)
            try:
                p.set_frames_per_launch(1)
                p.set_single_kernel(single)
                p.set_tile_order(order)
                p.set_update_submit(submit)
                p.set_update_queues(q)
                a, b = p.new_image(w, rows), p.new_image(w, rows)
                n0 = p.update_frames(a, b, w, h, cam, sc, g["seeds"][:5], rank, nranks)
                if n0 == 1:
                    a, b = b, a
                newest = p.update_frames(a, b, w, h, cam_t, sc, g["seeds"][5:25], rank, nranks)
                info = p.last_launch_info()
                assert info["queues"] == q and info["launches"] == 20 * q, (q, info)
                imgs = (host(b if newest == 1 else a), host(a if newest == 1 else b))
            finally:
                p.close()
            if ref is None:
                ref = imgs
                if nranks == 1:
                    k = list(g["frame_counts"]).index(25)
                    assert_same(imgs[0][g["py"], g["px"]], g["pixels"][k])
            else:
                for x, y in zip(imgs, ref):
                    assert_same(x, y)


@pytest.mark.parametrize("single", ["auto", "one"])
def test_update_submit_aql_matches_hip(rt, single):
    """rt_set_update_submit: one-frame updates as AQL packets on the context's HSA queues
    (1-4 parts, one queue each, no cache fence between a part's frames) leave both ping-pong
    images bit-identical to HIP launches — whole image and a rank share, across the reset
    frame, the workgroup order's first build and a second call; the first call starts on an
    idle stream (no go packet), the second is issued while the stream still waits for the
    first (the go packet path) — and match the oracle's sampled pixels; no go wait gave up.
    AUTO submits HIP launches at every size (AQL is opt-in since round 4)."""
    g = load_golden("bench_k3.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    cam_t = cam.with_fields(camera_has_moved=0.0)
    p = rt.ComputeShaderPipeline(0)
    st = p.submit_status()
    assert st["aql_available"], st["why"]
    p.set_frames_per_launch(1)
    p.set_single_kernel(single)
    try:
        for rank, nranks in ((0, 1), (5, 8), (1, 4)):
            rows = rt.stripe_local_rows(h, rank, nranks)
            ref = None
            for mode, q in (("hip", 1), ("aql", 1), ("aql", 2), ("aql", 3), ("aql", 4),
                            ("aql", 0), ("auto", 0)):
                p.set_update_submit(mode)
                p.set_update_queues(q)
                a, b = p.new_image(w, rows), p.new_image(w, rows)
                torch.cuda.synchronize()
                n0 = p.update_frames(a, b, w, h, cam, sc, g["seeds"][:5], rank, nranks)
                if n0 == 1:
                    a, b = b, a
                newest = p.update_frames(a, b, w, h, cam_t, sc, g["seeds"][5:25], rank, nranks)
                info = p.last_launch_info()
                want = mode if mode != "auto" else "hip"
                assert info["submit"] == want and info["frames"] == 20, (mode, q, info)
                if q:
                    assert info["queues"] == q, (mode, q, info)
                imgs = (host(b if newest == 1 else a), host(a if newest == 1 else b))
                if ref is None:
                    ref = imgs
                    if nranks == 1:
                        k = list(g["frame_counts"]).index(25)
                        assert_same(imgs[0][g["py"], g["px"]], g["pixels"][k])
                else:
                    for x, y in zip(imgs, ref):
                        assert_same(x, y)
        st = p.submit_status()
        assert st["go_give_ups"] == 0 and st["packets"] > 0, st
    finally:
        p.close()


class _HipStreamGate:
    """Holds a HIP stream at a hipStreamWaitValue32 on a signal-memory word until release()
    (hipStreamWriteValue32 from a second stream): the stream is busy, and whatever is queued
    behind the wait cannot start — a caller's stream that never reaches an AQL segment."""

    def __init__(self, stream):
        import ctypes
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.word = ctypes.c_void_p()
        assert self.hip.hipExtMallocWithFlags(ctypes.byref(self.word), ctypes.c_size_t(8),
                                              ctypes.c_uint(2)) == 0   # hipMallocSignalMemory
        assert self.hip.hipMemset(self.word, 0, ctypes.c_size_t(8)) == 0
        assert self.hip.hipDeviceSynchronize() == 0
        self.other = torch.cuda.Stream()
        self.ctypes = ctypes
        # wait until *word >= 1 (hipStreamWaitValueGte = 0), full mask
        assert self.hip.hipStreamWaitValue32(ctypes.c_void_p(stream.cuda_stream), self.word,
                                             ctypes.c_uint32(1), ctypes.c_uint(0),
                                             ctypes.c_uint32(0xFFFFFFFF)) == 0

    def release(self):
        c = self.ctypes
        assert self.hip.hipStreamWriteValue32(c.c_void_p(self.other.cuda_stream), self.word,
                                              c.c_uint32(1), c.c_uint(0)) == 0

    def close(self):
        torch.cuda.synchronize()
        self.hip.hipFree(self.word)


def test_aql_go_wait_gives_up_and_falls_back(rt, monkeypatch):
    """The AQL path's bounded go wait (rt_chain.cpp): a segment submitted while the caller's
    stream is held (a hipStreamWaitValue32 nobody satisfies within RT_CHAIN_GO_MS = 300 ms)
    gives up without running its frames early (their stores are dropped: the images keep
    what they held), the context's next call returns RT_ERR_HIP with the reason, and the calls
    after it run on HIP launches — bit-exact against tests/golden/bench_k3.npz from a reset."""
    import time
    monkeypatch.setenv("RT_CHAIN_GO_MS", "300")
    g = load_golden("bench_k3.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    cam_t = cam.with_fields(camera_has_moved=0.0)
    p = rt.ComputeShaderPipeline(0)
    gate = None
    try:
        st = p.submit_status()
        assert st["aql_available"], st["why"]
        p.set_frames_per_launch(1)
        p.set_update_submit("aql")
        a, b = p.new_image(w, h), p.new_image(w, h)
        p.update_frames(a, b, w, h, cam, sc, g["seeds"][:3])      # a working segment
        assert p.last_launch_info()["submit"] == "aql"
        torch.cuda.synchronize()
        before = (host(a).copy(), host(b).copy())
        stream = torch.cuda.current_stream()
        gate = _HipStreamGate(stream)                              # the stream is held
        p.update_frames(a, b, w, h, cam_t, sc, g["seeds"][3:7])   # go wait: never satisfied
        assert p.last_launch_info()["submit"] == "aql"
        time.sleep(1.5)                                            # > the 300-ms bound
        gate.release()
        torch.cuda.synchronize()
        # the segment's frames did not run: both images hold what they held before
        after = (host(a), host(b))
        for x, y in zip(after, before):
            assert_same(x, y)
        with pytest.raises(rt.RtError, match="go wait gave up"):
            p.update_frames(a, b, w, h, cam_t, sc, g["seeds"][3:7])
        st = p.submit_status()
        assert not st["aql_available"] and st["go_give_ups"] == 1, st
        # from now on HIP launches: the driver's 5 + 20 frames from a reset, bit-exact
        n0 = p.update_frames(a, b, w, h, cam, sc, g["seeds"][:5])
        assert p.last_launch_info()["submit"] == "hip"
        if n0 == 1:
            a, b = b, a
        newest = p.update_frames(a, b, w, h, cam_t, sc, g["seeds"][5:25])
        assert p.last_launch_info()["submit"] == "hip"
        img = host(b if newest == 1 else a)
        k = list(g["frame_counts"]).index(25)
        assert_same(img[g["py"], g["px"]], g["pixels"][k])
    finally:
        if gate is not None:
            gate.release()
            gate.close()
        p.close()


def test_bench_k5_launches_match_golden(rt):
    """bench.py --config K5's timed structure on one GPU: rt_update_frames of 64 frames
    (the bounce instance, all 64 fused in one launch) at 3840x2160, depth 8: the whole
    image's digest and every band's (the oracle rendered all 8.3 M pixels), and the 16 384
    sampled pixels for locating a difference."""
    g = load_golden("k5.npz")
    w, h = int(g["width"]), int(g["height"])
    p = rt.ComputeShaderPipeline(0)
    try:
        a, b = p.new_image(w, h), p.new_image(w, h)
        newest = p.update_frames(a, b, w, h, rt.SceneCamera(g["camera"]),
                                 rt.SphereCollection(g["spheres"]), g["seeds"])
        info = p.last_launch_info()
        assert info["frames"] == 64 and info["kernel_name"] == "rt_bounce_kernel<0>"
        img = host(b if newest == 1 else a)
        assert_same(img[g["py"], g["px"]], g["pixels"])
        assert bands_match(img, range(h // 8), g["band_sha"]) == []
        assert canon_sha(img) == str(g["sha256"])
    finally:
        p.close()


@pytest.mark.parametrize("world,paths", [(1, "split"), (4, "split"), (4, "auto"), (8, "auto"),
                                         (8, "per_wave")])
def test_bench_k5_shares_match_golden(rt, world, paths):
    """bench.py --config K5 per rank: EVERY rank's stripe share of the 64-spp 3840x2160
    depth-8 render (one 64-frame bounce launch), every pixel, against the fixture's per-band
    digests (each 8-row band of the oracle's whole image), on two consecutive steps: the
    first runs per wave under AUTO and measures the tile costs, the second runs the cost order
    (AUTO on an 8-rank share: the split schedule's unit order, the costliest tiles in four
    chunks on separate waves; the arrival counters are reused).  Forced splits on the whole
    image and a 4-rank share.  Every band boundary of the 4- and 8-rank partitions is a rank
    boundary, so this covers the pixels on both sides of each."""
    g = load_golden("k5.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    for rank in range(world):
        p = rt.ComputeShaderPipeline(0)
        p.set_path_compaction(paths)
        try:
            rows = rt.stripe_local_rows(h, rank, world)
            bands = list(range(rank, h // 8, world))
            assert rows == 8 * len(bands)
            a, b = p.new_image(w, rows), p.new_image(w, rows)
            for step in range(2):
                newest = p.update_frames(a, b, w, h, cam, sc, g["seeds"], rank, world)
                info = p.last_launch_info()
                split = paths == "split" or (paths == "auto" and world >= 8 and step == 1)
                assert info["kernel_name"] == ("rt_bounce_kernel<3>" if split
                                               else "rt_bounce_kernel<0>"), info
                img = host(b if newest == 1 else a)
                assert bands_match(img, bands, g["band_sha"]) == [], (rank, step)
                assert np.all(img[:rows, :, 3] == 64)
        finally:
            p.close()


def test_golden_k5_whole_image(rt, pipe):
    """configs[4] shape on one GPU through rt_render: 3840x2160, 500 spheres, 64 spp, depth
    8 — the whole image's digest (the oracle's 8.3 M pixels), in every scan mode."""
    g = load_golden("k5.npz")
    w, h = int(g["width"]), int(g["height"])
    a = pipe.new_image(w, h)
    pipe.render(a, a, w, h, rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]),
                g["seeds"])
    img = host(a)
    assert_same(img[g["py"], g["px"]], g["pixels"])
    assert np.all(img[..., 3] == 64)
    assert canon_sha(img) == str(g["sha256"])


@pytest.mark.parametrize("frames", [1, 3, 130])
def test_render_equals_chained_updates(rt, oracle, pipe, frames):
    """rt_render == `frames` chained rt_update calls (and the oracle), incl. >128 frames
    (several launches) and the f32 sample-count round trip."""
    w, h = 40, 32
    sc = rt.create_default_spheres(3)
    seeds = rt.frame_seeds(11, frames)
    cam = camera(rt, w, h, depth=3, spp=100)  # cap hit inside the 130-frame run
    a = pipe.new_image(w, h)
    pipe.render(a, a, w, h, cam, sc, seeds)
    fused = host(a)
    cur, nxt = pipe.new_image(w, h), pipe.new_image(w, h)
    for f in range(frames):
        c = cam.with_fields(random_seed=float(seeds[f]), camera_has_moved=cam.camera_has_moved if f == 0 else 0.0)
        pipe.update(cur, nxt, w, h, c, sc)
        cur, nxt = nxt, cur
    assert_same(fused, host(cur))
    if frames <= 3:
        want, _ = oracle.render(np.zeros((h, w, 4), np.float32), cam.blob, sc.spheres, seeds)
        assert_same(fused, want)


@pytest.mark.parametrize("nranks", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("w,h", [(64, 72), (50, 37)])
def test_stripes_partition_invariance(rt, pipe, nranks, w, h):
    """Rendering each rank's stripes separately and de-interleaving gives the full image."""
    sc = rt.synthetic_scene(100)
    seeds = rt.frame_seeds(5, 2)
    cam = camera(rt, w, h, depth=2)
    full = pipe.new_image(w, h)
    pipe.render(full, full, w, h, cam, sc, seeds)
    rows0 = rt.stripe_local_rows(h, 0, nranks)
    gathered = torch.zeros((nranks * rows0, w, 4), dtype=torch.float32, device="cuda")
    for r in range(nranks):
        rows = rt.stripe_local_rows(h, r, nranks)
        loc = pipe.new_image(w, max(rows, 1))
        if rows:
            pipe.render_stripes(loc, loc, w, h, r, nranks, cam, sc, seeds)
            gathered[r * rows0:r * rows0 + rows] = loc[:rows]
    out = pipe.new_image(w, h)
    pipe.deinterleave(gathered, out, w, h, nranks)
    assert_same(host(out), host(full))
    # numpy restatement of the de-interleave
    g = host(gathered).reshape(nranks, rows0, w, 4)
    ref = np.empty((h, w, 4), np.float32)
    for y in range(h):
        band = y // 8
        ref[y] = g[band % nranks, (band // nranks) * 8 + y % 8]
    assert_same(host(out), ref)


def test_init_and_frame_driver(rt, pipe):
    """ComputeShaderNode (lib.rs:326-421): Loading->Init zeroes B, then B->A, A->B, ..."""
    w, h = 32, 24
    sc = rt.three_spheres()
    imgs = rt.ComputeShaderImages(pipe, w, h)
    imgs.texture_b.fill_(7.0)
    node = rt.ComputeShaderNode(pipe, imgs)
    assert node.state == "Loading"
    seeds = rt.frame_seeds(9, 5)
    newest = node.frame(camera(rt, w, h, seed=float(seeds[0])), sc)
    assert node.state == "Init" and newest.data_ptr() == imgs.texture_b.data_ptr()
    assert torch.count_nonzero(imgs.texture_b).item() == 0
    ref_a, ref_b = pipe.new_image(w, h), pipe.new_image(w, h)
    states = []
    for f in range(4):
        cam = camera(rt, w, h, seed=float(seeds[f + 1]), moved=(f == 0))
        newest = node.frame(cam, sc)
        states.append(node.state)
        src, dst = (ref_b, ref_a) if f % 2 == 0 else (ref_a, ref_b)
        pipe.update(src, dst, w, h, cam, sc)
        assert_same(host(newest), host(dst))
    assert states == ["Update(1)", "Update(0)", "Update(1)", "Update(0)"]
    node.close()


def test_errors_on_device(rt, pipe):
    sc = rt.three_spheres()
    cam = camera(rt, 8, 8)
    a = pipe.new_image(8, 8)
    with pytest.raises(rt.RtError) as e:
        pipe.update(a, a, 8, 8, cam, sc)   # in == out is forbidden for update
    assert e.value.status == 1
    L = rt._lib.lib()
    import ctypes
    c = ctypes.c_void_p()
    assert L.rt_create(999, ctypes.byref(c)) == 3
    assert L.rt_init_image(pipe._ctx, ctypes.c_void_p(a.data_ptr()), 0, 8, None) == 2
    assert L.rt_init_image(pipe._ctx, ctypes.c_void_p(a.data_ptr()), 70000, 8, None) == 2


def test_nan_camera_propagates_like_oracle(rt, oracle, pipe):
    """A degenerate camera (zero pixel deltas + zero disk => zero direction => NaN) gives
    NaN where the oracle does; every sphere then counts as hit (!(NaN < 0))."""
    w, h = 16, 8
    cam = camera(rt, w, h, depth=3, defocus=0.0).with_fields(
        pixel_delta_u=(0.0, 0.0, 0.0), pixel_delta_v=(0.0, 0.0, 0.0))
    cam = cam.with_fields(viewport_upper_left=tuple(cam.center))
    three = rt.three_spheres().spheres
    # last sphere Lambertian: the NaN direction survives scatter (the metal-last scene
    # absorbs it to black instead: dot(NaN, n) > 0 is false).
    for spheres, expect_nan in ((three[[2, 1]], True), (three, False)):
        sc = rt.SphereCollection(np.ascontiguousarray(spheres))
        a, b = pipe.new_image(w, h), pipe.new_image(w, h)
        pipe.update(a, b, w, h, cam, sc)
        want, _ = oracle.update(np.zeros((h, w, 4), np.float32), cam.blob, sc.spheres)
        assert np.isnan(want).any() == expect_nan
        assert_same(host(b), want)


def test_first_sphere_wins_ties(rt, oracle, pipe):
    """Two coincident spheres: the first in the list is the hit (strict tmax <= root)."""
    w, h = 32, 32
    s = rt.three_spheres().spheres.copy()
    dup = s[1].copy()
    dup[4:8] = [0.9, 0.1, 0.1, -2.0]          # same geometry, different albedo
    sc = rt.SphereCollection(np.vstack([s, dup]))
    cam = camera(rt, w, h, depth=1)
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.update(a, b, w, h, cam, sc)
    want, _ = oracle.update(np.zeros((h, w, 4), np.float32), cam.blob, sc.spheres)
    assert_same(host(b), want)
    sc2 = rt.SphereCollection(s)
    c = pipe.new_image(w, h)
    pipe.update(a, c, w, h, cam, sc2)
    assert_same(host(b), host(c))


def test_scene_reupload_on_change(rt, oracle, pipe):
    """Changing sphere bytes between calls re-uploads (prepare_sphere_buffer semantics)."""
    w, h = 24, 16
    cam = camera(rt, w, h, depth=2)
    sc1, sc2 = rt.synthetic_scene(50, seed=1), rt.synthetic_scene(300, seed=2)
    for sc in (sc1, sc2, sc1):
        a, b = pipe.new_image(w, h), pipe.new_image(w, h)
        pipe.update(a, b, w, h, cam, sc)
        want, _ = oracle.update(np.zeros((h, w, 4), np.float32), cam.blob, sc.spheres)
        assert_same(host(b), want)


def test_full_size_properties(rt, pipe):
    """3840x2160 (configs[4] frame size), depth 8: fused == chained, stripes == full,
    deterministic across runs."""
    w, h = 3840, 2160
    sc = rt.synthetic_scene(500)
    seeds = rt.frame_seeds(0x5EED, 2)
    cam = camera(rt, w, h, depth=8, spp=64)
    full = pipe.new_image(w, h)
    pipe.render(full, full, w, h, cam, sc, seeds)
    again = pipe.new_image(w, h)
    pipe.render(again, again, w, h, cam, sc, seeds)
    assert torch.equal(full, again)
    cur, nxt = pipe.new_image(w, h), pipe.new_image(w, h)
    for f in range(2):
        pipe.update(cur, nxt, w, h, cam.with_fields(random_seed=float(seeds[f]),
                                                   camera_has_moved=1.0 if f == 0 else 0.0), sc)
        cur, nxt = nxt, cur
    assert torch.equal(full, cur)
    n = 8
    rows0 = rt.stripe_local_rows(h, 0, n)
    gathered = torch.zeros((n * rows0, w, 4), dtype=torch.float32, device="cuda")
    for r in range(n):
        rows = rt.stripe_local_rows(h, r, n)
        loc = pipe.new_image(w, rows)
        pipe.render_stripes(loc, loc, w, h, r, n, cam, sc, seeds)
        gathered[r * rows0:r * rows0 + rows] = loc
    out = pipe.new_image(w, h)
    pipe.deinterleave(gathered, out, w, h, n)
    assert torch.equal(out, full)


def _random_scene(rng, n):
    """Spheres of mixed sizes (incl. huge, tiny, zero and negative radii) and materials."""
    s = np.zeros((n, 8), np.float32)
    s[:, 0:3] = rng.uniform(-15, 15, (n, 3))
    s[:, 1] = rng.uniform(-1, 4, n)
    s[:, 3] = rng.choice([0.2, 0.5, 1.0, 3.0, 0.01, 0.0, -0.4], n)
    kind = rng.integers(0, 3, n)
    s[:, 4:7] = rng.uniform(0, 1, (n, 3))
    s[:, 7] = np.where(kind == 0, -2.0, np.where(kind == 1, rng.uniform(0, 0.5, n), 2.0))
    s[kind == 2, 4] = 1.5
    s[0] = [0, -1000, 0, 1000, 0.5, 0.5, 0.5, -2]
    return s


@pytest.mark.parametrize("seed", range(6))
def test_culled_scan_equals_exhaustive(rt, seed):
    """Exactness of the wave-level culling: random cameras (position, fov, lens), random
    scenes of 40-700 spheres, depth 1-6, several frames — bitwise equal to the exhaustive
    linear scan on the full image."""
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(64, 400)), int(rng.integers(48, 300))
    n = int(rng.integers(40, 700))
    sc = rt.SphereCollection(_random_scene(rng, n))
    s = rt.CameraSettings(field_of_view=float(rng.uniform(5, 120)),
                          max_depth=int(rng.integers(1, 7)),
                          defocus_angle=float(rng.choice([0.0, 0.6, 3.0])),
                          focus_distance=float(rng.uniform(2, 20)),
                          look_from=tuple(rng.uniform(-20, 20, 3)),
                          look_at=tuple(rng.uniform(-3, 3, 3)))
    cam = rt.SceneCamera.from_settings(s, w, h, float(rng.uniform()))
    seeds = rt.frame_seeds(seed, 3)
    out = {}
    for mode in ("culled", "exhaustive"):
        p = rt.ComputeShaderPipeline(0)
        p.set_scan_mode(mode)
        img = p.new_image(w, h)
        p.render(img, img, w, h, cam, sc, seeds)
        out[mode] = host(img)
        p.close()
    assert_same(out["culled"], out["exhaustive"])


def _lattice_scene(rng, jitter=0.9, twins=False, y_spread=0.0):
    """RTIOW-like layout: small spheres on a unit lattice, three large ones, the ground."""
    rows = []
    for a in range(-11, 11):
        for b in range(-11, 11):
            x = a + jitter * rng.uniform()
            z = b + jitter * rng.uniform()
            y = 0.2 + y_spread * rng.uniform()
            mat = rng.integers(0, 3)
            fuzz = -2.0 if mat == 0 else (rng.uniform(0, 0.5) if mat == 1 else 2.0)
            col = [1.5, 1.0, 1.0] if mat == 2 else list(rng.uniform(0, 1, 3))
            rows.append([x, y, z, 0.2] + col + [fuzz])
            if twins and rng.uniform() < 0.3:
                rows.append(rows[-1][:])          # coincident: the lower index must win
    rows += [[0, 1, 0, 1.0, 1.5, 1, 1, 2.0], [-4, 1, 0, 1.0, 0.4, 0.2, 0.1, -2.0],
             [4, 1, 0, 1.0, 0.7, 0.6, 0.5, 0.0]]
    s = np.array([[0, -1000, 0, 1000, 0.5, 0.5, 0.5, -2]] + rows, np.float32)
    return s


@pytest.mark.parametrize("case", ["lattice", "twins", "inside", "down", "tall", "aligned"])
def test_grid_walk_equals_exhaustive(rt, case):
    """Bounce rays whose wave cone is too wide walk the XZ grid of the small spheres
    (rt_kernels.hip scan_grid): bitwise equal to the exhaustive scan, for coincident
    spheres (index tie-break), a camera inside the cluster, rays straight down (zero x/z
    direction components), a tall slab and spheres centred on cell boundaries."""
    rng = np.random.default_rng(["lattice", "twins", "inside", "down", "tall",
                                 "aligned"].index(case) + 11)
    spheres = _lattice_scene(rng, jitter=0.0 if case == "aligned" else 0.9,
                             twins=case == "twins", y_spread=25.0 if case == "tall" else 0.0)
    sc = rt.SphereCollection(spheres)
    # (looking straight down: a tiny z offset keeps the camera basis defined)
    look_from, look_at, fov, lens = {
        "inside": ((0.3, 0.6, 0.2), (5.0, 0.3, 2.0), 90.0, 0.6),
        "down": ((0.0, 20.0, 1e-3), (0.0, 0.0, 0.0), 60.0, 0.0)}.get(
        case, ((13.0, 2.0, 3.0), (0.0, 0.0, 0.0), 20.0, 0.6))
    settings = rt.CameraSettings(field_of_view=fov, max_depth=8, defocus_angle=lens,
                                 focus_distance=10.0, look_from=look_from, look_at=look_at)
    w, h = 192, 128
    cam = rt.SceneCamera.from_settings(settings, w, h, 0.375)
    seeds = rt.frame_seeds(5, 3)
    out = {}
    for mode in ("culled", "exhaustive"):
        p = rt.ComputeShaderPipeline(0)
        p.set_scan_mode(mode)
        img = p.new_image(w, h)
        p.render(img, img, w, h, cam, sc, seeds)
        out[mode] = host(img)
        p.close()
    assert_same(out["culled"], out["exhaustive"])


@pytest.mark.parametrize("depth", [1, 2])
def test_candidate_lists_follow_camera_and_scene(rt, oracle, depth):
    """The per-tile camera-ray candidate lists are rebuilt when the camera geometry, the
    scene or the stripe partition change, and reused across frames (seed, reset, spp).
    depth 1 runs the list-only kernel instance, depth 2 the list + cone-culling one."""
    w, h = 96, 64
    p = rt.ComputeShaderPipeline(0)
    p.set_scan_mode("culled")
    sc = rt.synthetic_scene(300, seed=3)
    cams = [camera(rt, w, h, depth=depth, seed=0.125),
            rt.SceneCamera.from_settings(rt.CameraSettings(look_from=(-9.0, 3.0, 7.0),
                                                           max_depth=depth), w, h, 0.625)]
    for cam in cams + cams[:1]:
        for seed in (0.25, 0.75):
            c = cam.with_fields(random_seed=seed)
            a, b = p.new_image(w, h), p.new_image(w, h)
            p.update(a, b, w, h, c, sc)
            want, _ = oracle.update(np.zeros((h, w, 4), np.float32), c.blob, sc.spheres)
            assert_same(host(b), want)
    p.close()


@pytest.mark.parametrize("depth", [1, 3])
def test_candidate_list_overflow_falls_back(rt, depth):
    """A tile whose camera rays can reach more spheres than a list holds (a dense cluster
    straight ahead) uses the per-wave culled scan instead — still bit-exact."""
    rng = np.random.default_rng(7)
    n = 400
    s = np.zeros((n, 8), np.float32)
    s[:, 0:3] = rng.normal(0, 0.05, (n, 3)) + np.array([0, 1, 0], np.float32)
    s[:, 3] = 0.01
    s[:, 4:7] = 0.5
    s[:, 7] = -2.0
    s[0] = [0, -1000, 0, 1000, 0.5, 0.5, 0.5, -2]
    sc = rt.SphereCollection(s)
    w, h = 64, 64
    # aimed at the cluster: the middle tiles' cones admit far more than kCandMax spheres
    cam = rt.SceneCamera.from_settings(rt.CameraSettings(field_of_view=3.0, max_depth=depth,
                                                         look_at=(0.0, 1.0, 0.0)), w, h, 0.5)
    out = {}
    for mode in ("culled", "exhaustive"):
        p = rt.ComputeShaderPipeline(0)
        p.set_scan_mode(mode)
        img = p.new_image(w, h)
        p.render(img, img, w, h, cam, sc, rt.frame_seeds(3, 2))
        out[mode] = host(img)
        if mode == "culled":
            st = p.candidate_stats()
            # the cluster fills the middle tiles: more spheres than a list holds
            assert st["tiles"] == 64 and st["tiles_without_list"] > 0
            assert st["capacity"] == 19 and st["max_entries"] <= 19
        p.close()
    assert_same(out["culled"], out["exhaustive"])


@pytest.mark.parametrize("nranks", [1, 3])
@pytest.mark.parametrize("frames,depth,spp,per", [(5, 2, 500, 0), (20, 1, 500, 0), (3, 8, 500, 0),
                                                  (7, 1, 4, 0), (4, 1, 500, 1), (6, 3, 500, 4),
                                                  (5, 8, 500, 4), (9, 2, 3, 3), (14, 1, 500, 4),
                                                  (11, 1, 6, 3)])
@pytest.mark.parametrize("pairs", ["off", "on", "quad", "on2", "quad2"])
@pytest.mark.parametrize("images", ["last_two", "every"])
def test_update_frames_equals_chained_updates(rt, pipe, nranks, frames, depth, spp, per, pairs,
                                              images):
    """rt_update_frames (frames fused per launch, the last two or every frame's image stored
    to the ping-pong buffers, rt_set_frame_images; or one dispatch per frame) leaves BOTH
    buffers exactly as chained
    rt_update calls do: the newest frame and the one before, for the whole image and for
    stripe ranks (compact local buffers), across launch boundaries and the spp cap, with
    and without frame groups (several waves per tile on alternate frames); the depth-1
    cases with several fused launches also run the cost-ordered tile schedule (the first
    launch records tile costs, the later ones trace the costliest tiles first)."""
    w, h = 56, 40
    sc = rt.synthetic_scene(120)
    seeds = rt.frame_seeds(21, frames)
    cam = camera(rt, w, h, depth=depth, spp=spp)
    full_a, full_b = pipe.new_image(w, h), pipe.new_image(w, h)
    cur, nxt = full_a, full_b
    for f in range(frames):
        pipe.update(cur, nxt, w, h, cam.with_fields(random_seed=float(seeds[f]),
                                                   camera_has_moved=1.0 if f == 0 else 0.0), sc)
        cur, nxt = nxt, cur
    want_new, want_prev = host(cur), host(nxt)
    rows0 = rt.stripe_local_rows(h, 0, nranks)
    got_new = np.zeros((h, w, 4), np.float32)
    got_prev = np.zeros((h, w, 4), np.float32)
    pipe.set_frames_per_launch(per)
    pipe.set_frame_pairs(pairs)
    pipe.set_frame_images(images)
    try:
        for r in range(nranks):
            a, b = pipe.new_image(w, rows0), pipe.new_image(w, rows0)
            newest = pipe.update_frames(a, b, w, h, cam, sc, seeds, r, nranks)
            img_new, img_prev = (host(a), host(b)) if newest == 0 else (host(b), host(a))
            rows = rt.stripe_local_rows(h, r, nranks)
            for lr in range(rows):
                band = r + (lr // 8) * nranks
                y = band * 8 + lr % 8
                if y < h:
                    got_new[y], got_prev[y] = img_new[lr], img_prev[lr]
    finally:
        pipe.set_frames_per_launch(0)
        pipe.set_frame_pairs("auto")
        pipe.set_frame_images("last_two")
    assert (newest == 0) == (frames % 2 == 0)
    assert_same(got_new, want_new)
    if frames >= 2:
        assert_same(got_prev, want_prev)


# (AUTO splits only once a launch has measured the tile costs: each launch of
# _check_bounce_launches without frames_per_launch is the first of its candidate generation,
# so AUTO runs per wave there; the K5 share test covers its split on the second step)
BOUNCE_PATH_KERNEL = {"per_wave": 0, "compact": 1, "pair": 2, "auto": 0, "split": 3,
                      "split_part": 3, "split_lpt": 3}
# split_part: three chunks for the costliest 30 % of the tiles (the order's first slots), one
# unit for every other tile; split_lpt: once an order is measured, the unit order with a
# threshold that splits only the costlier tiles of these small images (alpha 150: tiles above
# ~1.8 % of the launch's total cost) — rt_abi.cpp plan_split, RT_BOUNCE_SPLIT / RT_SPLIT_FRAC /
# RT_SPLIT_ALPHA
SPLIT_ENV = {"split_part": {"RT_BOUNCE_SPLIT": "3", "RT_SPLIT_FRAC": "0.3"},
             "split_lpt": {"RT_BOUNCE_SPLIT": "2", "RT_SPLIT_ALPHA": "150"}}
SPLIT_ENV_KEYS = ("RT_BOUNCE_SPLIT", "RT_SPLIT_FRAC", "RT_SPLIT_ALPHA")


def bounce_kernel(paths, frames_per_launch):
    """The instance a bounce launch runs: AUTO / split at these small sizes split each tile's
    frames into chunks (rt_bounce_kernel<3>) when the launch carries two frames or more."""
    k = BOUNCE_PATH_KERNEL[paths]
    return 0 if k == 3 and frames_per_launch < 2 else k


def _check_bounce_launches(rt, oracle, paths, w, h, depth, frames, scene, nranks, fpl,
                           images="last_two"):
    sc = {"n120": rt.synthetic_scene(120), "default": rt.create_default_spheres(seed=3),
          "three": rt.three_spheres()}[scene]
    seeds = rt.frame_seeds(33, frames)
    cam = camera(rt, w, h, depth=depth, spp=500)
    yy, xx = np.mgrid[0:h, 0:w]
    want_new, _ = oracle.render_pixels(np.zeros((h * w, 4), np.float32), xx.ravel(), yy.ravel(),
                                       cam.blob, sc.spheres, seeds)
    want_prev, _ = oracle.render_pixels(np.zeros((h * w, 4), np.float32), xx.ravel(),
                                        yy.ravel(), cam.blob, sc.spheres, seeds[:frames - 1])
    p = rt.ComputeShaderPipeline(0)
    p.set_path_compaction("split" if paths in SPLIT_ENV else paths)
    p.set_frame_images(images)
    if fpl:
        p.set_frames_per_launch(fpl)
    rows0 = rt.stripe_local_rows(h, 0, nranks)
    got_new = np.zeros((h, w, 4), np.float32)
    got_prev = np.zeros((h, w, 4), np.float32)
    saved = {k: os.environ.get(k) for k in SPLIT_ENV_KEYS}
    for k in SPLIT_ENV_KEYS:
        os.environ.pop(k, None)
    os.environ.update(SPLIT_ENV.get(paths, {}))
    try:
        for r in range(nranks):
            a, b = p.new_image(w, rows0), p.new_image(w, rows0)
            newest = p.update_frames(a, b, w, h, cam, sc, seeds, r, nranks)
            info = p.last_launch_info()
            if depth >= 2:
                per = (frames % fpl or fpl) if fpl else frames   # the call's last launch
                assert info["kernel_name"] == "rt_bounce_kernel<%d>" % bounce_kernel(paths, per)
                if fpl and rt.stripe_local_rows(h, r, nranks):
                    assert info["launches"] == -(-frames // fpl)
            img_new, img_prev = (host(a), host(b)) if newest == 0 else (host(b), host(a))
            for lr in range(rt.stripe_local_rows(h, r, nranks)):
                y = (r + (lr // 8) * nranks) * 8 + lr % 8
                if y < h:
                    got_new[y], got_prev[y] = img_new[lr], img_prev[lr]
    finally:
        p.close()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert_same(got_new, want_new.reshape(h, w, 4))
    if frames >= 2:
        assert_same(got_prev, want_prev.reshape(h, w, 4))


@pytest.mark.parametrize("paths", ["per_wave", "compact", "pair", "split", "split_part",
                                   "split_lpt", "auto"])
@pytest.mark.parametrize("w,h,depth,frames,scene,nranks", [
    (56, 40, 2, 5, "n120", 1), (67, 45, 8, 3, "default", 1), (64, 48, 3, 1, "n120", 1),
    (50, 37, 8, 6, "default", 3), (40, 32, 0, 2, "n120", 1), (72, 48, 5, 4, "three", 2)])
def test_bounce_launches_match_oracle(rt, oracle, paths, w, h, depth, frames, scene, nranks):
    """The bounce instance (max_depth >= 2, frames fused per launch, 4-tile workgroups),
    with live paths compacted across the workgroup after every bounce or kept per wave:
    both ping-pong buffers equal the oracle's chained updates (the newest frame and the one
    before), whole image and stripe ranks, ragged edges included."""
    _check_bounce_launches(rt, oracle, paths, w, h, depth, frames, scene, nranks, 0)


@pytest.mark.parametrize("paths", ["per_wave", "compact", "pair", "split", "split_part",
                                   "split_lpt"])
@pytest.mark.parametrize("w,h,depth,frames,scene,nranks", [
    (56, 40, 2, 5, "n120", 1), (50, 37, 8, 6, "default", 3), (72, 48, 5, 4, "three", 2)])
@pytest.mark.parametrize("images", ["last_two", "every"])
def test_bounce_launches_in_tile_order(rt, oracle, paths, w, h, depth, frames, scene, nranks,
                                       images):
    """Two frames per launch (rt_set_frames_per_launch(2)): the first launch records the
    per-tile (compact mode: per-workgroup) costs, every later launch runs the measured
    cost order (tile_order) — both ping-pong buffers still equal the oracle's chain, in
    every path mode, with the last two or every frame's image stored."""
    _check_bounce_launches(rt, oracle, paths, w, h, depth, frames, scene, nranks, 2, images)


@pytest.mark.parametrize("variant", ["far_sphere", "huge_ground", "mixed_counts"])
def test_bounce_fast_core_fallbacks_match_oracle(rt, oracle, variant):
    """The bounce instance's exact fast cores on the inputs their wave-wide
    checks send back to the IEEE operations, against the oracle's chained updates:
    far_sphere — one sphere 2^41 away, so the scene fails TraceParams::roots_fast (IEEE
    roots, no grid: cone and exhaustive scans); huge_ground — a ground sphere of radius 2^21,
    outside the normal's [2^-20, 2^20] (its hits take the IEEE (p - C) / R while the small
    spheres' take the cores); mixed_counts — an image the library believes at count 1 with a
    sprinkling of pixels rewritten to other counts behind its back: waves holding one of them
    compute their scatter random numbers per lane and accumulate by the IEEE division, the
    others read the device table and take the Markstein step."""
    w, h, depth = 64, 48, 3
    base = np.array(rt.create_default_spheres(3).spheres, np.float32).reshape(-1, 8)
    if variant == "far_sphere":
        far = np.array([[2.0 ** 41, 0.0, 0.0, 1.0, 0.5, 0.5, 0.5, -2.0]], np.float32)
        base = np.concatenate([base, far])
    elif variant == "huge_ground":
        base[0, 1], base[0, 3] = -(2.0 ** 21), 2.0 ** 21
    sc = rt.SphereCollection(base)
    seeds = rt.frame_seeds(21, 4)
    cam = camera(rt, w, h, depth=depth, spp=500, seed=0.375)
    p = rt.ComputeShaderPipeline(0)
    try:
        a, b = p.new_image(w, h), p.new_image(w, h)
        if variant != "mixed_counts":
            newest = p.update_frames(a, b, w, h, cam, sc, seeds, 0, 1)
            assert p.last_launch_info()["kernel_name"].startswith("rt_bounce_kernel")
            yy, xx = np.mgrid[0:h, 0:w]
            want, _ = oracle.render_pixels(np.zeros((h * w, 4), np.float32), xx.ravel(),
                                           yy.ravel(), cam.blob, sc.spheres, seeds)
            assert_same(host(b if newest == 1 else a), want.reshape(h, w, 4))
            return
        # one reset frame: the library records count 1 for b
        assert p.update_frames(a, b, w, h, cam, sc, seeds[:1], 0, 1) == 1
        state = host(b).copy()
        rng = np.random.default_rng(5)
        pick = rng.random((h, w)) < 0.01          # ~30 pixels in a few waves
        state[pick, 3] = rng.integers(2, 6, int(pick.sum())).astype(np.float32)
        state[pick, :3] = rng.random((int(pick.sum()), 3), np.float32)
        b.copy_(to_dev(state))
        still = cam.with_fields(camera_has_moved=0.0)
        newest = p.update_frames(b, a, w, h, still, sc, seeds[1:], 0, 1)
        ref, prev = state, None
        for s_ in seeds[1:]:
            prev = ref
            ref, _ = oracle.update(ref, still.with_fields(random_seed=float(s_)).blob,
                                   sc.spheres)
        got_new, got_prev = (host(a), host(b)) if newest == 1 else (host(b), host(a))
        assert_same(got_new, ref)
        assert_same(got_prev, prev)
    finally:
        p.close()


def test_accumulator_written_outside_the_library(rt, oracle, pipe):
    """Accumulators written behind the library's back (mixed per-pixel counts, NaN,
    fractional and negative counts) after init_image and between fused frames."""
    w, h = 67, 45
    sc = rt.create_default_spheres(3)
    rng = np.random.default_rng(7)
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.init_image(a, w, h)
    counts = rng.integers(0, 6, (h, w, 1)).astype(np.float32)
    counts[::3, ::2] = 0.0
    counts[5, 7], counts[6, 8], counts[7, 9] = np.nan, 2.5, -3.0
    state = np.concatenate([rng.random((h, w, 3), np.float32), counts], axis=2)
    a.copy_(to_dev(state))                        # written behind the library's back
    cam = camera(rt, w, h, depth=3, spp=4, moved=False, seed=0.40625)
    pipe.update(a, b, w, h, cam, sc)
    want, _ = oracle.update(state, cam.blob, sc.spheres)
    assert_same(host(b), want)
    # a fused 3-frame render continues from it
    seeds = np.array([0.125, 0.5, 0.875], np.float32)
    pipe.render(b, a, w, h, cam, sc, seeds)
    cur = want
    for s in seeds:
        cur, _ = oracle.update(cur, cam.with_fields(random_seed=float(s)).blob, sc.spheres)
    assert_same(host(a), cur)


@pytest.mark.parametrize("encoding", ["linear", "srgb"])
def test_present_matches_restatement(rt, pipe, encoding):
    """rt_present_rgba8 == the numpy restatement: every threshold neighbour,
    special values, and a rendered image."""
    from oracle import present_ref as P
    t = P.srgb_thresholds()
    vals = np.concatenate([t, np.nextafter(t, np.float32(-1)), np.nextafter(t, np.float32(2)),
                           np.float32([np.nan, np.inf, -np.inf, -0.0, 1.0, 1.5, -2.0]),
                           np.linspace(-0.1, 1.1, 1000, dtype=np.float32)]).astype(np.float32)
    n = vals.size
    w = 64
    h = (n + w * 3 - 1) // (w * 3)
    img = np.zeros(h * w * 4, np.float32).reshape(h, w, 4)
    flat = np.resize(vals, h * w * 3).reshape(h, w, 3)
    img[..., :3] = flat
    got = host(pipe.present(to_dev(img), w, h, encoding))
    np.testing.assert_array_equal(got, P.present(img, encoding))
    # a rendered frame
    w, h = 96, 64
    sc = rt.create_default_spheres(5)
    cam = camera(rt, w, h, depth=4, seed=0.25)
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.update(a, b, w, h, cam, sc)
    np.testing.assert_array_equal(host(pipe.present(b, w, h, encoding)),
                                  P.present(host(b), encoding))


def test_image_files_from_device(rt, pipe, tmp_path):
    w, h = 40, 24
    sc = rt.three_spheres()
    cam = camera(rt, w, h, depth=3, seed=0.75)
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.update(a, b, w, h, cam, sc)
    rt.image_io.save_png(tmp_path / "f.png", pipe.present(b, w, h))
    rt.image_io.save_npy(tmp_path / "f.npy", b)
    from oracle import present_ref as P
    np.testing.assert_array_equal(rt.image_io.load_png(tmp_path / "f.png"),
                                  P.present(host(b), "srgb"))
    assert np.load(tmp_path / "f.npy").tobytes() == host(b).tobytes()


def test_fastmath_selftest(rt):
    """The exact fast paths of division / sqrt (rt_device.h) return the IEEE bits: all 2^32
    inputs of the defocus-disk normalisation, 2^26 random division and sqrt cases, and
    the scan's root selection on them (consider_fast) picks the same root and sphere as
    the IEEE one on 2^26 random camera-domain rays and spheres."""
    p = rt.ComputeShaderPipeline(0)
    out = p.selftest_fastmath(1 << 26)
    p.close()
    assert out[:4] == [0, 0, 0, 0], out
    assert out[4] == (1 << 32) + (1 << 26)


@pytest.mark.parametrize("depth,spp", [(1, 500), (3, 3), (8, 500)])
def test_hinted_chain_matches_oracle(rt, oracle, pipe, depth, spp):
    """Chained updates the library can hint (init, reset, then its own outputs), including
    the spp cap, and an image rewritten behind the library's back mid-chain (all pixels,
    then some pixels, with counts other than the hinted one)."""
    w, h = 40, 24
    sc = rt.synthetic_scene(500)
    seeds = rt.frame_seeds(5, 6)
    cur, nxt = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.init_image(cur, w, h)
    ref = np.zeros((h, w, 4), np.float32)
    for f in range(6):
        cam = camera(rt, w, h, depth=depth, spp=spp, moved=(f == 2), seed=float(seeds[f]))
        if f == 3:   # every pixel: a count the hint does not expect
            ref = ref.copy()
            ref[..., 3] += 1.0
            cur.copy_(to_dev(ref))
        if f == 4:   # one pixel only
            ref = ref.copy()
            ref[3, 5, 3] = 0.0
            cur.copy_(to_dev(ref))
        pipe.update(cur, nxt, w, h, cam, sc)
        ref, _ = oracle.update(ref, cam.blob, sc.spheres)
        cur, nxt = nxt, cur
        assert_same(host(cur), ref)


@pytest.mark.parametrize("pairs", ["off", "on", "quad", "on2", "quad2"])
def test_update_frames_with_foreign_counts(rt, oracle, pipe, pairs):
    """rt_update_frames on an image whose counts the library did not write (mixed per-pixel
    counts behind its back, after init_image): the hinted / frame-pair launch falls back to
    per-pixel counts and still equals the oracle's chain, both buffers."""
    w, h = 40, 24
    sc = rt.synthetic_scene(200)
    rng = np.random.default_rng(3)
    a, b = pipe.new_image(w, h), pipe.new_image(w, h)
    pipe.init_image(a, w, h)                      # the library now expects count 0
    counts = rng.integers(0, 3, (h, w, 1)).astype(np.float32)
    state = np.concatenate([rng.random((h, w, 3), np.float32), counts], axis=2)
    a.copy_(to_dev(state))
    seeds = rt.frame_seeds(9, 5)
    cam = camera(rt, w, h, depth=1, spp=500, moved=False)
    pipe.set_frame_pairs(pairs)
    try:
        newest = pipe.update_frames(a, b, w, h, cam, sc, seeds, 0, 1)
    finally:
        pipe.set_frame_pairs("auto")
    ref, prev = state, None
    for s_ in seeds:
        prev = ref
        ref, _ = oracle.update(ref, cam.with_fields(random_seed=float(s_)).blob, sc.spheres)
    assert newest == 1
    assert_same(host(b), ref)
    assert_same(host(a), prev)


def test_tile_order_does_not_change_pixels(rt, pipe):
    """Cost-ordered tiles (rt_set_tile_order AUTO: the first fused launch of a camera
    measures, the next ones sort and reorder the workgroups) leave both ping-pong buffers
    bit-identical to raster order, for the whole image and a stripe rank."""
    w, h = 72, 48
    sc = rt.synthetic_scene(300)
    seeds = rt.frame_seeds(31, 24)
    cam = camera(rt, w, h, depth=1, spp=500)
    out = {}
    pipe.set_frames_per_launch(6)
    try:
        for mode in ("off", "auto"):
            pipe.set_tile_order(mode)
            for r, n in ((0, 1), (1, 2)):
                rows = rt.stripe_local_rows(h, r, n) if n > 1 else h
                a, b = pipe.new_image(w, rows), pipe.new_image(w, rows)
                newest = pipe.update_frames(a, b, w, h, cam, sc, seeds, r, n)
                out[mode, r, n] = (newest, host(a), host(b))
    finally:
        pipe.set_frames_per_launch(0)
        pipe.set_tile_order("auto")
    for key in ((0, 1), (1, 2)):
        na, a0, b0 = out[("off",) + key]
        nb, a1, b1 = out[("auto",) + key]
        assert na == nb
        assert_same(a1, a0)
        assert_same(b1, b0)


def _k5_partition(rt, p, g, world):
    """rt_partition_bands over the band costs a whole-image 64-frame K5 launch records."""
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    a, b = p.new_image(w, h), p.new_image(w, h)
    p.update_frames(a, b, w, h, cam, sc, g["seeds"])          # records the tile costs
    costs = p.band_costs(w, h, (0, 1, h // 8))
    assert costs.shape == (h // 8,) and np.all(costs > 0) and np.all(np.isfinite(costs))
    with pytest.raises(rt.RtError):                            # not the share that ran
        p.band_costs(w, h, (0, 2, h // 16))
    return rt.partition_bands(costs, world), costs


@pytest.mark.parametrize("world", [4, 8])
def test_k5_cost_balanced_partition_matches_golden(rt, world):
    """The cost-balanced partition (verdict r05 item 2): the band costs of a whole-image K5
    launch (rt_band_costs), cut into `world` contiguous ranges (rt_partition_bands); every
    rank renders its range with rt_update_frames_bands (two steps: per wave, then the cost
    order / split schedule), every band of every rank equal to the oracle's (per-band
    digests); the ranks' buffers, padded to the largest range, de-interleaved by
    rt_deinterleave_bands into the image whose digest is the oracle's whole image."""
    g = load_golden("k5.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    p = rt.ComputeShaderPipeline(0)
    try:
        part, costs = _k5_partition(rt, p, g, world)
        loads = [costs[f:f + c].sum() for f, _, c in part]
        assert max(loads) <= costs.sum() / world + costs.max()
        rows0 = max(c for _, _, c in part) * 8
        gathered = torch.zeros((world * rows0, w, 4), dtype=torch.float32, device="cuda")
        for rank, bs in enumerate(part):
            f, st, c = bs
            a = gathered[rank * rows0:rank * rows0 + rows0]
            b = p.new_image(w, rows0)
            for step in range(2):
                newest = p.update_frames_bands(a, b, w, h, bs, cam, sc, g["seeds"])
                img = host(b if newest == 1 else a)
                assert bands_match(img, range(f, f + c), g["band_sha"]) == [], (rank, step)
            if newest == 1:
                a.copy_(b)
        out = p.new_image(w, h)
        p.deinterleave_bands(gathered, out, w, h, part, rows0)
        assert canon_sha(host(out)) == str(g["sha256"])
    finally:
        p.close()


def test_band_set_equals_stripes(rt):
    """rt_update_frames_bands with the round-robin set of rank r of n is rt_update_frames
    (r, n): the same bits (K3 bench fixture, 5 + 20 frames, frame chains and one launch per
    frame); a contiguous range of the K3 image against the fixture's band digests."""
    g = load_golden("bench_k3.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    still = cam.with_fields(camera_has_moved=0.0)
    k = list(g["frame_counts"]).index(25)
    for fpl, bs in ((0, rt.stripe_band_set(h, 3, 8)), (1, rt.stripe_band_set(h, 1, 4)),
                    (0, (40, 1, 57)), (1, (7, 1, 30)), (0, (0, 3, 45))):
        p = rt.ComputeShaderPipeline(0)
        p.set_frames_per_launch(fpl)
        p.set_frame_images("every")
        try:
            rows = bs[2] * 8
            a, b = p.new_image(w, rows), p.new_image(w, rows)
            if p.update_frames_bands(a, b, w, h, bs, cam, sc, g["seeds"][:5]) == 1:
                a, b = b, a
            newest = p.update_frames_bands(a, b, w, h, bs, still, sc, g["seeds"][5:25])
            img = host(b if newest == 1 else a)
            bands = [bs[0] + j * bs[1] for j in range(bs[2])]
            assert bands_match(img, bands, g["band_sha"][k]) == [], (fpl, bs)
        finally:
            p.close()
    p = rt.ComputeShaderPipeline(0)
    try:
        with pytest.raises(rt.RtError):
            p.update_frames_bands(p.new_image(w, 8), p.new_image(w, 8), w, h, (135, 1, 1),
                                  cam, sc, g["seeds"][:1])        # past the image
        with pytest.raises(rt.RtError):
            p.update_frames_bands(p.new_image(w, 16), p.new_image(w, 16), w, h, (0, 0, 2),
                                  cam, sc, g["seeds"][:1])        # step 0
    finally:
        p.close()


def test_launch_timing_keeps_bits(rt):
    """rt_set_launch_timing: the fused launches carry the timing events in their own dispatch
    packets (hipExtModuleLaunchKernel); the image is the same bits (bench fixture's 25-frame
    digest), the time is positive and covers the call's launches, and a call of one-frame
    launches reports no timed launch."""
    g = load_golden("bench_k3.npz")
    w, h = int(g["width"]), int(g["height"])
    cam, sc = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"])
    k = list(g["frame_counts"]).index(25)
    p = rt.ComputeShaderPipeline(0)
    try:
        p.set_frame_images("every")
        p.set_launch_timing(True)
        a, b = p.new_image(w, h), p.new_image(w, h)
        if p.update_frames(a, b, w, h, cam, sc, g["seeds"][:5]) == 1:
            a, b = b, a
        newest = p.update_frames(a, b, w, h, cam.with_fields(camera_has_moved=0.0), sc,
                                 g["seeds"][5:25])
        t, n = p.last_call_kernel_time()
        assert n == p.last_launch_info()["launches"] == 1 and 1e-6 < t < 0.1
        assert canon_sha(host(b if newest == 1 else a)) == str(g["sha256"][k])
        p.set_frames_per_launch(1)
        p.update_frames(a, b, w, h, cam, sc, g["seeds"][:2])
        with pytest.raises(rt.RtError):
            p.last_call_kernel_time()
    finally:
        p.close()
