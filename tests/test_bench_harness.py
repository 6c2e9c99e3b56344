"""CPU tests of bench.py's harness logic (no GPU): the max-over-ranks reduction of the rank
shares and the StreamGate-free timed region on one rank."""
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def test_over_ranks_takes_the_slowest_rank(bench):
    times = {0: 3.0, 1: 3.4, 2: 2.9}
    oks = {0: True, 1: True, 2: True}
    out = bench.over_ranks(lambda r: {"us_per_step": times[r], "kernel": "k",
                                      "image_ok": oks[r]}, 3)
    assert out["us_per_step"] == 3.4 and out["slowest_rank"] == 1
    assert out["rank_us"] == [3.0, 3.4, 2.9] and out["rank0_us"] == 3.0
    assert out["max_over_ranks"] is True and out["image_ok"] is True
    oks[2] = False
    assert bench.over_ranks(lambda r: {"us_per_step": times[r], "image_ok": oks[r]},
                            3)["image_ok"] is False
    oks[2] = None                      # (no fixture for that frame count)
    assert bench.over_ranks(lambda r: {"us_per_step": times[r], "image_ok": oks[r]},
                            3)["image_ok"] is None


def test_timed_steps_one_rank(bench):
    """At N = 1 there is no barrier: the time is the steps plus the closing wait (the wait
    hook runs instead of the plain synchronize), on CLOCK_MONOTONIC."""
    import time
    calls = []
    ts = bench.timed_steps(lambda: time.sleep(0.01), lambda: calls.append("sync"), 1,
                           barrier=lambda: calls.append("barrier"),
                           wait=lambda: calls.append("wait"))
    assert calls == ["sync", "wait"]
    assert 0.01 <= ts["dt"] < 0.2 and ts["per_rank"] == [ts["dt"]] and ts["barrier_s"] == 0.0
    assert ts["start_skew_s"] == 0.0 and ts["max_rank_s"] == ts["dt"]
    assert 0.01 <= ts["issue"] <= ts["dt"]


def test_one_launch_structure_at_every_n(bench):
    """Round 6 (verdict item 1): K2/K3 run the same launch structure at every N — frame
    chains by default, one launch per frame on request — with no size-dependent switch."""
    assert bench.parse([]).frame_launch == "chain"
    assert bench.parse(["--frame-launch", "dispatch"]).frame_launch == "dispatch"
    assert not hasattr(bench, "frame_launch_mode")


def test_stripe_bands_round_robin(bench):
    assert bench.stripe_bands(1080, 0, 8)[:3] == [0, 8, 16]
    assert bench.stripe_bands(1080, 7, 8)[-1] == 127
    bands = sorted(b for r in range(8) for b in bench.stripe_bands(1080, r, 8))
    assert bands == list(range(135))


def test_canon_sha_matches_fixture_script(bench):
    """bench.py's digest and the fixture generator's (tests/golden/make_band_digests.py)
    agree, NaN payloads canonical: any NaN hashes as 0x7FC00000."""
    import hashlib
    import numpy as np
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import make_band_digests as M
    a = np.arange(64, dtype=np.float32).reshape(2, 8, 4)
    a.view(np.uint32)[0, 3, 1] = 0xFFC00001          # a negative NaN with a payload
    b = a.copy()
    b.view(np.uint32)[0, 3, 1] = 0x7FC00000
    assert bench.canon_sha(a) == bench.canon_sha(b) == hashlib.sha256(b.tobytes()).hexdigest()
    assert bytes(M.band_digests(np.concatenate([a[0:1]] * 8).reshape(8, 8, 4))[0]).hex() == \
        bench.canon_sha(np.concatenate([b[0:1]] * 8).reshape(8, 8, 4))


def test_fixtures_carry_band_digests(bench):
    """Every full-size fixture has a whole-image digest and one digest per 8-row band (K5:
    the exact segment count too), so bench.py checks every rank's share band by band."""
    for cfg, frames in (("K2", 25), ("K3", 25), ("K3", 220), ("K4", 64), ("K5", 64)):
        g = bench._fixture(cfg)
        sha, bands, pixels, segs = bench._fixture_at(g, frames)
        h = int(g["height"])
        assert sha is not None and len(sha) == 64, cfg
        assert bands is not None and bands.shape == (h // 8, 32), cfg
        assert segs is not None and segs > 0, cfg
    assert bench._fixture("K5")["px"].size >= 16384


def test_roofline_object(bench):
    """The roofline of a timed launch: HBM bytes against 8 TB/s, and with a PMC summary of
    the kernel the VALU issue fraction as the bound (SQ_INSTS_VALU x 2 cycles over 1024
    SIMDs x 2.4 GHz x the launch time), the PMC bytes as `traffic`; the reference's per-frame
    bytes beside the moved ones when they differ (a fused chain)."""
    r = bench.roofline("k", 100e-6, 400e6, None, None)
    assert r["bound"] == "hbm" and r["frac"] == 0.5 and r["traffic"] is None
    pmc = {"valu_insts_per_launch": 1e8, "hbm_bytes_per_launch": 2e8}
    r = bench.roofline("k", 100e-6, 400e6, pmc, "p.json", ref_bytes=800e6)
    assert r["bound"] == "valu" and r["pmc"] == "p.json" and r["traffic"] == 2e8
    assert abs(r["frac"] - 1e8 * 2 / (1024 * 2.4e9 * 100e-6)) < 1e-4
    assert r["hbm"]["frac"] == 0.5 and r["hbm"]["traffic_GBs"] == 2000.0
    assert r["hbm"]["reference_semantics"]["frac"] == 1.0


def test_committed_pmc_and_weighted_model_match(bench):
    """The committed PMC summaries are found for the kernel instances the bench lines time
    (K3: rt_tpair_kernel<2>, one 20-frame launch; K5: rt_bounce_kernel<0>, 64 frames), and the
    weighted VALU model is found for the K3 summary and priced its instruction count — so the
    driver's line carries roofline.valu from them and roofline.weighted."""
    pmc3, p3 = bench.load_pmc("K3", "rt_tpair_kernel<2>", 20)
    assert pmc3 is not None and p3 == "profiles/pmc_r06_K3.json"
    w, wp = bench.load_weighted("K3", "rt_tpair_kernel<2>", p3)
    assert w is not None and wp == "profiles/valu_weighted_r06_K3.json"
    assert w["valu_insts_per_launch"] == pmc3["median_per_launch"]["SQ_INSTS_VALU"]
    pmc5, p5 = bench.load_pmc("K5", "rt_bounce_kernel<0>", 64)
    assert pmc5 is not None and p5 == "profiles/pmc_r06_K5.json"
