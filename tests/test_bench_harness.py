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
    """At N = 1 there is no barrier: the time is the steps plus the closing wait, and the
    wait hook (bench.py --host-wait spin) runs instead of the plain synchronize."""
    import time
    calls = []
    ts = bench.timed_steps(lambda: time.sleep(0.01), lambda: calls.append("sync"), 1,
                           barrier=lambda: calls.append("barrier"),
                           wait=lambda: calls.append("wait"))
    assert calls == ["sync", "wait"]
    assert 0.01 <= ts["dt"] < 0.2 and ts["per_rank"] == [ts["dt"]] and ts["barrier_s"] == 0.0
    assert 0.01 <= ts["issue"] <= ts["dt"]


def test_frame_launch_policy(bench):
    """--frame-launch auto: the whole 1920x1080 image (32 400 tiles) one launch per frame,
    every rank share of N >= 2 (at most 17 280 tiles) frame chains."""
    from gpu_ray_tracing import stripe_local_rows
    assert bench.frame_launch_mode("auto", 1920, 1080) == "dispatch"
    for n in (2, 4, 8):
        assert bench.frame_launch_mode("auto", 1920, stripe_local_rows(1080, 0, n)) == "chain"
    assert bench.frame_launch_mode("dispatch", 1920, 136) == "dispatch"
