"""Interleaved A/B of library builds on the K3 frame-chain structure (the main line's):
    python tools/chain_ab.py ROUNDS LIB [LIB ...]        (LIB: a librt_hip.so path, or "tree")
Each round runs every build in its own process (RT_HIP_LIB), the order rotating from round
to round; a process warms 50 ms,
then times the driver's region R = 7 times — a reset + 5 frames, then 20 frames in one
rt_update_frames call, wall-clock around the call and a synchronize — for the whole image
and rank 0's 8-rank share, reads the kernel time of three more calls from the timing events
their launches carry, and checks the whole image's digest after the 25 frames against
tests/golden/bench_k3.npz.  Prints one JSON line per (round, build) and the medians.
kernel_us comes from back-to-back calls (no synchronize between the reset and the 20 frames)
and reads above the wall time: compare it between builds only; wall_us is the measure."""
import hashlib
import json
import os
import statistics as st
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def one():
    sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT)]
    import numpy as np
    import torch
    import gpu_ray_tracing as rt
    from gpu_ray_tracing.distributed import StripeRenderer
    g = dict(np.load(ROOT / "tests" / "golden" / "bench_k3.npz"))
    w, h = int(g["width"]), int(g["height"])
    cam, sc, seeds = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]), g["seeds"]
    still = cam.with_fields(camera_has_moved=0.0)
    pipe = rt.ComputeShaderPipeline(0)
    pipe.set_frame_images("every")
    out = {}
    for world in (1, 8):
        r = StripeRenderer(pipe, w, h, 0, world)
        scratch = StripeRenderer(pipe, w, h, 0, world)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.05:
            scratch.frames(cam, sc, seeds[:20])
            torch.cuda.synchronize()
        walls, ks = [], []
        for _ in range(7):
            r.frames(cam, sc, seeds[:5])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.frames(still, sc, seeds[5:25])
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) / 20 * 1e6)
        img = r.local.cpu().numpy()
        ok = None
        if world == 1:
            k = list(g["frame_counts"]).index(25)
            ok = hashlib.sha256(np.ascontiguousarray(img[:h]).tobytes()).hexdigest() == \
                str(g["sha256"][k])
        pipe.set_launch_timing(True)
        for _ in range(3):
            r.frames(cam, sc, seeds[:5])
            r.frames(still, sc, seeds[5:25])
            ks.append(pipe.last_call_kernel_time()[0] / 20 * 1e6)
        pipe.set_launch_timing(False)
        out[str(world)] = {"wall_us": round(st.median(walls), 3),
                           "kernel_us": round(st.median(ks), 3),
                           "kernel": pipe.last_launch_info()["kernel_name"], "ok": ok}
        del r, scratch
    pipe.close()
    print(json.dumps(out))


def main():
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    res = {l: [] for l in libs}
    for rd in range(rounds):
        # the order rotates every round (a process's place in the round measurably moves its
        # time by up to ~2 %: profiles/r06/r06ac/chain_ab_same_build.jsonl)
        k = rd % len(libs)
        for l in libs[k:] + libs[:k]:
            env = dict(os.environ)
            # every build through RT_HIP_LIB, the tree's too: an experiment build runs without
            # the CPython binding of rt_update_frames (ctypes instead), ~0.1 us more per frame
            # of a 20-frame call — a bias of ~3 % on the 8-rank share against the tree with
            # the binding (profiles/r06/r06ac/, r06ad/)
            env["RT_HIP_LIB"] = str(Path(l).resolve() if l != "tree" else
                                    ROOT / "gpu-ray-tracing_amd" / "build" / "librt_hip.so")
            p = subprocess.run([sys.executable, __file__, "--one"], env=env, capture_output=True,
                               text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode or not line:
                print(l, "FAILED", p.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            res[l].append(d)
            print(json.dumps({"round": rd, "lib": Path(l).name, **d}), flush=True)
    summary = {}
    for l, ds in res.items():
        summary[Path(l).name] = {
            w: {k: round(st.median(d[w][k] for d in ds), 3) for k in ("wall_us", "kernel_us")}
            for w in ("1", "8")}
        summary[Path(l).name]["all_ok"] = all(d["1"]["ok"] for d in ds)
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    if "--one" in sys.argv:
        one()
    else:
        main()
