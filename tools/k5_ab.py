"""Interleaved A/B of library builds on bench.py --config K5's step (diagnostic):
    python tools/k5_ab.py ROUNDS LIB [LIB ...]        (LIB: a librt_hip.so path, or "tree")
Each round runs every build in its own process (RT_HIP_LIB), the order rotating from round
to round.  A process renders
the K5 fixture's 64-spp step (3840x2160, 500 spheres, depth 8: one 64-frame bounce launch from
a reset) twice to warm up, then R = 5 more, each timed wall-clock around the call and a
synchronize, and checks the last image's whole-image digest against tests/golden/k5.npz;
then the same for rank 0's 8-rank share (round-robin bands, the default path schedule: its
second step runs the measured split order), checked band by band.  Prints one JSON line per
(round, build) and the medians."""
import json
import os
import statistics as st
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def one():
    sys.path[:0] = [str(ROOT / "gpu-ray-tracing_amd"), str(ROOT), str(ROOT / "tests")]
    import numpy as np
    import torch
    import gpu_ray_tracing as rt
    from conftest import bands_match, canon_sha
    g = dict(np.load(ROOT / "tests" / "golden" / "k5.npz"))
    w, h = int(g["width"]), int(g["height"])
    cam, sc, seeds = rt.SceneCamera(g["camera"]), rt.SphereCollection(g["spheres"]), g["seeds"]
    out = {}
    for world in (1, 8):
        pipe = rt.ComputeShaderPipeline(0)
        rows = rt.stripe_local_rows(h, 0, world)
        a, b = pipe.new_image(w, rows), pipe.new_image(w, rows)
        walls = []
        newest = 0
        for k in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            newest = pipe.update_frames(a, b, w, h, cam, sc, seeds, 0, world)
            torch.cuda.synchronize()
            if k >= 2:
                walls.append((time.perf_counter() - t0) * 1e6)
        img = (b if newest == 1 else a).cpu().numpy()
        if world == 1:
            ok = canon_sha(img) == str(g["sha256"])
        else:
            ok = bands_match(img, range(0, h // 8, world), g["band_sha"]) == []
        out[str(world)] = {"wall_us": round(st.median(walls), 1),
                           "kernel": pipe.last_launch_info()["kernel_name"], "ok": ok}
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
            if l != "tree":
                env["RT_HIP_LIB"] = str(Path(l).resolve())
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
        summary[Path(l).name] = {w: round(st.median(d[w]["wall_us"] for d in ds), 1)
                                 for w in ("1", "8")}
        summary[Path(l).name]["all_ok"] = all(d[w]["ok"] for d in ds for w in ("1", "8"))
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    if "--one" in sys.argv:
        one()
    else:
        main()
