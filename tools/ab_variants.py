"""Interleaved A/B of library builds: python tools/ab_variants.py cfg rounds lib1 lib2 ..."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
cfg, rounds, libs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
res = {l: [] for l in libs}
fres = {l: [] for l in libs}
def spec(l):
    """lib[:K=V,K=V] -> (lib path, extra env)"""
    path, _, rest = l.partition(":")
    env = dict(kv.split("=", 1) for kv in rest.split(",") if kv)
    return path, env

for r in range(rounds):
    for l in libs:
        path, extra = spec(l)
        out = subprocess.run([sys.executable, str(ROOT / "tools" / "time_kernel.py"), cfg],
                             env=dict(os.environ, RT_HIP_LIB=path, **extra), capture_output=True,
                             text=True, timeout=300)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")]
        if not line:
            print(l, "FAILED", out.stderr[-2000:], flush=True); sys.exit(1)
        d = json.loads(line[-1]); res[l].append(d["median_us"]); fres[l].append(d.get("fused_us", 0.0))
        print(r, Path(l).name, d, flush=True)
for l in libs:
    v = sorted(res[l]); fv = sorted(fres[l])
    print(f"{Path(l).name:40s} median {v[len(v)//2]:8.2f} us  min {v[0]:8.2f}  "
          f"fused {fv[len(fv)//2]:7.2f} us/frame  min {fv[0]:7.2f}")
