#!/bin/bash
# AUTO's new frame-group thresholds (four waves per tile pair up to 12 288 tiles, two per pair
# above) against the previous ones, through the driver's own command: bench.py's rank_shares
# (K3 chains at 20 and 200 steps, every rank's share, max over ranks), both builds through
# RT_HIP_LIB, alternating, three times each; then the GPU tests of the share paths.
set -o pipefail
TAG=${1:-r06ao}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
L=(old base)
for rd in 0 1 2; do
  for i in 0 1; do
    l=${L[$(( (i + rd) % 2 ))]}
    RT_HIP_LIB=$V/librt_hip_$l.so timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 \
      > $O/bench_${l}_$rd.json 2> $O/bench_${l}_$rd.err || { echo "bench $l failed"; tail $O/bench_${l}_$rd.err; exit 1; }
  done
  echo "round $rd done"
done
python - <<PY
import json, statistics as st
for l in ("old", "base"):
    ds=[json.load(open(f"$O/bench_{l}_{r}.json"))["rank_shares"] for r in range(3)]
    for c in ("K3_chain_20_steps", "K3_chain_200_steps"):
        print(l, c, {n: (round(st.median(d[c][n]["us_per_step"] for d in ds), 3), ds[0][c][n]["kernel"],
                         round(st.median(d[c][n]["efficiency"] for d in ds), 3)) for n in ("1","2","4","8")})
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pair or share or stripe or band or rank" \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
