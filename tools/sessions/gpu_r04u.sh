#!/bin/bash
# Round 4, session u: RT_GROUP_FLAGS (frame groups hand colours over through an LDS ring with
# counters instead of a barrier per group; every wait bounded): the -m gpu suite on it, then
# K3 frame-chain rank shares with it and with the in-tree build (tools/rank_sim.py, 5 blocks).
# Usage: bash tools/sessions/gpu_r04u.sh TAG
set -o pipefail
TAG=${1:-r04u}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_gflags.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/pytest_gpu_gflags.log 2>&1 \
  || { tail -20 $O/pytest_gpu_gflags.log; exit 1; }
tail -2 $O/pytest_gpu_gflags.log
for r in 1 2; do
  for lib in default gflags; do
    E=""; [ $lib != default ] && E="RT_HIP_LIB=$V/librt_hip_$lib.so"
    env $E RT_FPL=0 RT_IMAGES=every RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 20 \
      > $O/rank_K3_${lib}_$r.jsonl 2>> $O/rank.err || { echo "rank_sim $lib failed"; tail -5 $O/rank.err; exit 1; }
    python -c "import json; [print('$lib r$r', d['world'], d['us_per_step'], d['predicted_efficiency'], d.get('kernel')) for d in map(json.loads, open('$O/rank_K3_${lib}_$r.jsonl'))]"
  done
done
