#!/bin/bash
# Round-3 session zi: one tile per wave up to 20 000 tiles per launch (2-rank shares) against
# the default 9 000: per-rank K3 / K2 predictions, three interleaved rounds.
# Usage: bash tools/gpu_r03zi.sh TAG
set -o pipefail
TAG=${1:-r03zi}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
for r in 1 2 3; do
  for lib in default $V/librt_hip_one20k.so; do
    for c in K3 K2; do
      n=$(basename $lib .so)
      if [ $lib = default ]; then E=""; else E="RT_HIP_LIB=$lib"; fi
      env $E RT_FPL=1 RT_REPS=7 timeout -k 10 300 python tools/rank_sim.py $c 50 > $O/rank_${c}_${n}_$r.jsonl || exit 1
      echo "rank $c $n round $r"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_${c}_${n}_$r.jsonl
    done
  done
done
