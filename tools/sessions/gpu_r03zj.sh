#!/bin/bash
# Round-3 session zj: AUTO submission range up to 20 000 tiles (2-rank shares as AQL packets)
# against the default 12 000, per-rank K3 / K2, three interleaved rounds.
# Usage: bash tools/gpu_r03zj.sh TAG
set -o pipefail
TAG=${1:-r03zj}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
for r in 1 2 3; do
  for lib in default $V/librt_hip_aql20k.so; do
    for c in K3 K2; do
      n=$(basename $lib .so)
      if [ $lib = default ]; then E=""; else E="RT_HIP_LIB=$lib"; fi
      env $E RT_FPL=1 RT_REPS=7 timeout -k 10 300 python tools/rank_sim.py $c 50 > $O/rank_${c}_${n}_$r.jsonl || exit 1
      python -c "import json,sys; print(sys.argv[2], sys.argv[3], sys.argv[4], ' '.join('%d:%s:%s' % (d['world'], d['us_per_step'], d['submit']) for d in map(json.loads, open(sys.argv[1]))))" $O/rank_${c}_${n}_$r.jsonl $c $n $r
    done
  done
done
