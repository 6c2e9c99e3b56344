#!/bin/bash
# Round-3 session zg: 2 against 3 concurrent parts (HIP launches) at warm start: bench.py
# default length for K3 / K2 (4 rounds) and the driver's 20-step K3 command (4 rounds).
# Usage: bash tools/gpu_r03zg.sh TAG
set -o pipefail
TAG=${1:-r03zg}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 4 default:RT_QUEUES=2 default:RT_QUEUES=3 || exit 1
for r in 1 2 3 4; do
  for q in 2 3; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      --queues $q > $O/driver_q${q}_$r.json 2>> $O/err.log || { tail $O/err.log; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('driver q', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_avg_us'], d['image_ok'])" $O/driver_q${q}_$r.json $q $r
  done
done
