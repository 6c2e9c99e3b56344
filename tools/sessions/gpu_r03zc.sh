#!/bin/bash
# Round-3 session zc: the driver's 20-step K3 command cold (--warm-ms 0) and warm (50 ms) with
# HIP launches and with AQL packets (VRAM argument ring): is the cold-start penalty the host's
# launch issue rate?  Usage: bash tools/gpu_r03zc.sh TAG
set -o pipefail
TAG=${1:-r03zc}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for wm in 0 50; do
    for m in hip aql; do
      timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
        --warm-ms $wm --submit $m > $O/driver_${m}_w${wm}_$r.json 2>> $O/err.log || { tail $O/err.log; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('driver', sys.argv[2], 'warm', sys.argv[3], sys.argv[4], d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['submit'], d['image_ok'])" $O/driver_${m}_w${wm}_$r.json $m $wm $r
    done
  done
done
