#!/bin/bash
# Round-3 session w: the driver's 20-step command with and without the untimed clock warm-up
# (bench.py --warm-ms), interleaved.  Usage: bash tools/gpu_r03w.sh TAG
set -o pipefail
TAG=${1:-r03w}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for wm in 0 50 200; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      --warm-ms $wm > $O/driver_w${wm}_$r.json 2>> $O/err.log || { tail $O/err.log; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver warm', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['warm_up']['ms'], d['image_ok'])" $O/driver_w${wm}_$r.json $wm $r
  done
done
