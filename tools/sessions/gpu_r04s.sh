#!/bin/bash
# Round 4, session s: the warm-up length before the driver's 20 timed steps (--warm-ms 50, the
# default, against 300), four interleaved rounds of the driver's command (side lines off).
# Usage: bash tools/sessions/gpu_r04s.sh TAG
set -o pipefail
TAG=${1:-r04s}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2 3 4; do
  for w in 50 300; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 --warm-ms $w \
      > $O/driver_w${w}_$r.json 2>> $O/driver.err || { echo bench failed; tail -5 $O/driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/driver_w${w}_$r.json')); print('driver warm $w r$r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['image_ok'])"
  done
done
