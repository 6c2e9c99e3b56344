#!/bin/bash
# Round-3 session h: host cost of graph replay vs direct launches, and the driver's bench
# command at 1 / 2 / 4 concurrent update parts (two rounds).  Usage: bash tools/gpu_r03h.sh TAG
set -o pipefail
TAG=${1:-r03h}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/launch_rate > $O/launch_rate.jsonl 2>&1 || { echo launch_rate failed; cat $O/launch_rate.jsonl; exit 1; }
cat $O/launch_rate.jsonl
for r in 1 2; do
  for q in 1 2 4; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --queues $q --side 0 --cpu-seconds 0 \
      > $O/bench_driver_q${q}_$r.json 2> $O/bench_driver.err || { echo bench failed; tail $O/bench_driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_driver_q${q}_$r.json')); r=d['roofline']; print('driver q$q', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], d['image_ok'])"
  done
done
