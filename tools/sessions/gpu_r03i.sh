#!/bin/bash
# Round-3 session i: -m gpu suite with update graphs, then update graphs against direct
# launches: per-rank prediction (K3, parts 1 / 2 / 4) and the driver's bench command.
# Usage: bash tools/gpu_r03i.sh TAG
set -o pipefail
TAG=${1:-r03i}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for cfg in "off 1" "auto 1" "auto 2" "auto 4"; do
  set -- $cfg
  RT_GRAPHS=$1 RT_QUEUES=$2 RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_g$1_q$2.jsonl 2>&1 || exit 1
  echo k3 graphs=$1 q=$2; grep '^{' $O/rank_k3_g$1_q$2.jsonl
done
for r in 1 2; do
  for cfg in "off 2" "auto 1" "auto 2" "auto 4"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --graphs $1 --queues $2 --side 0 --cpu-seconds 0 \
      > $O/bench_driver_g$1_q$2_$r.json 2> $O/bench_driver.err || { echo bench failed; tail $O/bench_driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_driver_g$1_q$2_$r.json')); r=d['roofline']; print('driver g=$1 q=$2', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['graph_frames'], d['image_ok'])"
  done
done
