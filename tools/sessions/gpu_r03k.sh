#!/bin/bash
# Round-3 session k: -m gpu suite with the packed one-frame launches, per-call host cost,
# per-rank prediction at 1 / 2 parts, the driver's command (two rounds) and the default
# K3 / K2 lines at 2 and 4 parts.  Usage: bash tools/gpu_r03k.sh TAG
set -o pipefail
TAG=${1:-r03k}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/call_overhead.py > $O/call_overhead.jsonl 2>&1 || { echo call_overhead failed; tail $O/call_overhead.jsonl; exit 1; }
grep '^{' $O/call_overhead.jsonl
for q in 1 2; do
  RT_QUEUES=$q RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_q$q.jsonl 2>&1 || exit 1
  echo k3 q$q; grep '^{' $O/rank_k3_q$q.jsonl
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver.err \
    || { echo bench failed; tail $O/bench_driver.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], d['image_ok'])"
done
bash tools/gpu_ab_bench.sh $TAG/abq "K3 K2" 2 default:RT_QUEUES=2 default:RT_QUEUES=4 || exit 1
