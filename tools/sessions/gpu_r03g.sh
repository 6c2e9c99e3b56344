#!/bin/bash
# Round-3 session g: -m gpu suite with the automatic concurrent update parts, host launch
# rate, per-rank prediction with host issue time (K3 / K2, parts auto / 1 / 2 / 4), the
# driver's bench command, the default bench lines and a rocprofv3 kernel trace of K3.
# Usage: bash tools/gpu_r03g.sh TAG
set -o pipefail
TAG=${1:-r03g}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/launch_rate > $O/launch_rate.jsonl 2>&1 || { echo launch_rate failed; cat $O/launch_rate.jsonl; exit 1; }
cat $O/launch_rate.jsonl
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo bench failed; tail $O/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['frac'], d['image_ok'])"
for q in 0 1 2 4; do
  RT_QUEUES=$q RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_q$q.jsonl 2>&1 || exit 1
  echo k3 q$q; grep '^{' $O/rank_k3_q$q.jsonl
done
RT_QUEUES=0 RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K2 100 > $O/rank_k2_q0.jsonl 2>&1 || exit 1
echo k2 q0; grep '^{' $O/rank_k2_q0.jsonl
for c in K3 K2; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err \
    || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['frac'], d['image_ok'], d['cpu_baseline']['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k3 -o k3 -- python3 bench.py --side 0 --cpu-seconds 0 \
  > $O/prof_k3.log 2>&1 || { echo "rocprof failed"; tail $O/prof_k3.log; exit 1; }
find $O/prof_k3 -name "*kernel_stats.csv" | head -3
