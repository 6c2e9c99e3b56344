#!/bin/bash
# Round-3 final lines on the last build: the driver's command (twice), the default bench
# lines of K3 / K2 / K4 / K5, the rocprofv3 kernel traces of the K3 line (two parts and one),
# per-rank predictions of K3 / K2 / K5.  Usage: bash tools/gpu_r03v.sh TAG
set -o pipefail
TAG=${1:-r03v}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver.err \
    || { echo bench failed; tail $O/bench_driver.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['frac'], r.get('binding_frac'), d['image_ok'])"
done
for c in K3 K2 K4 K5; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err \
    || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['frac'], r.get('binding_frac'), d['image_ok'], d['cpu_baseline']['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k3 -o k3 -- python3 bench.py --side 0 --cpu-seconds 0 \
  > $O/prof_k3.log 2>&1 || { echo "rocprof failed"; tail $O/prof_k3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k3q1 -o k3q1 -- python3 bench.py --side 0 --cpu-seconds 0 --queues 1 \
  > $O/prof_k3q1.log 2>&1 || { echo "rocprof q1 failed"; tail $O/prof_k3q1.log; exit 1; }
echo rocprof done
for c in K3 K2; do
  RT_FPL=1 RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py $c 50 > $O/rank_$c.jsonl || exit 1
  echo "rank $c"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_$c.jsonl
done
RT_REPS=3 timeout -k 10 400 python tools/rank_sim.py K5 64 > $O/rank_K5.jsonl || exit 1
echo "rank K5"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_K5.jsonl
