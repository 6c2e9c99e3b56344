#!/bin/bash
# Round-3 final lines: -m gpu suite, the driver's command (twice), the default bench lines of
# K3 / K2 / K4 / K5 and the rocprofv3 kernel trace of the K3 line.  Usage: bash tools/gpu_r03n.sh TAG
set -o pipefail
TAG=${1:-r03n}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver.err \
    || { echo bench failed; tail $O/bench_driver.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['frac'], d['image_ok'])"
done
for c in K3 K2 K4 K5; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err \
    || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['frac'], d['image_ok'], d['cpu_baseline']['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k3 -o k3 -- python3 bench.py --side 0 --cpu-seconds 0 \
  > $O/prof_k3.log 2>&1 || { echo "rocprof failed"; tail $O/prof_k3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k3q1 -o k3q1 -- python3 bench.py --side 0 --cpu-seconds 0 --queues 1 \
  > $O/prof_k3q1.log 2>&1 || { echo "rocprof q1 failed"; tail $O/prof_k3q1.log; exit 1; }
echo rocprof done
