#!/bin/bash
# Round-3 closing check after RT_SINGLE_HASH 1: the whole -m gpu suite, smoke, the driver's
# command (twice) and its rocprofv3 kernel trace, the K2 default line.
# Usage: bash tools/gpu_r03zo.sh TAG
set -o pipefail
TAG=${1:-r03zo}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; tail $O/smoke.log; exit 1; }
echo smoke ok
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver.err \
    || { echo bench failed; tail $O/bench_driver.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['submit'], r['frac'], r.get('binding_frac'), d['image_ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > $O/prof_driver.log 2>&1 || { echo "rocprof failed"; tail $O/prof_driver.log; exit 1; }
echo rocprof done
timeout -k 10 300 python bench.py --config K2 > $O/bench_K2.json 2> $O/bench_K2.err \
  || { echo "bench K2 failed"; tail $O/bench_K2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_K2.json')); r=d['roofline']; print('K2', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['frac'], d['image_ok'])"
for c in K3 K2; do
  RT_FPL=1 RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py $c 50 > $O/rank_$c.jsonl || exit 1
  echo "rank $c"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_$c.jsonl
done
