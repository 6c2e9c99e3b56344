#!/bin/bash
# Round-2 artifacts on the product build: -m gpu tests, smoke(), the driver's bench command,
# one bench line per config, a rocprofv3 kernel trace of the default bench, per-rank
# predictions (K3 per dispatch, K5).  Usage: bash tools/gpu_final2.sh TAG
set -o pipefail
TAG=${1:-final2}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench.err \
  || { echo bench failed; tail $O/bench.err; exit 1; }
for c in K3 K2 K4 K5; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 8 > $O/bench_$c.json 2>> $O/bench.err \
    || { echo "bench $c failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['image_ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench \
  -- python3 bench.py --side 0 --cpu-seconds 0 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
grep '^{' $O/prof.log > $O/bench_profiled.json
head -3 $O/prof/bench_kernel_stats.csv | cut -c1-200
RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_dispatch.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k3_dispatch.jsonl
timeout -k 10 300 python tools/rank_sim.py K5 64 > $O/rank_k5.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k5.jsonl
