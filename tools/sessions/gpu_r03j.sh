#!/bin/bash
# Round-3 session j: -m gpu suite of the reverted one-frame path with the new bounce register
# plan, host launch cost by API, the driver's bench command and K5.
# Usage: bash tools/gpu_r03j.sh TAG
set -o pipefail
TAG=${1:-r03j}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/launch_rate > $O/launch_rate.jsonl 2>&1 || { echo launch_rate failed; cat $O/launch_rate.jsonl; exit 1; }
grep -v graph_kernels $O/launch_rate.jsonl
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver.err \
    || { echo bench failed; tail $O/bench_driver.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], d['image_ok'])"
done
timeout -k 10 400 python bench.py --config K5 > $O/bench_K5.json 2> $O/bench_K5.err \
  || { echo "bench K5 failed"; tail $O/bench_K5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_K5.json')); r=d['roofline']; print('K5', d['value'], d['ms_per_step'], r['kernel_avg_us'], d['image_ok'])"
