#!/bin/bash
# Round 4, last check of the committed tree: the -m gpu suite, smoke(), the driver's bench
# command.
# Usage: bash tools/sessions/gpu_r04zz.sh TAG
set -o pipefail
TAG=${1:-r04zz}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo bench failed; tail $O/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], 'side_error' in d, d['k4']['image_ok'], d['k5']['image_ok'], d['k2']['image_ok'])"
