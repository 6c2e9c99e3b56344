#!/bin/bash
# Round 6: the whole GPU suite and smoke on the tree with launch timing, the exact
# bisection partition and the checked band-set gather; the driver's command with the
# weighted roofline.
set -o pipefail
TAG=${1:-r06k}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "bench failed"; tail $O/bench_driver.err; exit 1; }
python tools/summarize_bench.py $O/bench_driver.json > $O/summary.txt; head -4 $O/summary.txt
python -c "import json; r=json.load(open('$O/bench_driver.json'))['roofline']; print('weighted', r.get('weighted', {}).get('frac'), 'ref', r['hbm'].get('reference_semantics', {}).get('frac'), 'traffic GB/s', r['hbm'].get('traffic_GBs'))"
