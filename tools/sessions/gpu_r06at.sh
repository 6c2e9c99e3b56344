#!/bin/bash
# Round 6, re-entry check of the restored tree (built in a fresh container): the whole GPU
# suite, smoke and the driver's K3 command once.
set -o pipefail
TAG=${1:-r06at}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_1.json 2> $O/bench_driver_1.err \
  || { echo "bench failed"; tail $O/bench_driver_1.err; exit 1; }
python tools/summarize_bench.py $O/bench_driver_1.json > $O/summary_driver_1.txt; cat $O/summary_driver_1.txt | head -30
