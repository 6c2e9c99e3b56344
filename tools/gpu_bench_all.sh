#!/bin/bash
# -m gpu tests, smoke(), then one bench line per config (K3 default, K2, K4, K5) and the
# driver's command.  Usage: bash tools/gpu_bench_all.sh TAG
set -o pipefail
TAG=${1:-benchall}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench.err \
  || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench_driver.json
for c in K3 K2 K4 K5; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 6 > $O/bench_$c.json 2>> $O/bench.err \
    || { echo "bench $c failed"; tail $O/bench.err; exit 1; }
  cat $O/bench_$c.json
done
