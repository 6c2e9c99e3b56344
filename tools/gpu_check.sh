#!/bin/bash
# One GPU check of the product build: -m gpu tests, smoke(), bench (K3 default + K2), and a
# rocprofv3 kernel-trace summary of the bench.  Usage: bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-check}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err \
  || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config K2 --cpu-seconds 0 > $O/bench_k2.json 2>> $O/bench.err \
  || { echo bench K2 failed; tail $O/bench.err; exit 1; }
cat $O/bench_k2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench \
  -- python3 bench.py --cpu-seconds 0 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
head -5 $O/prof/bench_kernel_stats.csv
