#!/bin/bash
# One GPU session: tests, bench, rocprof kernel trace.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench failed; tail gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o bench -- python3 bench.py --cpu-frames 0 > gpurun_out/$TAG/prof.log 2>&1 || { echo prof failed; tail gpurun_out/$TAG/prof.log; exit 1; }
head -3 gpurun_out/$TAG/prof/bench_kernel_stats.csv
