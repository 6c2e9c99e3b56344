#!/bin/bash
# Round 6: PMC summaries of the timed kernels (K3 frame chain at the driver's 20 frames per
# launch, K5 64-frame bounce launch), the driver's command under rocprofv3 --kernel-trace
# --stats, and the driver's command itself.
set -o pipefail
TAG=${1:-r06f}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
PMC_ROUND=r06 bash tools/pmc_bench.sh $TAG "K3 K5" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 \
  > $O/prof_driver.json 2> $O/prof_driver.err || { echo "rocprof driver failed"; tail $O/prof_driver.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "bench failed"; tail $O/bench_driver.err; exit 1; }
python tools/summarize_bench.py $O/bench_driver.json
