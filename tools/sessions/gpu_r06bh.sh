#!/bin/bash
# Round 6: the driver's K3 command three more times on another box (the final tree), for
# the headline's box-to-box spread.
set -o pipefail
TAG=${1:-r06bh}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo "bench failed"; tail $O/bench_driver_$r.err; exit 1; }
  python tools/summarize_bench.py $O/bench_driver_$r.json > $O/summary_driver_$r.txt; head -1 $O/summary_driver_$r.txt
done
