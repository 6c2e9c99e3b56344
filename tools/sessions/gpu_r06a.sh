#!/bin/bash
# Round 6 baseline on a fresh box: the driver's K3 command (with side lines) on the
# round-5 tree, before any round-6 change.
set -o pipefail
TAG=${1:-r06a}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "bench failed"; tail $O/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); r=d['roofline']; print('K3', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
