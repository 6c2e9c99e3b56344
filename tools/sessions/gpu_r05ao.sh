#!/bin/bash
# Round 5: the final tree's default-length lines (200 timed updates): bench.py (K3) and
# bench.py --config K2, main lines only (--side 0), twice each.
# Usage: bash tools/sessions/gpu_r05ao.sh TAG
set -o pipefail
TAG=${1:-r05ao}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for c in K3 K2; do
    timeout -k 10 300 python bench.py --config $c --side 0 --cpu-seconds 0 > $O/bench_${c}_$r.json 2> $O/bench_${c}_$r.err \
      || { echo "bench failed"; tail $O/bench_${c}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${c}_$r.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
  done
done
