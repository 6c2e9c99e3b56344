#!/bin/bash
# Round 6: the 8-rank / 4-rank K3 chain shares under each frame-group mode
# (tools/share_region.py: 20-frame calls, wall and events), two passes interleaved.
set -o pipefail
TAG=${1:-r06c}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for pass in 1 2; do
for n in 8 4; do
for m in auto quad2 on2 quad on; do
  timeout -k 10 100 python tools/share_region.py $n 0 15 20 $m > $O/share_n${n}_${m}_$pass.json 2> $O/err.txt \
    || { echo "failed"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.load(open('$O/share_n${n}_${m}_$pass.json')); print($n, '$m', d['kernel'], d['wall_us_per_step_q1_med_q3'], d['events_us_per_step_q1_med_q3'])"
done; done; done
