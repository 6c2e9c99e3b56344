#!/bin/bash
# Round 6: K5 8-rank share schedules again after the far-ray and grid-pad changes
# per wave, pairs, split at S = 2 / 4 / 8 chunks and alpha 0.125 / 0.25 / 0.5.
set -o pipefail
TAG=${1:-r06aa}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python tools/k5_share_sweep.py 8 > $O/sweep_n8.jsonl 2> $O/sweep_n8.err \
  || { echo "sweep failed"; tail $O/sweep_n8.err; tail -3 $O/sweep_n8.jsonl; exit 1; }
tail -1 $O/sweep_n8.jsonl
