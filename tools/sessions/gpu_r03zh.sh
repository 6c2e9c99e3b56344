#!/bin/bash
# Round-3 session zh: per-rank K3 shares with the one-frame kernel's tiles per wave forced
# (RT_SINGLE=pair: two, one: one) against AUTO, AUTO submission, two interleaved rounds.
# Usage: bash tools/gpu_r03zh.sh TAG
set -o pipefail
TAG=${1:-r03zh}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for s in auto pair one; do
    RT_FPL=1 RT_SINGLE=$s RT_REPS=7 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_${s}_$r.jsonl || exit 1
    echo "rank K3 single=$s round $r"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_${s}_$r.jsonl
  done
done
