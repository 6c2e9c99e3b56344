#!/bin/bash
# Round-3 session x: with the clock warm-up, re-check the concurrent-parts choice (K3 / K2 at
# 1-4 parts, default length, interleaved) and the per-rank predictions (K3 at 1 and 2 parts).
# Usage: bash tools/gpu_r03x.sh TAG
set -o pipefail
TAG=${1:-r03x}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 2 default:RT_QUEUES=1 default:RT_QUEUES=2 default:RT_QUEUES=3 default:RT_QUEUES=4 || exit 1
for q in 0 1 2; do
  RT_FPL=1 RT_QUEUES=$q RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_q$q.jsonl || exit 1
  echo "rank K3 q$q"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_q$q.jsonl
done
