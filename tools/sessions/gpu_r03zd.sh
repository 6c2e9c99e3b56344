#!/bin/bash
# Round-3 session zd: per-rank K3 shares, HIP launches (AUTO parts) against AQL packets at 2
# queues, two interleaved rounds of 7 timed blocks each.  Usage: bash tools/gpu_r03zd.sh TAG
set -o pipefail
TAG=${1:-r03zd}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for spec in hip:0 aql:2 hip:1; do
    m=${spec%:*}; q=${spec#*:}
    RT_FPL=1 RT_SUBMIT=$m RT_QUEUES=$q RT_REPS=7 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_${m}_q${q}_$r.jsonl || exit 1
    echo "rank K3 $m q$q round $r"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_${m}_q${q}_$r.jsonl
  done
done
