#!/bin/bash
# Round-3 session ze: AUTO = AQL for mid-sized shares: the whole -m gpu suite, smoke, and the
# per-rank predictions of the AUTO policy.  Usage: bash tools/gpu_r03ze.sh TAG
set -o pipefail
TAG=${1:-r03ze}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
RT_FPL=1 RT_REPS=7 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_auto.jsonl || exit 1
echo "rank K3 auto"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_auto.jsonl
RT_FPL=1 RT_REPS=7 timeout -k 10 300 python tools/rank_sim.py K2 50 > $O/rank_k2_auto.jsonl || exit 1
echo "rank K2 auto"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k2_auto.jsonl
