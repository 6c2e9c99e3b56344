#!/bin/bash
# Round-3 session z: AQL submission with the frame packets' arguments in a host-visible VRAM
# ring (HDP flush per segment): the AQL / queue / dispatch-chain parity tests, then A/B at warm
# clocks against HIP launches (K3 / K2) and per-rank predictions.  Usage: bash tools/gpu_r03z.sh TAG
set -o pipefail
TAG=${1:-r03z}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "submit or queues or dispatch_chain" > $O/pytest_aql.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_aql.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 2 default default:RT_SUBMIT=aql,RT_QUEUES=1 \
  default:RT_SUBMIT=aql,RT_QUEUES=2 default:RT_SUBMIT=aql,RT_QUEUES=3 || exit 1
for spec in hip:0 aql:1 aql:2; do
  m=${spec%:*}; q=${spec#*:}
  RT_FPL=1 RT_SUBMIT=$m RT_QUEUES=$q RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_${m}_q$q.jsonl || exit 1
  echo "rank K3 $m q$q"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_${m}_q$q.jsonl
done
