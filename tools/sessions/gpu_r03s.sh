#!/bin/bash
# Round-3 session s: AQL one-frame updates with device-staged kernel arguments: the AQL and
# dispatch-chain parity tests, then A/B against HIP launches (K3 / K2, default length and the
# driver's 20-step command) and per-rank predictions.  Usage: bash tools/gpu_r03s.sh TAG
set -o pipefail
TAG=${1:-r03s}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "submit or queues or dispatch_chain" > $O/pytest_aql.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_aql.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 3 default:RT_SUBMIT=hip default:RT_SUBMIT=aql || exit 1
for r in 1 2; do
  for m in hip aql; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      --submit $m > $O/driver_${m}_$r.json || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['queues'], d['roofline']['submit'], d['image_ok'])" $O/driver_${m}_$r.json $m
  done
done
for spec in hip:0 aql:0 aql:1 aql:2 aql:4; do
  m=${spec%:*}; q=${spec#*:}
  RT_FPL=1 RT_SUBMIT=$m RT_QUEUES=$q RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_${m}_q$q.jsonl || exit 1
  echo "rank K3 $m q$q"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_${m}_q$q.jsonl
done
