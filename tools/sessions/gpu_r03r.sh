#!/bin/bash
# Round-3 session r: one-frame updates as AQL packets on context-owned HSA queues
# (rt_set_update_submit): parity (the whole -m gpu suite runs AUTO = AQL), A/B against HIP
# launches on K3 / K2 (bench.py default length and the driver's 20-step command), per-rank
# predictions.  Usage: bash tools/gpu_r03r.sh TAG
set -o pipefail
TAG=${1:-r03r}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 3 default:RT_SUBMIT=hip default:RT_SUBMIT=aql || exit 1
for r in 1 2; do
  for m in hip aql; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      --submit $m > $O/driver_${m}_$r.json || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['queues'], d['roofline']['submit'], d['image_ok'])" $O/driver_${m}_$r.json $m
  done
done
for m in hip aql; do
  RT_FPL=1 RT_SUBMIT=$m RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_$m.jsonl || exit 1
  echo "rank K3 $m"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_$m.jsonl
done
for q in 1 2 4; do
  RT_FPL=1 RT_SUBMIT=aql RT_QUEUES=$q RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3_aql_q$q.jsonl || exit 1
  echo "rank K3 aql q$q"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['host_issue_us_per_step'], d['queues'], d['submit']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_k3_aql_q$q.jsonl
done
