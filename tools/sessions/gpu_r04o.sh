#!/bin/bash
# Round 4, session o: concurrent parts per one-frame update (RT_QUEUES 1 / 2 / 3 / 4) at
# bench.py's default length and in the driver's 20-step command, interleaved; then the
# default bench line (K5 shares after two untimed launches, median of five).
# Usage: bash tools/sessions/gpu_r04o.sh TAG
set -o pipefail
TAG=${1:-r04o}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_ab_bench.sh ${TAG}_ab "K3" 2 default default:RT_QUEUES=1 default:RT_QUEUES=3 \
  default:RT_QUEUES=4 || exit 1
for r in 1 2 3; do
  for q in 2 3; do
    RT_QUEUES=$q timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      > $O/driver_q${q}_$r.json 2>> $O/driver.err || { echo bench failed; tail -5 $O/driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/driver_q${q}_$r.json')); print('driver q$q r$r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['image_ok'])"
  done
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo bench failed; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; k=d['rank_shares']['K5']['fused_64']; print('default', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], {w: (v['us_per_step'], v['predicted_efficiency']) for w, v in k.items()})"
