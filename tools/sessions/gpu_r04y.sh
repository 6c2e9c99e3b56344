#!/bin/bash
# Round 4, session y: the bench line with its K4 side measurement — the driver's command and
# the default line.
# Usage: bash tools/sessions/gpu_r04y.sh TAG
set -o pipefail
TAG=${1:-r04y}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
t0=$(date +%s.%N)
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo bench failed; tail $O/bench_driver.err; exit 1; }
echo "$(date +%s.%N) $t0" | awk '{printf "%.1f s\n", $1 - $2}' > $O/bench_driver.time
python -c "import json; d=json.load(open('$O/bench_driver.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['k4'])"
cat $O/bench_driver.time
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo bench failed; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; k=d['rank_shares']['K5']['fused_64']; print('default', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['k4']['us_per_step'], d['k4']['image_ok'], {w: (v['us_per_step'], v['predicted_efficiency']) for w, v in k.items()})"
