#!/bin/bash
# Round 4, first session: the -m gpu suite (new: AQL give-up test, frame-images EVERY mode,
# fresh-context queue tests), smoke, the driver's bench command, and per-rank K3 shares:
# one dispatch per frame (RT_FPL=1) against fused frame chains storing every frame's image.
# Usage: bash tools/sessions/gpu_r04a.sh TAG
set -o pipefail
TAG=${1:-r04a}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; tail $O/smoke.log; exit 1; }
echo smoke ok
for mode in "RT_FPL=1" "RT_FPL=0 RT_IMAGES=every" "RT_FPL=0 RT_IMAGES=last_two"; do
  for steps in 20 64; do
    tag=$(echo "$mode $steps" | tr ' =' '__')
    env $mode RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 $steps > $O/rank_K3_$tag.jsonl || exit 1
    echo "rank K3 $mode steps=$steps"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['kernel'], d['frames_per_launch']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_K3_$tag.jsonl
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo bench failed; tail $O/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['queues'], r['submit'], r['frac'], d['image_ok'])"
