#!/bin/bash
# Round 4, session c: the -m gpu suite (split bounce mode), then K5 per-rank shares with the
# split schedule (AUTO) against per wave, and RT_BOUNCE_SPLIT 2 / 4 / 8 at 8 ranks.
# Usage: bash tools/sessions/gpu_r04c.sh TAG
set -o pipefail
TAG=${1:-r04c}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for mode in "RT_PATHS=auto" "RT_PATHS=per_wave" "RT_PATHS=split RT_BOUNCE_SPLIT=8"; do
  tag=$(echo "$mode" | tr ' =' '__')
  env $mode RT_REPS=3 timeout -k 10 300 python tools/rank_sim.py K5 64 > $O/rank_K5_$tag.jsonl || exit 1
  echo "rank K5 $mode"; python -c "import json,sys; [print(' ', d['world'], d['us_per_step'], d['predicted_efficiency'], d['kernel'], d['runs_us']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_K5_$tag.jsonl
done
