#!/bin/bash
# Round 4, session x: frame groups of eight waves per tile (RT_FRAME_PAIRS_OCT, opt-in): the
# -m gpu suite (oct cases added), then K3 frame-chain rank shares with auto / quad / oct
# (tools/rank_sim.py, RT_FPL=0 RT_IMAGES=every, 5 blocks), two rounds.
# Usage: bash tools/sessions/gpu_r04x.sh TAG
set -o pipefail
TAG=${1:-r04x}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2; do
  for m in auto oct; do
    RT_FPL=0 RT_IMAGES=every RT_REPS=5 RT_FRAME_PAIRS=$m timeout -k 10 300 python tools/rank_sim.py K3 20 \
      > $O/rank_K3_${m}_$r.jsonl 2>> $O/rank.err || { echo "rank_sim $m failed"; tail -5 $O/rank.err; exit 1; }
    python -c "import json; [print('$m r$r', d['world'], d['us_per_step'], d['predicted_efficiency'], d.get('kernel')) for d in map(json.loads, open('$O/rank_K3_${m}_$r.jsonl'))]"
  done
done
