#!/bin/bash
# Round 4, session t: K3 rank shares as frame chains (every frame's image, 20 frames per call)
# with each frame-group mode (RT_FRAME_PAIRS auto / off / on / quad): rank 0's share timed
# alone at 1 / 2 / 4 / 8 ranks (tools/rank_sim.py, 5 timed blocks).
# Usage: bash tools/sessions/gpu_r04t.sh TAG
set -o pipefail
TAG=${1:-r04t}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for m in auto off on quad; do
  RT_FPL=0 RT_IMAGES=every RT_REPS=5 RT_FRAME_PAIRS=$m timeout -k 10 300 python tools/rank_sim.py K3 20 \
    > $O/rank_K3_pairs_$m.jsonl 2>> $O/rank.err || { echo "rank_sim $m failed"; tail -5 $O/rank.err; exit 1; }
  python -c "import json,sys; [print('$m', d['world'], d['us_per_step'], d['predicted_efficiency'], d.get('kernel')) for d in map(json.loads, open('$O/rank_K3_pairs_$m.jsonl'))]"
done
