#!/bin/bash
# Round-3 A/B: rank shares of the per-dispatch step with the workgroup cost order (auto)
# against raster order (off).  At 8 ranks a share's waves are all resident at once, so the
# order cannot shorten its tail, while the order entry is one more dependent load per wave.
# Three interleaved rounds.  Usage: bash tools/gpu_r03zl.sh TAG
set -o pipefail
TAG=${1:-r03zl}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for c in K3 K2; do
    for o in auto off; do
      RT_TILE_ORDER=$o RT_FPL=1 RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py $c 50 \
        > $O/rank_${c}_${o}_$r.jsonl 2> $O/rank.err || { echo "rank_sim $c $o failed"; tail $O/rank.err; exit 1; }
      python -c "import json,sys; print('$c $o $r', ' '.join(f\"{d['world']}:{d['us_per_step']}:{d['submit']}\" for d in map(json.loads, open(sys.argv[1]))))" $O/rank_${c}_${o}_$r.jsonl
    done
  done
done
