#!/bin/bash
# The share's frame-group modes re-measured on the kept tree (r06c measured them the same,
# before the tile-pair kernel's later changes): rank 0's 8-, 4- and 2-rank K3 shares, 20 steps,
# in `quad` (four waves per tile, AUTO's choice at 8 ranks), `quad2` (four per tile pair),
# `on` and `on2`, the order rotating over three rounds.
set -o pipefail
TAG=${1:-r06al}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
M=(quad quad2 on on2)
for rd in 0 1 2; do
  for n in 8 4 2; do
    for i in 0 1 2 3; do
      m=${M[$(( (i + rd) % 4 ))]}
      timeout -k 10 120 python tools/share_region.py $n 0 15 20 $m > $O/line.json 2> $O/err.txt \
        || { echo "share_region $n $m failed"; tail $O/err.txt; exit 1; }
      python -c "import json,sys; d=json.load(open('$O/line.json')); d.pop('timeline_host'); d['round']=$rd; print(json.dumps(d))" >> $O/modes.jsonl || exit 1
    done
  done
  echo "round $rd done"
done
python - <<PY
import json, statistics as st
rows=[json.loads(l) for l in open("$O/modes.jsonl")]
for n in (8,4,2):
    for m in ("quad","quad2","on","on2"):
        r=[x for x in rows if x["share"]==f"rank 0 of {n}" and x["pairs"]==m]
        print(n, m, r[0]["kernel"], "wall", round(st.median(x["wall_us_per_step_q1_med_q3"][1] for x in r),3),
              "events", round(st.median(x["events_us_per_step_q1_med_q3"][1] for x in r),3))
PY
