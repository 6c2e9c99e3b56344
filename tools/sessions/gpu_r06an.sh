#!/bin/bash
# The share's frame-group modes where AUTO picks plain frame pairs today (rt_trace_kernel<3>,
# 6 145 - 23 999 tiles): rank 0's K3 share at 3, 4 and 2 ranks (20 steps, and 200 at 4 and 2),
# and the K2 scene's shares at 8, 4 and 2 ranks, in `quad2` / `on` / `on2` (and `quad`), the
# order rotating over three rounds (tools/share_region.py).
set -o pipefail
TAG=${1:-r06an}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
run() {  # cfg n frames modes...
  local cfg=$1 n=$2 f=$3; shift 3
  local M=("$@") k=${#M[@]}
  for i in $(seq 0 $((k - 1))); do
    m=${M[$(( (i + rd) % k ))]}
    SHARE_CFG=$cfg timeout -k 10 120 python tools/share_region.py $n 0 11 $f $m > $O/line.json 2> $O/err.txt \
      || { echo "share_region $cfg $n $f $m failed"; tail $O/err.txt; return 1; }
    python -c "import json; d=json.load(open('$O/line.json')); d.pop('timeline_host'); d['round']=$rd; print(json.dumps(d))" >> $O/modes.jsonl || return 1
  done
}
for rd in 0 1 2; do
  run K3 3 20 quad quad2 on on2 || exit 1
  run K3 4 20 quad2 on on2 || exit 1
  run K3 2 20 quad2 on on2 || exit 1
  run K3 4 200 quad2 on on2 || exit 1
  run K3 2 200 quad2 on on2 || exit 1
  run K2 8 20 quad quad2 on on2 || exit 1
  run K2 4 20 quad quad2 on on2 || exit 1
  run K2 2 20 quad quad2 on on2 || exit 1
  echo "round $rd done"
done
python - <<PY
import json, statistics as st
from collections import defaultdict
g=defaultdict(list)
for l in open("$O/modes.jsonl"):
    x=json.loads(l); g[(x["config"], x["share"], x["steps"], x["pairs"], x["kernel"])].append(x)
for k, r in g.items():
    print(*k, "wall", round(st.median(x["wall_us_per_step_q1_med_q3"][1] for x in r),3),
          "events", round(st.median(x["events_us_per_step_q1_med_q3"][1] for x in r),3))
PY
