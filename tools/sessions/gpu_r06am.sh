#!/bin/bash
# tpair<4> (four waves per tile pair) compiled for 8 waves per SIMD (64 VGPRs, 40 B scratch)
# against the tree's 7 (71 VGPRs): at 8 ranks the share's 8 160 waves then fit one generation
# (8 192 slots) instead of 1.14 of 7 168.  Rank 0's K3 share, 20 steps (tools/share_region.py),
# both builds through RT_HIP_LIB, the order rotating over four rounds.
set -o pipefail
TAG=${1:-r06am}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
L=(base t48)
for rd in 0 1 2 3; do
  for i in 0 1; do
    l=${L[$(( (i + rd) % 2 ))]}
    for nm in "8 quad" "8 quad2" "4 quad2" "2 quad2"; do
      set -- $nm
      RT_HIP_LIB=$V/librt_hip_$l.so timeout -k 10 120 python tools/share_region.py $1 0 15 20 $2 > $O/line.json 2> $O/err.txt \
        || { echo "share_region $l $nm failed"; tail $O/err.txt; exit 1; }
      python -c "import json; d=json.load(open('$O/line.json')); d.pop('timeline_host'); d['round']=$rd; d['lib']='$l'; print(json.dumps(d))" >> $O/ab.jsonl || exit 1
    done
  done
  echo "round $rd done"
done
python - <<PY
import json, statistics as st
rows=[json.loads(l) for l in open("$O/ab.jsonl")]
for n, m in ((8,"quad"),(8,"quad2"),(4,"quad2"),(2,"quad2")):
    for l in ("base","t48"):
        r=[x for x in rows if x["share"]==f"rank 0 of {n}" and x["pairs"]==m and x["lib"]==l]
        print(n, m, l, r[0]["kernel"], "wall", round(st.median(x["wall_us_per_step_q1_med_q3"][1] for x in r),3),
              "events", round(st.median(x["events_us_per_step_q1_med_q3"][1] for x in r),3))
PY
