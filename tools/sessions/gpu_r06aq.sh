#!/bin/bash
# Tile-pair frame groups with the accumulating wave rotating by group (RT_TPAIR_ROTATE=1)
# against wave 0 accumulating every group: tools/chain_ab.py (whole image: rt_tpair_kernel<2>;
# its 8-rank share runs rt_trace_kernel<4>, unchanged), then rank 0's 4- and 2-rank K3 shares
# (rt_tpair_kernel<4> / <2>) by tools/share_region.py; both builds through RT_HIP_LIB, the
# order rotating.
set -o pipefail
TAG=${1:-r06aq}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 600 python tools/chain_ab.py 4 $V/librt_hip_base.so $V/librt_hip_rot.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
L=(base rot)
for rd in 0 1 2 3; do
  for i in 0 1; do
    l=${L[$(( (i + rd) % 2 ))]}
    for n in 4 2; do
      RT_HIP_LIB=$V/librt_hip_$l.so timeout -k 10 120 python tools/share_region.py $n 0 11 20 auto > $O/line.json 2> $O/err.txt \
        || { echo "share_region $l $n failed"; tail $O/err.txt; exit 1; }
      python -c "import json; d=json.load(open('$O/line.json')); d.pop('timeline_host'); d['round']=$rd; d['lib']='$l'; print(json.dumps(d))" >> $O/shares.jsonl || exit 1
    done
  done
done
python - <<PY
import json, statistics as st
rows=[json.loads(l) for l in open("$O/shares.jsonl")]
for n in (4, 2):
    for l in ("base", "rot"):
        r=[x for x in rows if x["share"]==f"rank 0 of {n}" and x["lib"]==l]
        print(n, l, r[0]["kernel"], "wall", round(st.median(x["wall_us_per_step_q1_med_q3"][1] for x in r),3),
              "events", round(st.median(x["events_us_per_step_q1_med_q3"][1] for x in r),3))
PY
