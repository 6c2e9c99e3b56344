#!/bin/bash
# Upper bound of taking the foreign-count fallback out of the tile-pair kernel: without it
# (RT_TPAIR_NOFB=1: wrong only for pixels whose counts differ from the hint, which no timed
# region has) the instances need 58 VGPRs instead of 71 — 8 waves per SIMD instead of 7 —
# and spill 10-14 SGPRs instead of 28-30.  tools/chain_ab.py (whole image; digests checked)
# and rank 0's 8-rank (quad2), 4-rank and 2-rank (AUTO) K3 shares, tree / nofb (planned for 7
# waves) / nofb8 (for 8), through RT_HIP_LIB, the order rotating.
set -o pipefail
TAG=${1:-r06ar}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 700 python tools/chain_ab.py 4 $V/librt_hip_base.so $V/librt_hip_nofb.so $V/librt_hip_nofb8.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
L=(base nofb nofb8)
for rd in 0 1 2; do
  for i in 0 1 2; do
    l=${L[$(( (i + rd) % 3 ))]}
    for nm in "8 quad2" "4 auto" "2 auto"; do
      set -- $nm
      RT_HIP_LIB=$V/librt_hip_$l.so timeout -k 10 120 python tools/share_region.py $1 0 11 20 $2 > $O/line.json 2> $O/err.txt \
        || { echo "share_region $l $nm failed"; tail $O/err.txt; exit 1; }
      python -c "import json; d=json.load(open('$O/line.json')); d.pop('timeline_host'); d['round']=$rd; d['lib']='$l'; print(json.dumps(d))" >> $O/shares.jsonl || exit 1
    done
  done
done
python - <<PY
import json, statistics as st
rows=[json.loads(l) for l in open("$O/shares.jsonl")]
for n, m in ((8, "quad2"), (4, "auto"), (2, "auto")):
    for l in ("base", "nofb", "nofb8"):
        r=[x for x in rows if x["share"]==f"rank 0 of {n}" and x["pairs"]==m and x["lib"]==l]
        print(n, m, l, r[0]["kernel"], "wall", round(st.median(x["wall_us_per_step_q1_med_q3"][1] for x in r),3),
              "events", round(st.median(x["events_us_per_step_q1_med_q3"][1] for x in r),3))
PY
