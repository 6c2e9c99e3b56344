#!/bin/bash
# Per-rank stripe timings (tools/rank_sim.py) for each library build given as
# lib[:ENV=V,...]; world sizes 1/2/4/8 on this one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${TAG:-rank}; mkdir -p $O
i=0
for L in "$@"; do
  i=$((i+1)); lib=${L%%:*}; envs=""; [ "$lib" != "$L" ] && envs=$(echo ${L#*:} | tr ',' ' ')
  env RT_HIP_LIB=$lib $envs timeout -k 10 200 python tools/rank_sim.py ${CFG:-K3} 50 > $O/rank_$i.jsonl 2>&1 || { tail -3 $O/rank_$i.jsonl; exit 1; }
  echo "$L"; grep '^{' $O/rank_$i.jsonl | python3 -c "import sys,json; print(' '.join('%d:%.2f' % (d['world'], d['us_per_step']) for d in map(json.loads, sys.stdin)))"
done
