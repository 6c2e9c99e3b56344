#!/bin/bash
# GPU session: -m gpu tests on the product build, interleaved A/B of library builds
# (args) on K3 and K2, then per-rank stripe timings (tools/rank_sim.py) for each build.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${TAG:-order}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for c in k3 k2; do
  timeout -k 10 400 python tools/ab_variants.py $c 3 "$@" > $O/ab_$c.log 2>&1 || exit 1
  tail -$# $O/ab_$c.log
done
i=0
for L in "$@"; do
  i=$((i+1))
  RT_HIP_LIB=${L%%:*} timeout -k 10 200 python tools/rank_sim.py K3 50 > $O/rank_$i.jsonl 2>&1 || exit 1
  echo "$L"; grep '^{' $O/rank_$i.jsonl | python3 -c "import sys,json; print(' '.join('%d:%.2f' % (d['world'], d['us_per_step']) for d in map(json.loads, sys.stdin)))"
done
