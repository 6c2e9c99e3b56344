#!/bin/bash
# -m gpu tests, K5 launch modes on the whole image, per-rank K5 prediction per path mode.
set -o pipefail
TAG=${1:-k5paths}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/k5_modes.py per_wave pair > $O/k5_modes.jsonl 2>&1 || { tail $O/k5_modes.jsonl; exit 1; }
grep '"launch": 2' $O/k5_modes.jsonl
for m in auto per_wave pair; do
  RT_PATHS=$m timeout -k 10 600 python tools/rank_sim.py K5 64 > $O/rank_$m.jsonl 2>&1 || { tail $O/rank_$m.jsonl; exit 1; }
  echo "== $m"; grep '^{' $O/rank_$m.jsonl
done
