#!/bin/bash
# K5 launch modes + per-rank prediction for library builds: bash tools/gpu_k5ab.sh TAG lib...
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for L in "$@"; do
  n=$(basename $L .so)
  RT_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python tools/k5_modes.py per_wave > $O/k5_$n.jsonl 2>&1 || { tail $O/k5_$n.jsonl; exit 1; }
  echo "$n $(tail -1 $O/k5_$n.jsonl)"
  RT_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 600 python tools/rank_sim.py K5 64 > $O/rank_$n.jsonl 2>&1 || { tail $O/rank_$n.jsonl; exit 1; }
  grep '^{' $O/rank_$n.jsonl | tail -3
done
