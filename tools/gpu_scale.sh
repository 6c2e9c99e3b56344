#!/bin/bash
# Product build: -m gpu tests, per-rank stripe timings (K3, K5) and a short K5 bench.
set -o pipefail
TAG=${1:-scale}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3.jsonl 2>&1 || { tail $O/rank_k3.jsonl; exit 1; }
cat $O/rank_k3.jsonl
timeout -k 10 300 python tools/rank_sim.py K5 4 > $O/rank_k5.jsonl 2>&1 || { tail $O/rank_k5.jsonl; exit 1; }
cat $O/rank_k5.jsonl
