#!/bin/bash
# -m gpu tests, then K5 launch modes and the K5 per-rank prediction (fused launches).
set -o pipefail
TAG=${1:-k5}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/k5_modes.py per_wave compact > $O/k5_modes.jsonl 2>&1 || { tail $O/k5_modes.jsonl; exit 1; }
cat $O/k5_modes.jsonl
timeout -k 10 600 python tools/rank_sim.py K5 64 > $O/rank_k5.jsonl 2>&1 || { tail $O/rank_k5.jsonl; exit 1; }
grep '^{' $O/rank_k5.jsonl
