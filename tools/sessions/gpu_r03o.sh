#!/bin/bash
# Round-3 final counters and predictions: PMC passes of the K3 / K2 one-frame kernel (one
# part per update, as the weighted-VALU tool expects) and the per-rank predictions (medians
# of repeated launches).  Usage: bash tools/gpu_r03o.sh TAG
set -o pipefail
TAG=${1:-r03o}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_bench.sh $TAG "K3 K2" || exit 1
RT_REPS=5 RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k3.jsonl | cut -c1-220
RT_REPS=3 RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K2 100 > $O/rank_k2.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k2.jsonl | cut -c1-220
RT_REPS=3 timeout -k 10 400 python tools/rank_sim.py K5 64 > $O/rank_k5.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k5.jsonl | cut -c1-220
