#!/bin/bash
# Round-3 session m: raised wave priority for the costliest workgroups, repeated per-rank
# predictions (medians of RT_REPS launches): bounce instance (K5) and one-frame kernel (K3).
# Usage: bash tools/gpu_r03m.sh TAG
set -o pipefail
TAG=${1:-r03m}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_sprio1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "dispatch or queues or stripes" --timeout 200 --timeout-method thread > $O/pytest_sprio.log 2>&1
rc=$?; echo "pytest sprio1024 rc=$rc"; tail -2 $O/pytest_sprio.log; [ $rc -eq 0 ] || exit 1
for round in 1 2; do
  for v in default prio512 prio2048; do
    E=""; [ $v != default ] && E="RT_HIP_LIB=$V/librt_hip_$v.so"
    env $E RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K5 64 > $O/rank_k5_${v}_$round.jsonl 2>&1 || exit 1
    echo k5 $v $round; grep '^{' $O/rank_k5_${v}_$round.jsonl | cut -c1-200
  done
done
for v in default sprio512 sprio1024 sprio2048; do
  E=""; [ $v != default ] && E="RT_HIP_LIB=$V/librt_hip_$v.so"
  env $E RT_REPS=5 RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_$v.jsonl 2>&1 || exit 1
  echo k3 $v; grep '^{' $O/rank_k3_$v.jsonl | cut -c1-200
done
