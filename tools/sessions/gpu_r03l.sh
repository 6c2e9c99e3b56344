#!/bin/bash
# Round-3 session l: raised wave priority for the costliest bounce tiles (RT_BOUNCE_PRIO):
# parity, K5 lines and the per-rank prediction.  Usage: bash tools/gpu_r03l.sh TAG
set -o pipefail
TAG=${1:-r03l}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_prio1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "bounce or k5" --timeout 200 --timeout-method thread > $O/pytest_prio.log 2>&1
rc=$?; echo "pytest prio1024 rc=$rc"; tail -2 $O/pytest_prio.log; [ $rc -eq 0 ] || exit 1
for v in default prio512 prio1024 prio2048 prio4096; do
  E=""; [ $v != default ] && E="RT_HIP_LIB=$V/librt_hip_$v.so"
  env $E timeout -k 10 300 python tools/rank_sim.py K5 64 > $O/rank_k5_$v.jsonl 2>&1 || exit 1
  echo k5 $v; grep '^{' $O/rank_k5_$v.jsonl
done
