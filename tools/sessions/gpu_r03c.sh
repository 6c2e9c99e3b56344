#!/bin/bash
# Round-3 session c: tests of the reset-split one-frame kernel (7-wave register plan), then
# A/B of its instruction-level switches (RT_SINGLE_NCHK, RT_SINGLE_VCONST, 8-wave plan) on
# K3 / K2 and their rank shares.  Usage: bash tools/gpu_r03c.sh TAG
set -o pipefail
TAG=${1:-r03c}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 3 default $V/librt_hip_nchk.so $V/librt_hip_vconst.so \
  $V/librt_hip_mw8.so $V/librt_hip_nv.so $V/librt_hip_nvm8.so || exit 1
for v in default nv nvm8; do
  E=""; [ $v != default ] && E="RT_HIP_LIB=$V/librt_hip_$v.so"
  env $E RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_dispatch_$v.jsonl 2>&1 || exit 1
  echo k3 $v; grep '^{' $O/rank_k3_dispatch_$v.jsonl
done
