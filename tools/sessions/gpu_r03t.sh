#!/bin/bash
# Round-3 session t: the head build's -m gpu suite, the lane-mask build (RT_SINGLE_MASKS) and
# the combined build (masks + f32 defocus normalisation + lens centre in VGPRs) checked, then
# an interleaved A/B on K3 / K2.  Usage: bash tools/gpu_r03t.sh TAG
set -o pipefail
TAG=${1:-r03t}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_head.log 2>&1
rc=$?; echo "pytest head rc=$rc"; tail -2 $O/pytest_head.log; [ $rc -eq 0 ] || exit 1
for v in masks all; do
  RT_HIP_LIB=$V/librt_hip_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit 1
done
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 4 default $V/librt_hip_masks.so $V/librt_hip_all.so || exit 1
