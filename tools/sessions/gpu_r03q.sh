#!/bin/bash
# Round-3 session q: lane-mask decisions in the one-frame kernel (RT_SINGLE_MASKS) alone and
# with the f32 defocus normalisation + lens centre in VGPRs: parity and A/B on K3 / K2.
# Usage: bash tools/gpu_r03q.sh TAG
set -o pipefail
TAG=${1:-r03q}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
for v in all masks; do
  RT_HIP_LIB=$V/librt_hip_$v.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 \
    --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit 1
done
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 4 default $V/librt_hip_masks.so $V/librt_hip_all.so || exit 1
