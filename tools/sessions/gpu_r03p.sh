#!/bin/bash
# Round-3 session p: the all-f32 defocus normalisation (RT_SINGLE_DISK=3) and the lens
# centre in VGPRs (RT_ORIGIN_VGPR): parity (selftest over all 2^32 seeds included) and A/B
# on K3 / K2.  Usage: bash tools/gpu_r03p.sh TAG
set -o pipefail
TAG=${1:-r03p}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_d3ovg.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread > $O/pytest_d3ovg.log 2>&1
rc=$?; echo "pytest d3ovg rc=$rc"; tail -2 $O/pytest_d3ovg.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 3 default $V/librt_hip_disk3.so $V/librt_hip_ovg.so \
  $V/librt_hip_d3ovg.so || exit 1
