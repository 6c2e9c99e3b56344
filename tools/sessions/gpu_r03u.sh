#!/bin/bash
# Round-3 session u: the new one-frame defaults (lane masks, f32 defocus normalisation, lens
# centre in VGPRs): -m gpu suite, fused / bounce instances A/B against the previous defaults
# (K4 / K5: RT_ORIGIN_VGPR reaches them through get_ray), PMC passes of K3 / K2 for the
# weighted VALU roofline.  Usage: bash tools/gpu_r03u.sh TAG
set -o pipefail
TAG=${1:-r03u}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_bench.sh $TAG/ab "K4 K5" 2 default $V/librt_hip_r03old.so || exit 1
bash tools/pmc_bench.sh $TAG "K3 K2" || exit 1
echo pmc done
