#!/bin/bash
# Round 4, session i: timing of the one-frame kernel's knock-out builds (RT_SKO 1 no
# accumulator load, 2 no sphere scan, 4 no random camera ray, 8 no hit shading) against the
# in-tree build, interleaved bench.py K3 runs (images differ: timing only), to see how far
# the update's time follows its VALU count (profiles/r04/r04fg_knockout_valu.txt).
# Usage: bash tools/sessions/gpu_r04i.sh TAG
set -o pipefail
TAG=${1:-r04i}
cd $GRAFT_REPO_ROOT
V=gpu-ray-tracing_amd/build/variants
bash tools/gpu_ab_bench.sh $TAG "K3" 2 default $V/librt_hip_sko1.so $V/librt_hip_sko2.so \
  $V/librt_hip_sko4.so $V/librt_hip_sko8.so
