#!/bin/bash
# Round 4, session a2: the one-frame kernel's shape — three or four tiles per wave
# (RT_SINGLE_PIX), eight- or two-wave workgroups (RT_SINGLE_WG) — against the in-tree build
# (two tiles, four waves), K3 at bench.py's default length, three interleaved rounds.
# Usage: bash tools/sessions/gpu_r04a2.sh TAG
set -o pipefail
TAG=${1:-r04a2}
cd $GRAFT_REPO_ROOT
V=gpu-ray-tracing_amd/build/variants
bash tools/gpu_ab_bench.sh $TAG "K3" 3 default $V/librt_hip_pix3.so $V/librt_hip_pix4.so \
  $V/librt_hip_wg8.so $V/librt_hip_wg2.so || exit 1
