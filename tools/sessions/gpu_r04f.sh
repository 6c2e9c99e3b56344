#!/bin/bash
# Round 4, session f: interleaved bench.py A/B of one-frame-kernel variants (K3 and K2,
# three rounds): the sky's reciprocal from its rsq (sky), one record per tile and step in
# the joint list walk (chunk1), each tile's list in its own loop (scan2), the bit-compare
# count check (nchk), against the in-tree build.
# Usage: bash tools/sessions/gpu_r04f.sh TAG
set -o pipefail
TAG=${1:-r04f}
cd $GRAFT_REPO_ROOT
V=gpu-ray-tracing_amd/build/variants
bash tools/gpu_ab_bench.sh $TAG "K3 K2" 3 default $V/librt_hip_sky.so $V/librt_hip_chunk1.so \
  $V/librt_hip_scan2.so $V/librt_hip_nchk.so
