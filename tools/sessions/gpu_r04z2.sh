#!/bin/bash
# Round 4, session z2: K4 (64 fused frames per step at 1920x1080) with the final build and
# with RT_SKY_RSQ=0 (the sky's / normalize_w's reciprocal from v_rcp, as in round 3), three
# interleaved rounds of bench.py --config K4.
# Usage: bash tools/sessions/gpu_r04z2.sh TAG
set -o pipefail
TAG=${1:-r04z2}
cd $GRAFT_REPO_ROOT
V=gpu-ray-tracing_amd/build/variants
bash tools/gpu_ab_bench.sh $TAG "K4" 3 default $V/librt_hip_rsq0.so || exit 1
