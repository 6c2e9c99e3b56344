#!/bin/bash
# Round 6: the bounce kernel's register plan for 6 waves per SIMD (RT_BOUNCE_MIN_WAVES=6:
# 100 SGPRs, fewer SGPR spills into VGPR lanes, no scratch in rt_bounce_kernel<0>, 7 waves
# resident at most) against the tree's 7 (8 resident): interleaved K5 A/B (tools/k5_ab.py,
# 1 GPU and rank 0's 8-rank share, digests checked).
set -o pipefail
TAG=${1:-r06bb}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 600 python tools/k5_ab.py 3 $V/librt_hip_buf.so $V/librt_hip_bw6.so > $O/k5_ab.jsonl 2> $O/k5_ab.err \
  || { echo "k5_ab failed"; tail $O/k5_ab.err; exit 1; }
tail -1 $O/k5_ab.jsonl
