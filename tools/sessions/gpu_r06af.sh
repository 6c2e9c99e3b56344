#!/bin/bash
# Round 6: one VGPR copy of the lens centre for both pixels of a tile-pair lane (c0) and, on top,
# the tile-pair kernel re-reading its unit and list counts each frame (c0rm2), against the
# committed tree (head); every build through RT_HIP_LIB, order rotating (tools/chain_ab.py).
# The camera-ray GPU tests first.
set -o pipefail
TAG=${1:-r06af}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 1200 python tools/chain_ab.py 6 $V/librt_hip_head.so $V/librt_hip_c0.so $V/librt_hip_c0rm2.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
