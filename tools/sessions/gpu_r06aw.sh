#!/bin/bash
# Round 6: the camera-ray hit records through buffer loads (a 32-bit lane offset from the
# wave-uniform record array): the whole GPU suite on the tree, then an interleaved K3
# chain A/B against the committed tree (the r06au build; tools/chain_ab.py).
set -o pipefail
TAG=${1:-r06aw}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python tools/chain_ab.py 4 $V/librt_hip_acc.so $V/librt_hip_buf.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -4 $O/chain_ab.jsonl
