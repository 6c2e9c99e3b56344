#!/bin/bash
# Round 6: the pair sample in two instances by the hit normal's division mode (normal_rn a
# compile-time constant in the frame loop): the whole GPU suite, then a K3 chain A/B against
# the committed tree (the r06aw build; tools/chain_ab.py).
set -o pipefail
TAG=${1:-r06az}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python tools/chain_ab.py 4 $V/librt_hip_buf.so $V/librt_hip_rn2.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -4 $O/chain_ab.jsonl
