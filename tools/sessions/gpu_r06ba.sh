#!/bin/bash
# Round 6: persistent tile-pair workgroups (RT_TPAIR_PERSIST=1: as many workgroups as are
# resident at once, each taking the next cost-ordered unit from a device queue) against the
# same tree built without (K3 chain A/B, tools/chain_ab.py; each run checks the whole-image
# digest), then the GPU suite on the tree as built by default.
set -o pipefail
TAG=${1:-r06ba}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 400 python tools/chain_ab.py 4 $V/librt_hip_base2.so $V/librt_hip_persist.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
