#!/bin/bash
# Round 6: the tile-pair kernel re-deriving its list pointers and counts every frame (SALU)
# instead of keeping them live (45 -> 28 SGPR spills): the whole GPU suite, then the K3
# chain A/B against the tree before (pre).
set -o pipefail
TAG=${1:-r06ac}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python tools/chain_ab.py 5 $V/librt_hip_pre.so tree > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
