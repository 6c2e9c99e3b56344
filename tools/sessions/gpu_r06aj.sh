#!/bin/bash
# Round 6: the grid walk's cell ranges, item records and item indices through buffer loads:
# the bounce / grid / K5 parity tests, then a K5 A/B against the committed
# tree (head).
set -o pipefail
TAG=${1:-r06aj}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "fallbacks or bounce or k5 or grid or culled" > $O/pytest_sel.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_sel.log; exit 1; }
tail -1 $O/pytest_sel.log
timeout -k 10 900 python tools/k5_ab.py 4 $V/librt_hip_head.so tree > $O/k5_ab.jsonl 2> $O/k5_ab.err \
  || { echo "ab failed"; tail $O/k5_ab.err; exit 1; }
tail -1 $O/k5_ab.jsonl
