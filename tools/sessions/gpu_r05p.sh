#!/bin/bash
# Round 5, session p: the GPU suite with the random-radii parity case of the hit normal's
# two division paths.
# Usage: bash tools/sessions/gpu_r05p.sh TAG
set -o pipefail
TAG=${1:-r05p}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "random_radii" \
  > $O/pytest_radii.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_radii.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest_radii.log | tail -10
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
