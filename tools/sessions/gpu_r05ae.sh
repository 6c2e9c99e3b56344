#!/bin/bash
# Round 5: the GPU suite and smoke on the tree with one small sphere per grid cell
# (RT_GRID_PER_CELL 1.0, after r05ab / r05ac).
# Usage: bash tools/sessions/gpu_r05ae.sh TAG
set -o pipefail
TAG=${1:-r05ae}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
