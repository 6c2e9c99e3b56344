#!/bin/bash
# Round 6: the bounce instance's fast-core fallbacks against the oracle (new test), then the
# GPU suite's bounce and K5 tests.
set -o pipefail
TAG=${1:-r06t}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "fallbacks or bounce or k5" > $O/pytest_sel.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_sel.log; exit 1; }
grep -c PASSED $O/pytest_sel.log; tail -2 $O/pytest_sel.log
