#!/bin/bash
# Round 6: the ADVICE fixes, the digest-checked K5 / bench tests, band sets (ABI 7), and the
# new bench.py (one launch structure at every N, CLOCK_MONOTONIC job time, wall-clock rank
# shares).
set -o pipefail
TAG=${1:-r06e}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "selftest or markstein or normal or k5 or bench_dispatch or band_set or partition" > $O/pytest_sel.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_sel.log; exit 1; }
tail -2 $O/pytest_sel.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "bench failed"; tail $O/bench_driver.err; exit 1; }
python tools/summarize_bench.py $O/bench_driver.json
