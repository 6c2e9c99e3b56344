#!/bin/bash
# Round 6: the whole GPU suite and smoke on the tree with band sets and the knock-out-free
# kernel, the N > 1 bench path rehearsed over gloo, and the K4 / K5 main lines.
set -o pipefail
TAG=${1:-r06g}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_rehearse.sh $TAG/rehearse || exit 1
for c in K4 K5; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 > $O/bench_$c.json 2> $O/bench_$c.err \
    || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python tools/summarize_bench.py $O/bench_$c.json
done
