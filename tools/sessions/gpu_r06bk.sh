#!/bin/bash
# Round 6 final tree (the split frame-group accumulation, AUTO's four waves per tile pair up
# to 20 000 tiles): the whole GPU suite, smoke, the driver's K3 command twice (its
# rank_shares side lines run AUTO at 2 / 4 / 8 ranks), and the K3 PMC passes.
set -o pipefail
TAG=${1:-r06bk}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo "bench failed"; tail $O/bench_driver_$r.err; exit 1; }
  python tools/summarize_bench.py $O/bench_driver_$r.json > $O/summary_driver_$r.txt; cat $O/summary_driver_$r.txt | cut -c1-300
done
PMC_ROUND=r06 bash tools/pmc_bench.sh $TAG "K3" > $O/pmc.log 2>&1 || { echo "pmc failed"; tail $O/pmc.log; exit 1; }
ls $O/pmc_r06_K3.json
