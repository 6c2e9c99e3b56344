#!/bin/bash
# Round 6: the tree after the bounce and grid changes: the whole GPU suite, smoke, the driver's
# command and --config K5, the region counters, then the K5 and K3 PMC passes
# (tools/pmc_bench.sh) for the pmc_r06_K{3,5}.json the bench lines read.
set -o pipefail
TAG=${1:-r06z}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "bench failed"; tail $O/bench_driver.err; exit 1; }
timeout -k 10 400 python bench.py --config K5 > $O/bench_K5.json 2> $O/bench_K5.err \
  || { echo "bench K5 failed"; tail $O/bench_K5.err; exit 1; }
python tools/summarize_bench.py $O/bench_driver.json > $O/summary_driver.txt; head -3 $O/summary_driver.txt
python tools/summarize_bench.py $O/bench_K5.json > $O/summary_K5.txt; head -3 $O/summary_K5.txt
RT_HIP_LIB=$V/librt_hip_bc.so timeout -k 10 300 python tools/bounce_counts.py 1 > $O/counts_n1.json 2> $O/counts.err \
  || { echo "counts failed"; tail $O/counts.err; exit 1; }
PMC_ROUND=r06 bash tools/pmc_bench.sh $TAG "K5 K3" > $O/pmc.log 2>&1 || { echo "pmc failed"; tail $O/pmc.log; exit 1; }
ls $O/pmc_r06_K5.json $O/pmc_r06_K3.json
