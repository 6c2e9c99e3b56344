#!/bin/bash
# One GPU session: tests, bench (K3 both scan modes, K2), rocprof kernel trace, HBM PMC
# passes per mode, issue/stall counters, phase stamps.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --scan exhaustive --cpu-seconds 0 > $O/bench_exhaustive.json 2>> $O/bench.err && cat $O/bench_exhaustive.json || exit 1
timeout -k 10 300 python bench.py --config K2 --cpu-seconds 0 > $O/bench_k2.json 2>> $O/bench.err && cat $O/bench_k2.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-seconds 0 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
head -4 $O/prof/bench_kernel_stats.csv
for m in culled exhaustive; do
 for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc -o ${m}_$c -- python3 bench.py --scan $m --cpu-seconds 0 --exhaustive-steps 0 --steps 20 > $O/pmc_${m}_$c.log 2>&1 || { echo pmc failed; exit 1; }
 done
done
bash tools/pmc_kernel.sh $TAG "k3 k2" || exit 1
for c in k3 k2; do RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_gst.so timeout -k 10 120 python tools/time_kernel.py $c || exit 1; done
