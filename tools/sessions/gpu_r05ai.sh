#!/bin/bash
# Round 5: the tile-pair instances named rt_tpair_kernel<2> / <4> as rocprofv3 lists them
# (int template parameter): the GPU suite, the PMC passes of K4's timed kernel, then
# bench.py --config K4 twice with that summary in profiles/ (its roofline's `traffic`).
# Usage: bash tools/sessions/gpu_r05ai.sh TAG
set -o pipefail
TAG=${1:-r05ai}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
PMC_ROUND=r05 QUEUES=0 bash tools/pmc_bench.sh ${TAG}_pmc "K4" || exit 1
cat gpurun_out/${TAG}_pmc/pmc_r05_K4.json | head -c 600; echo
cp gpurun_out/${TAG}_pmc/pmc_r05_K4.json profiles/pmc_r05_K4.json
for r in 1 2; do
  timeout -k 10 300 python bench.py --config K4 --cpu-seconds 0 > $O/bench_k4_$r.json 2> $O/bench_k4_$r.err \
    || { echo "bench failed"; tail $O/bench_k4_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_k4_$r.json')); r=d['roofline']; print('K4', d['value'], d['ms_per_step'], d.get('image_ok'), r.get('kernel'), r.get('frac'), r.get('traffic'))"
done
