#!/bin/bash
# Round 5: the tree with AUTO's tile-pair groups from 24 000 tiles (r05ag): the GPU suite and
# smoke, bench.py --config K4 twice, the driver's K3 command once (main line only, --side 0),
# and the PMC passes of K4's timed kernel (rt_tpair_kernel<2>, 64 frames per launch) for
# its roofline's `traffic`.
# Usage: bash tools/sessions/gpu_r05ah.sh TAG
set -o pipefail
TAG=${1:-r05ah}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --config K4 --cpu-seconds 0 > $O/bench_k4_$r.json 2> $O/bench_k4_$r.err \
    || { echo "bench failed"; tail $O/bench_k4_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_k4_$r.json')); print('K4', d['value'], d['ms_per_step'], d.get('image_ok'), d['roofline'].get('kernel'), d['roofline'].get('frac'))"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 > $O/bench_k3_main.json 2> $O/bench_k3_main.err \
  || { echo "bench failed"; tail $O/bench_k3_main.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_k3_main.json')); r=d['roofline']; print('K3 main', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
PMC_ROUND=r05 QUEUES=0 bash tools/pmc_bench.sh ${TAG}_pmc "K4" || exit 1
echo pmc done
