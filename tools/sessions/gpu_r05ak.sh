#!/bin/bash
# Round 5, closing evidence of the final tree (after the sphere-grid and tile-pair changes):
# the GPU suite and smoke, the driver's K3 command's main line three times (--side 0), and
# bench.py --config K4 / K5 main lines (one GPU each).
# Usage: bash tools/sessions/gpu_r05ak.sh TAG
set -o pipefail
TAG=${1:-r05ak}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 > $O/bench_k3_$r.json 2> $O/bench_k3_$r.err \
    || { echo "bench failed"; tail $O/bench_k3_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_k3_$r.json')); r=d['roofline']; print('K3', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['cpu_baseline']['value'])"
done
for c in K4 K5; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 > $O/bench_$c.json 2> $O/bench_$c.err \
    || { echo "bench failed"; tail $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r.get('kernel'), r.get('frac'), d.get('image_ok'))"
done
