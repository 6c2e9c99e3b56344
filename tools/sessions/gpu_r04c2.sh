#!/bin/bash
# Round 4, session c2 (the final build, 2-wave one-frame workgroups): the -m gpu
# suite and smoke() on the committed build, the driver's
# bench command twice and the default bench line, the driver command's rocprofv3 kernel
# trace and the PMC passes of the timed K3 kernel.
# Usage: bash tools/sessions/gpu_r04c2.sh TAG
set -o pipefail
TAG=${1:-r04r}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  echo "$(date +%s.%N) $t0" | awk '{printf "%.1f s\n", $1 - $2}' > $O/bench_driver_$r.time
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
  cat $O/bench_driver_$r.time
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo bench failed; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > $O/prof_driver.log 2>&1 || { echo "rocprof failed"; tail $O/prof_driver.log; exit 1; }
echo rocprof done
PMC_ROUND=r04 bash tools/pmc_bench.sh ${TAG}_pmc "K3" || exit 1
echo pmc done
