#!/bin/bash
# Round 5, session c: where the driver's 20-step region loses time against bench.py's default
# length, on the GPU side.  Kernel traces (rocprofv3 --kernel-trace, RT_TIMELINE host stamps,
# tools/timeline.py) of bench.py --steps 20 --warmup 5 as the driver runs it and with the
# issue gated (--gate: the GPU runs the steps back to back whatever the profiler's per-launch
# host cost), and gated at --steps 200; bench.py with no flags (the default length); the PMC
# passes of the timed K3 kernel at the timed launch structure (two concurrent parts).
# Usage: bash tools/sessions/gpu_r05c.sh TAG
set -o pipefail
TAG=${1:-r05c}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in "g20:--gate --steps 20 --warmup 5" "u20:--steps 20 --warmup 5" "g200:--gate --steps 200 --warmup 20"; do
  n=${v%%:*}; a=${v#*:}
  RT_TIMELINE=1 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tl_$n -o tl -- python3 bench.py --gpus 1 $a --side 0 --cpu-seconds 0 \
    > $O/tl_${n}_line.json 2> $O/tl_$n.err || { echo "rocprof $n failed"; tail $O/tl_$n.err; exit 1; }
  python tools/timeline.py $O/tl_$n $O/tl_${n}_line.json > $O/timeline_$n.json || exit 1
  python -c "import json; d=json.load(open('$O/timeline_$n.json')); [d.pop(k) for k in ('hip_calls','kernels')]; print('$n', json.dumps(d))"
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo bench failed; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['timed_breakdown_ms'])"
done
PMC_ROUND=r05 QUEUES=0 bash tools/pmc_bench.sh ${TAG}_pmc "K3" || exit 1
echo pmc done
