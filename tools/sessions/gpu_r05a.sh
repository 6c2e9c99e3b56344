#!/bin/bash
# Round 5, session a: the -m gpu suite and smoke() on the round-4 build, the driver's bench
# command twice (this box's baseline), then the timeline of the driver's command (round-4
# verdict item 1): bench.py --gpus 1 --steps 20 --warmup 5 with RT_TIMELINE host stamps under
# rocprofv3 --kernel-trace (and once more with the HIP runtime API trace), analysed by
# tools/timeline.py.
# Usage: bash tools/sessions/gpu_r05a.sh TAG
set -o pipefail
TAG=${1:-r05a}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['timed_breakdown_ms'])"
done
RT_TIMELINE=1 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tlk -o tl -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
  > $O/tlk_line.json 2> $O/tlk.err || { echo "rocprof k failed"; tail $O/tlk.err; exit 1; }
python tools/timeline.py $O/tlk $O/tlk_line.json > $O/timeline_k.json || exit 1
python -c "import json; d=json.load(open('$O/timeline_k.json')); [d.pop(k) for k in ('hip_calls','kernels')]; print(json.dumps(d))"
RT_TIMELINE=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $O/tla -o tl -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
  > $O/tla_line.json 2> $O/tla.err || { echo "rocprof a failed"; tail $O/tla.err; exit 1; }
python tools/timeline.py $O/tla $O/tla_line.json > $O/timeline_a.json || exit 1
python -c "import json; d=json.load(open('$O/timeline_a.json')); [d.pop(k) for k in ('hip_calls','kernels')]; print(json.dumps(d))"
