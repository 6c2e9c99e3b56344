#!/bin/bash
# Round 5, session b: the fixed cost of the driver's 20-step K3 command, A/B in one process
# (tools/driver_region.py, variants interleaved repetition by repetition): the fork skipped on
# an idle stream (default) against the recorded fork (RT_FORK=0), the CPython binding of the
# call against ctypes (RT_FASTCALL=0), both off (round 4's path), two against three parts;
# then the same with the runtime's host wait spinning (ROC_ACTIVE_WAIT_TIMEOUT, hipDeviceScheduleSpin).
# Usage: bash tools/sessions/gpu_r05b.sh TAG
set -o pipefail
TAG=${1:-r05b}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python tools/driver_region.py 25 K3 base= spin=\;wait=spin fork0=RT_FORK=0 ctypes=RT_FASTCALL=0 r4=RT_FORK=0,RT_FASTCALL=0 q3=\;queues=3 q3spin=\;queues=3\;wait=spin \
  > $O/region_k3.jsonl 2> $O/region_k3.err || { tail $O/region_k3.err; exit 1; }
cat $O/region_k3.jsonl
ROC_ACTIVE_WAIT_TIMEOUT=2000 timeout -k 10 200 python tools/driver_region.py 25 K3 base= spin=\;wait=spin \
  > $O/region_k3_wait2000.jsonl 2> $O/region_k3_wait2000.err || { tail $O/region_k3_wait2000.err; exit 1; }
cat $O/region_k3_wait2000.jsonl
for r in 1 2; do
  for hw in spin block; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --host-wait $hw > $O/bench_driver_${hw}_$r.json 2> $O/bench_driver_${hw}_$r.err \
      || { echo bench failed; tail $O/bench_driver_${hw}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_driver_${hw}_$r.json')); r=d['roofline']; print('driver', '$hw', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['timed_breakdown_ms'], d.get('k2',{}).get('us_per_step'), d['rank_shares']['K3']['chain']['8'])"
  done
done
RT_REGION_SPIN=1 timeout -k 10 200 python tools/driver_region.py 25 K3 base= spin=\;wait=spin \
  > $O/region_k3_spin.jsonl 2> $O/region_k3_spin.err || { tail $O/region_k3_spin.err; exit 1; }
cat $O/region_k3_spin.jsonl
