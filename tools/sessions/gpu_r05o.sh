#!/bin/bash
# Round 5, session o: the runtime's active wait before it sleeps on the GPU's interrupt
# (ROC_ACTIVE_WAIT_TIMEOUT, µs; the HIP runtime's default 10) — the closing synchronize of the
# driver's region waits ~170 µs after the host's issue, past the default: the driver's K3
# region and the driver's command with 10 (default), 400 and 2000, separate processes,
# interleaved.
# Usage: bash tools/sessions/gpu_r05o.sh TAG
set -o pipefail
TAG=${1:-r05o}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in def 400 2000; do
    if [ $v = def ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$v; fi
    timeout -k 10 120 python tools/driver_region.py 25 K3 w$v= > $O/region_${v}_$r.json 2> $O/region_${v}_$r.err || { tail $O/region_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/region_${v}_$r.json')); print('K3', '$v', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
  done
done
for r in 1 2; do
  for v in def 400 2000; do
    if [ $v = def ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$v; fi
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err \
      || { echo bench failed; tail $O/bench_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); r=d['roofline']; print('driver', '$v', d['value'], d['ms_per_step'], r['kernel_avg_us'], d['image_ok'])"
  done
done
unset ROC_ACTIVE_WAIT_TIMEOUT
