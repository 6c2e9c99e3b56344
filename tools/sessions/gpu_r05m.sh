#!/bin/bash
# Round 5, session m: the host's wait for the GPU — HSA signal waits polled
# (HSA_ENABLE_INTERRUPT=0, set for the process before the runtime starts) against the default
# interrupt-driven wait: the driver's K3 region and the 8-rank chain share, separate
# processes, three interleaved rounds; then the driver's command with each, twice.
# Usage: bash tools/sessions/gpu_r05m.sh TAG
set -o pipefail
TAG=${1:-r05m}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in irq poll; do
    if [ $v = poll ]; then export HSA_ENABLE_INTERRUPT=0; else unset HSA_ENABLE_INTERRUPT; fi
    timeout -k 10 120 python tools/driver_region.py 25 K3 $v= > $O/region_${v}_$r.json 2> $O/region_${v}_$r.err || { tail $O/region_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/region_${v}_$r.json')); print('K3', '$v', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    timeout -k 10 120 python tools/share_region.py 8 0 15 20 > $O/share_${v}_n8_$r.json 2> $O/share_${v}_n8_$r.err || { tail $O/share_${v}_n8_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/share_${v}_n8_$r.json')); print('n8', '$v', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
  done
done
for r in 1 2; do
  for v in irq poll; do
    if [ $v = poll ]; then export HSA_ENABLE_INTERRUPT=0; else unset HSA_ENABLE_INTERRUPT; fi
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err \
      || { echo bench failed; tail $O/bench_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); r=d['roofline']; print('driver', '$v', d['value'], d['ms_per_step'], r['kernel_avg_us'], d['image_ok'])"
  done
done
unset HSA_ENABLE_INTERRUPT
# --- session n (tools/sessions/gpu_r05n.sh) in the same call ---
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
RT_HIP_LIB=$V/librt_hip_gs0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "chain or pair or share or frames or normal" > $O/pytest_gpu_gs0.log 2>&1 || { echo "pytest gs0 failed"; tail -30 $O/pytest_gpu_gs0.log; exit 1; }
tail -1 $O/pytest_gpu_gs0.log
for r in 1 2; do
  for n in 8 4 1; do
    for lib in cur gs0 sky; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/share_region.py $n 0 15 20 > $O/share_${lib}_n${n}_$r.json 2> $O/share_${lib}_n${n}_$r.err || { tail $O/share_${lib}_n${n}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/share_${lib}_n${n}_$r.json')); print('$lib', 'n$n', d['kernel'], 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
  done
done
