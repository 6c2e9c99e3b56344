#!/bin/bash
# Round 4, session q: RT_SINGLE_FRONT (face-flip selects only in waves with a back-face hit)
# and RT_SINCOS_FIN (no NaN guard on the lens sample's quadrant): the -m gpu suite on both
# together (ff), an interleaved K3 A/B of front / fin / ff against the in-tree build at the
# default length, and ff against the in-tree build in the driver's 20-step command.
# Usage: bash tools/sessions/gpu_r04q.sh TAG
set -o pipefail
TAG=${1:-r04q}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_ff.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu_ff.log 2>&1 \
  || { tail -20 $O/pytest_gpu_ff.log; exit 1; }
tail -2 $O/pytest_gpu_ff.log
bash tools/gpu_ab_bench.sh ${TAG}_ab "K3" 3 default $V/librt_hip_front.so $V/librt_hip_fin.so \
  $V/librt_hip_ff.so || exit 1
for r in 1 2 3; do
  for lib in default ff; do
    E=""; [ $lib != default ] && E="RT_HIP_LIB=$V/librt_hip_$lib.so"
    env $E timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      > $O/driver_${lib}_$r.json 2>> $O/driver.err || { echo bench failed; tail -5 $O/driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/driver_${lib}_$r.json')); print('driver $lib r$r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['image_ok'])"
  done
done
