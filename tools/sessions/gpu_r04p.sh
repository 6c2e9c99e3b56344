#!/bin/bash
# Round 4, session p: RT_SINGLE_SKYDD (the sky's |d|^2 from where the direction was made):
# the -m gpu suite on it, and an interleaved K3 A/B against the in-tree build at bench.py's
# default length and in the driver's 20-step command.
# Usage: bash tools/sessions/gpu_r04p.sh TAG
set -o pipefail
TAG=${1:-r04p}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_skydd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu_skydd.log 2>&1 \
  || { tail -20 $O/pytest_gpu_skydd.log; exit 1; }
tail -2 $O/pytest_gpu_skydd.log
bash tools/gpu_ab_bench.sh ${TAG}_ab "K3" 3 default $V/librt_hip_skydd.so || exit 1
for r in 1 2 3; do
  for lib in default skydd; do
    E=""; [ $lib != default ] && E="RT_HIP_LIB=$V/librt_hip_$lib.so"
    env $E timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      > $O/driver_${lib}_$r.json 2>> $O/driver.err || { echo bench failed; tail -5 $O/driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/driver_${lib}_$r.json')); print('driver $lib r$r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['image_ok'])"
  done
done
