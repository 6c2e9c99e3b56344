#!/bin/bash
# Round 4, session b2: two-wave workgroups for the one-frame kernel (RT_SINGLE_WG=2): the
# -m gpu suite on it, and the driver's 20-step command against the in-tree build, four
# interleaved rounds.
# Usage: bash tools/sessions/gpu_r04b2.sh TAG
set -o pipefail
TAG=${1:-r04b2}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_wg2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu_wg2.log 2>&1 \
  || { tail -20 $O/pytest_gpu_wg2.log; exit 1; }
tail -2 $O/pytest_gpu_wg2.log
for r in 1 2 3 4; do
  for lib in default wg2; do
    E=""; [ $lib != default ] && E="RT_HIP_LIB=$V/librt_hip_$lib.so"
    env $E timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      > $O/driver_${lib}_$r.json 2>> $O/driver.err || { echo bench failed; tail -5 $O/driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/driver_${lib}_$r.json')); print('driver $lib r$r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['image_ok'])"
  done
done
