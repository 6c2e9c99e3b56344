#!/bin/bash
# Round 4, session d2: with 2-wave one-frame workgroups (the default since b2), one-wave
# workgroups (RT_SINGLE_WG=1) and 1 / 3 concurrent parts per update (RT_QUEUES) against the
# in-tree build, in the driver's 20-step command, three interleaved rounds.
# Usage: bash tools/sessions/gpu_r04d2.sh TAG
set -o pipefail
TAG=${1:-r04d2}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
for r in 1 2 3; do
  for spec in default wg1 q1 q3; do
    case $spec in
      default) E="";; wg1) E="RT_HIP_LIB=$V/librt_hip_wg1.so";;
      q1) E="RT_QUEUES=1";; q3) E="RT_QUEUES=3";;
    esac
    env $E timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
      > $O/driver_${spec}_$r.json 2>> $O/driver.err || { echo bench failed; tail -5 $O/driver.err; exit 1; }
    python -c "import json; d=json.load(open('$O/driver_${spec}_$r.json')); print('driver $spec r$r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['image_ok'])"
  done
done
