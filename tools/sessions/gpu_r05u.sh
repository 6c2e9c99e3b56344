#!/bin/bash
# Round 5, session u: the scan's 1 / |d|^2 computed only where a wave has candidates (lazy:
# the tree, librt_hip_lazy.so) against computing it for every wave (librt_hip_base.so, the
# committed build): the GPU suite on the tree, the driver's region (K3, K2), three
# interleaved rounds, both through ctypes.
# Usage: bash tools/sessions/gpu_r05u.sh TAG
set -o pipefail
TAG=${1:-r05u}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
  for lib in base lazy; do
    for cfg in K3 K2; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/driver_region.py 25 $cfg $lib= \
        > $O/region_${cfg}_${lib}_$r.json 2> $O/region_${cfg}_${lib}_$r.err || { tail $O/region_${cfg}_${lib}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/region_${cfg}_${lib}_$r.json')); print('$cfg', '$lib', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
  done
done
