#!/bin/bash
# Round 5, session r: the exact fast paths' domain checks marked likely (librt_hip_likely.so,
# -DRT_LIKELY_FAST=1: the fast path laid out as the fall-through, the IEEE fallback as the
# taken branch) against the tree's build (librt_hip_cur.so), both through ctypes: the GPU
# parity cases on the variant, then the driver's region (K3, K2) and the 8-rank chain share,
# three interleaved rounds.
# Usage: bash tools/sessions/gpu_r05r.sh TAG
set -o pipefail
TAG=${1:-r05r}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_likely.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu_likely.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu_likely.log; exit 1; }
tail -1 $O/pytest_gpu_likely.log
for r in 1 2 3; do
  for lib in cur likely; do
    for cfg in K3 K2; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/driver_region.py 25 $cfg $lib= \
        > $O/region_${cfg}_${lib}_$r.json 2> $O/region_${cfg}_${lib}_$r.err || { tail $O/region_${cfg}_${lib}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/region_${cfg}_${lib}_$r.json')); print('$cfg', '$lib', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
    RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/share_region.py 8 0 15 20 > $O/share_${lib}_n8_$r.json 2> $O/share_${lib}_n8_$r.err || { tail $O/share_${lib}_n8_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/share_${lib}_n8_$r.json')); print('$lib', 'n8', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
  done
done
