#!/bin/bash
# (run inside tools/sessions/gpu_r05m.sh's call, whose output holds its lines)
# Round 5, session n: the general path's sky with |d| and its reciprocal from one rsq (sky:
# this tree, librt_hip_sky.so) and frame groups tracing each frame with the one-frame kernel's
# sample and scalar record loads (librt_hip_gs0.so: -DRT_GROUP_SINGLE=1 -DRT_SINGLE_LDS=0)
# against the build before them (librt_hip_cur.so), all through ctypes: the GPU suite on this
# tree, the frame-group parity cases on gs0, then the K3 chain shares at 8 / 4 / 1 ranks,
# two interleaved rounds.
# Usage: bash tools/sessions/gpu_r05n.sh TAG
set -o pipefail
TAG=${1:-r05n}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
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
