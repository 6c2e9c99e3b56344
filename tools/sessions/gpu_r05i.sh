#!/bin/bash
# Round 5, session i: the compiler's SLP vectorizer (packed f32 arithmetic, v_pk_fma/mul/add
# over the two pixel slots) on — the `slp` build (-fslp-vectorize) against the committed
# build: the GPU suite on slp, then the driver's region (K3, K2) and the K3 chain shares at
# 8 ranks and 1, separate processes, three interleaved rounds.
# Usage: bash tools/sessions/gpu_r05i.sh TAG
set -o pipefail
TAG=${1:-r05i}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_slp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu_slp.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu_slp.log; exit 1; }
tail -2 $O/pytest_gpu_slp.log
for r in 1 2 3; do
  for lib in base slp; do
    for cfg in K3 K2; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/driver_region.py 25 $cfg $lib= \
        > $O/region_${cfg}_${lib}_$r.json 2> $O/region_${cfg}_${lib}_$r.err || { tail $O/region_${cfg}_${lib}_$r.err; exit 1; }
      cat $O/region_${cfg}_${lib}_$r.json
    done
    for n in 8 1; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/share_region.py $n 0 15 20 \
        > $O/share_${lib}_n${n}_$r.json 2> $O/share_${lib}_n${n}_$r.err || { tail $O/share_${lib}_n${n}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/share_${lib}_n${n}_$r.json')); print('$lib', 'n$n', d['kernel'], 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
  done
done
