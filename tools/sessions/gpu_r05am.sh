#!/bin/bash
# Round 5: the AMDGPU machine scheduler's strategies for the kernels (-mllvm
# -amdgpu-sched-strategy=max-ilp / iterative-ilp / max-memory-clause / iterative-minreg,
# variants ilp / iilp / mclause / iminreg; all keep 8 waves per SIMD for rt_single_kernel<2>)
# against the tree: the driver's K3 and K2 regions (tools/driver_region.py, 15 repetitions per
# process), builds alternating process by process, three rounds.
# Usage: bash tools/sessions/gpu_r05am.sh TAG
set -o pipefail
TAG=${1:-r05am}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
for r in 1 2 3; do
  for L in tree ilp iilp mclause iminreg; do
    LIB=gpu-ray-tracing_amd/build/librt_hip.so; [ $L != tree ] && LIB=$V/librt_hip_$L.so
    for C in K3 K2; do
      RT_HIP_LIB=$LIB timeout -k 10 200 python tools/driver_region.py 15 $C base= > $O/region_${L}_${C}_$r.json 2> $O/region_${L}_${C}_$r.err \
        || { echo "region failed"; tail $O/region_${L}_${C}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/region_${L}_${C}_$r.json')); print('$r $L $C wall', d['wall_us_per_step_q1_med_q3'][1], 'ev', d['events_us_per_step_q1_med_q3'][1])"
    done
  done
done
