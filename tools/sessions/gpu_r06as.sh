#!/bin/bash
# Wave timelines of the K3 20-frame chain launch (bench.py's timed launch) at 1 and 8 ranks
# (rank 0's share), every wave's start and end saved (tools/wave_trace.py, RT_WAVE_TRACE build).
set -o pipefail
TAG=${1:-r06as}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_wt.so WT_FRAMES=20 WT_WORLDS=1,8 WT_SAVE=$O/wt_k3_f20 timeout -k 10 300 python tools/wave_trace.py K3 \
  > $O/wt_k3_f20.jsonl 2> $O/wt.err || { echo "wave_trace failed"; tail $O/wt.err; exit 1; }
cat $O/wt_k3_f20.jsonl
