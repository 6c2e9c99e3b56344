#!/bin/bash
# Round 6: wave timelines of the K3 frame chains (tools/wave_trace.py K3 on the RT_WAVE_TRACE
# build): the whole image's tile-pair launch and the 2/4/8-rank shares — resident waves per
# SIMD, SIMD finishing times, wave durations.
set -o pipefail
TAG=${1:-r06u}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
export RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_wt.so
timeout -k 10 300 python tools/wave_trace.py K3 > $O/wt_k3.jsonl 2> $O/wt_k3.err \
  || { echo "k3 failed"; tail $O/wt_k3.err; exit 1; }
cat $O/wt_k3.jsonl
