#!/bin/bash
# Round 6: wave timelines of K5's 64-frame bounce launch on 2/4/8-rank shares with the faster
# bounce kernel (tools/wave_trace.py on an RT_WAVE_TRACE=1 build): AUTO (split unit order) and
# per wave — the tail against the per-SIMD balance.
set -o pipefail
TAG=${1:-r06s}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
export RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_wt.so
RT_PATHS=auto timeout -k 10 300 python tools/wave_trace.py K5 > $O/wt_auto.jsonl 2> $O/wt_auto.err \
  || { echo "auto failed"; tail $O/wt_auto.err; exit 1; }
RT_PATHS=per_wave timeout -k 10 300 python tools/wave_trace.py K5 > $O/wt_per_wave.jsonl 2> $O/wt_per_wave.err \
  || { echo "per_wave failed"; tail $O/wt_per_wave.err; exit 1; }
cat $O/wt_auto.jsonl $O/wt_per_wave.jsonl
