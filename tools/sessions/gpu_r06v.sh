#!/bin/bash
# Round 6: the K5 step's bounce work by region (tools/bounce_counts.py on an
# RT_BOUNCE_COUNTS=1 build): whole image and rank 0's 8-rank share.
set -o pipefail
TAG=${1:-r06v}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
export RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_bc.so
timeout -k 10 300 python tools/bounce_counts.py 1 > $O/counts_n1.json 2> $O/counts.err \
  || { echo "n1 failed"; tail $O/counts.err; exit 1; }
timeout -k 10 300 python tools/bounce_counts.py 8 > $O/counts_n8.json 2>> $O/counts.err \
  || { echo "n8 failed"; tail $O/counts.err; exit 1; }
cat $O/counts_n1.json $O/counts_n8.json
