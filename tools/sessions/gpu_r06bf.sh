#!/bin/bash
# Round 6: the list-only trace instances (the 8-rank share's rt_trace_kernel<4>) walking the
# per-tile candidate lists one record per step (RT_LIST_CHUNK=1) instead of two: interleaved
# K3 chain A/B against the final tree (tools/chain_ab.py; world 8 runs the share kernel).
set -o pipefail
TAG=${1:-r06bf}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 400 python tools/chain_ab.py 4 $V/librt_hip_base3.so $V/librt_hip_lc1.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
