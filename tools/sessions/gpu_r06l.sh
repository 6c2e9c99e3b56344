#!/bin/bash
# Round 6: register-plan A/B on the main line's structure (tools/chain_ab.py): the tree
# against 6-wave plans for the tile-pair instance (tp6: no 94-SGPR cap, 25 SGPR spills
# instead of 45) and the frame-group instances (tr6: no SGPR spills), alternating builds
# process by process; the whole image and the 8-rank share.
set -o pipefail
TAG=${1:-r06l}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build
timeout -k 10 900 python tools/chain_ab.py 4 $B/librt_hip.so $B/variants/librt_hip_tp6.so $B/variants/librt_hip_tr6.so \
  > $O/chain_ab.jsonl 2> $O/chain_ab.err || { echo "ab failed"; tail $O/chain_ab.err; tail -3 $O/chain_ab.jsonl; exit 1; }
tail -1 $O/chain_ab.jsonl
