#!/bin/bash
# Round 6: the last two K3 chain changes re-measured with the build order rotating round by
# round (tools/chain_ab.py now does; the fixed order favoured the second build by up to 2 %,
# r06ac/chain_ab_same_build.jsonl): before the cold-branch zero colour (pzc), with it (zc),
# and with the tile-pair kernel's per-frame list pointers (the tree).
set -o pipefail
TAG=${1:-r06ad}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1200 python tools/chain_ab.py 6 $V/librt_hip_pzc.so $V/librt_hip_zc.so tree > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
