#!/bin/bash
# Round 6: the last two K3 chain changes re-measured with every build through RT_HIP_LIB (the
# in-tree build had run with the CPython binding, the variants through ctypes: a bias of
# ~0.1 us per frame) and the order rotating: before the cold-branch zero colour (pzc), with
# it (zc), with the tile-pair kernel's per-frame list pointers (remat).
set -o pipefail
TAG=${1:-r06ae}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1200 python tools/chain_ab.py 6 $V/librt_hip_pzc.so $V/librt_hip_zc.so $V/librt_hip_remat.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
