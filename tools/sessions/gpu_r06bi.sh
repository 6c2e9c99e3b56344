#!/bin/bash
# Round 6: the frame groups' accumulation split over the tile pair's waves (wave t accumulates
# tile t; every other wave leaves its colour of that tile in LDS) instead of all of it on
# wave 0: the whole GPU suite on the tree, then an interleaved K3 chain A/B against HEAD
# (tools/chain_ab.py) and the modes at 4 and 2 ranks (tools/pairs_ab.py, quad2 / on2).
set -o pipefail
TAG=${1:-r06bi}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python tools/chain_ab.py 4 $V/librt_hip_head.so $V/librt_hip_split.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
for L in head split; do
  RT_HIP_LIB=$V/librt_hip_$L.so timeout -k 10 300 python tools/pairs_ab.py 9 4,2 quad2,on2 20 every > $O/modes_$L.jsonl 2> $O/modes_$L.err \
    || { echo "pairs_ab failed"; tail $O/modes_$L.err; exit 1; }
  sed "s/^/$L /" $O/modes_$L.jsonl | cut -c1-200
done
