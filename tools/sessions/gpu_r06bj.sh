#!/bin/bash
# Round 6: the split frame-group accumulation at 2 and 4 ranks, processes alternating
# head / split twice (tools/pairs_ab.py, rank 0's K3 share, 20-frame calls, AUTO's modes).
set -o pipefail
TAG=${1:-r06bj}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
for R in 1 2; do for L in head split; do
  RT_HIP_LIB=$V/librt_hip_$L.so timeout -k 10 300 python tools/pairs_ab.py 9 2,4 on2,quad2 20 every > $O/modes_${L}_$R.jsonl 2> $O/modes_${L}_$R.err \
    || { echo "pairs_ab failed"; tail $O/modes_${L}_$R.err; exit 1; }
  sed "s/^/$L$R /" $O/modes_${L}_$R.jsonl | cut -c1-170
done; done
