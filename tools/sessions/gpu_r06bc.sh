#!/bin/bash
# Round 6: the "some |component| below 2^-100" domain checks (hit normal, normalize_w) as one
# v_min3_f32 on |.| and an ordered compare instead of three ands, an integer min3 and a
# compare: the whole GPU suite on the tree, then interleaved K3 chain and K5 A/Bs against
# the committed tree (tools/chain_ab.py, tools/k5_ab.py).
set -o pipefail
TAG=${1:-r06bc}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python tools/chain_ab.py 4 $V/librt_hip_buf.so $V/librt_hip_mn3.so > $O/chain_ab.jsonl 2> $O/chain_ab.err \
  || { echo "chain_ab failed"; tail $O/chain_ab.err; exit 1; }
tail -1 $O/chain_ab.jsonl
timeout -k 10 500 python tools/k5_ab.py 2 $V/librt_hip_buf.so $V/librt_hip_mn3.so > $O/k5_ab.jsonl 2> $O/k5_ab.err \
  || { echo "k5_ab failed"; tail $O/k5_ab.err; exit 1; }
tail -1 $O/k5_ab.jsonl
