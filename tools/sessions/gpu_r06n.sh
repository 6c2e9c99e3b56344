#!/bin/bash
# Round 6: the bounce instance on the exact fast cores (roots, normal, normalisations, sky,
# hinted accumulation) and reciprocal-steered grid walks: the whole GPU suite, then an
# interleaved K5 A/B against the previous tree's build (tools/k5_ab.py).
set -o pipefail
TAG=${1:-r06n}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python tools/k5_ab.py 3 $B/variants/librt_hip_base.so tree > $O/k5_ab.jsonl 2> $O/k5_ab.err \
  || { echo "ab failed"; tail $O/k5_ab.err; tail -3 $O/k5_ab.jsonl; exit 1; }
cat $O/k5_ab.jsonl
