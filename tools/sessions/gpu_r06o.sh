#!/bin/bash
# Round 6: the bounce instance with the scatter random numbers from a device table
# (hint_rs_dev, build hr) and the dielectric / cone roots on the fast cores (the tree): the
# whole GPU suite, then a K5 A/B against the fast-core build (fc) and
# the build before it (base).
set -o pipefail
TAG=${1:-r06o}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python tools/k5_ab.py 3 $B/variants/librt_hip_base.so $B/variants/librt_hip_fc.so $B/variants/librt_hip_hr.so tree > $O/k5_ab.jsonl 2> $O/k5_ab.err \
  || { echo "ab failed"; tail $O/k5_ab.err; tail -3 $O/k5_ab.jsonl; exit 1; }
cat $O/k5_ab.jsonl
