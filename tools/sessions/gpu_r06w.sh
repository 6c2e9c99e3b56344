#!/bin/bash
# Round 6: far bounce rays that miss every small sphere share the grid walk (grid_usable):
# the bounce / grid / K5 parity tests, the region counters, and a K5 A/B against the tree
# before (pre), and the grid at 0.5 / 0.7 / 2 small spheres per cell (pc05, pc07, pc2).
set -o pipefail
TAG=${1:-r06w}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "fallbacks or bounce or k5 or grid or culled" > $O/pytest_sel.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_sel.log; exit 1; }
tail -1 $O/pytest_sel.log
RT_HIP_LIB=$V/librt_hip_bc.so timeout -k 10 300 python tools/bounce_counts.py 1 > $O/counts_n1.json 2> $O/counts.err \
  || { echo "counts failed"; tail $O/counts.err; exit 1; }
timeout -k 10 600 python tools/k5_ab.py 3 $V/librt_hip_pre.so tree $V/librt_hip_pc05.so $V/librt_hip_pc07.so $V/librt_hip_pc2.so > $O/k5_ab.jsonl 2> $O/k5_ab.err \
  || { echo "ab failed"; tail $O/k5_ab.err; exit 1; }
tail -1 $O/k5_ab.jsonl
