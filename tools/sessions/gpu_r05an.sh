#!/bin/bash
# Round 5: the grid walk loads an item's sphere index only for a root that can win
# (RT_GRID_LAZY_INDEX, tree) against one index load per tested item (variant eager): the GPU
# suite on the tree, K5 update / fused-frame times (tools/ab_variants.py k5, builds
# alternating) and the whole-image 64-spp K5 step (tools/k5_ab.py, world 1).
# Usage: bash tools/sessions/gpu_r05an.sh TAG
set -o pipefail
TAG=${1:-r05an}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
TREE=gpu-ray-tracing_amd/build/librt_hip.so
EAGER=gpu-ray-tracing_amd/build/variants/librt_hip_eager.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python tools/ab_variants.py k5 4 $TREE $EAGER > $O/ab_k5.log 2>&1 \
  || { echo "ab failed"; tail $O/ab_k5.log; exit 1; }
tail -2 $O/ab_k5.log
for r in 1 2; do
  for v in tree eager; do
    L=$TREE; [ $v = eager ] && L=$EAGER
    RT_HIP_LIB=$L timeout -k 10 300 python tools/k5_ab.py 5 1 auto > $O/k5whole_${v}_$r.jsonl 2> $O/k5whole_${v}_$r.err \
      || { echo "k5_ab failed"; tail $O/k5whole_${v}_$r.err; exit 1; }
    python -c "import json; [print('$v', d['world'], d['median_us'], d['min_us']) for d in map(json.loads, open('$O/k5whole_${v}_$r.jsonl'))]"
  done
done
