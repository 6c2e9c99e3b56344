#!/bin/bash
# Round 5: the sphere grid's registration pad sqrt(R^2 + m^2) (tree) against round 4's R + m
# (variant pad4, -DRT_GRID_PAD_ROUND4=1) — the GPU suite on the tree, then K5 update / fused
# 64-frame times (tools/ab_variants.py) and K5 rank shares at 1 / 4 / 8 ranks
# (tools/k5_ab.py, mode auto), the builds alternating process by process.
# Usage: bash tools/sessions/gpu_r05aa.sh TAG
set -o pipefail
TAG=${1:-r05aa}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
TREE=gpu-ray-tracing_amd/build/librt_hip.so
PAD4=gpu-ray-tracing_amd/build/variants/librt_hip_pad4.so
[ -n "$SKIP_PYTEST" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
[ -n "$SKIP_PYTEST" ] || tail -2 $O/pytest_gpu.log
timeout -k 10 400 python tools/ab_variants.py k5 4 $TREE $PAD4 > $O/ab_k5.log 2>&1 \
  || { echo "ab failed"; tail $O/ab_k5.log; exit 1; }
tail -2 $O/ab_k5.log
for r in 1 2; do
  for v in tree pad4; do
    L=$TREE; [ $v = pad4 ] && L=$PAD4
    RT_HIP_LIB=$L timeout -k 10 300 python tools/k5_ab.py 5 1,4,8 auto > $O/k5share_${v}_$r.jsonl 2> $O/k5share_${v}_$r.err \
      || { echo "k5_ab failed"; tail $O/k5share_${v}_$r.err; exit 1; }
    python -c "import json; [print('$v', d['world'], d['median_us'], d['min_us']) for d in map(json.loads, open('$O/k5share_${v}_$r.jsonl'))]"
  done
done
