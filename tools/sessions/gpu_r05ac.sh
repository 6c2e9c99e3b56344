#!/bin/bash
# Round 5: the sphere grid's density, second pass (after r05ab) — RT_GRID_PER_CELL 0.5 /
# 0.75 / 1 / 2 (tree), RT_GRID_REACHES 3, and 1 with 3: K5 update / fused-frame times
# (tools/ab_variants.py, builds alternating) and the 8-rank K5 share (tools/k5_ab.py, mode
# auto, 9 launches per measurement).
# Usage: bash tools/sessions/gpu_r05ac.sh TAG
set -o pipefail
TAG=${1:-r05ac}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
LIBS="gpu-ray-tracing_amd/build/librt_hip.so $V/librt_hip_pc1.so $V/librt_hip_pc075.so $V/librt_hip_pc05.so $V/librt_hip_r3.so $V/librt_hip_pc1r3.so"
timeout -k 10 600 python tools/ab_variants.py k5 3 $LIBS > $O/ab_k5.log 2>&1 \
  || { echo "ab failed"; tail $O/ab_k5.log; exit 1; }
tail -6 $O/ab_k5.log
for r in 1 2; do
  for L in $LIBS; do
    n=$(basename $L .so)
    RT_HIP_LIB=$L timeout -k 10 300 python tools/k5_ab.py 9 8 auto > $O/k5share_${n}_$r.jsonl 2> $O/k5share_${n}_$r.err \
      || { echo "k5_ab failed"; tail $O/k5share_${n}_$r.err; exit 1; }
    python -c "import json; [print('$n', d['world'], d['median_us'], d['min_us']) for d in map(json.loads, open('$O/k5share_${n}_$r.jsonl'))]"
  done
done
