#!/bin/bash
# Round 5: the tile-pair instances with a lighter fallback for foreign counts (each tile's
# pixels traced with their own counts by the one-frame kernel's one-tile pending path:
# 63 VGPRs, 8 waves per SIMD, no scratch — variants fb7 (register plan for 7 waves) and fb1
# (for 8)) against the tree (trace_pixel fallback, 71 VGPRs, 7 waves): the frame-group parity
# tests under fb7, then tools/pairs_ab.py per build (on = the unchanged one-tile groups as the
# in-process reference, on2 = tile pairs) at the whole image and 2- / 4-rank shares.
# Usage: bash tools/sessions/gpu_r05al.sh TAG
set -o pipefail
TAG=${1:-r05al}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_fb7.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "foreign_counts or equals_chained or k4 or frame" > $O/pytest_fb7.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_fb7.log; exit 1; }
tail -1 $O/pytest_fb7.log
for r in 1 2; do
  for L in tree fb7 fb1; do
    LIB=gpu-ray-tracing_amd/build/librt_hip.so; [ $L != tree ] && LIB=$V/librt_hip_$L.so
    RT_HIP_LIB=$LIB timeout -k 10 300 python tools/pairs_ab.py 9 1,2,4 on,on2 20 every > $O/pairs_${L}_$r.jsonl 2> $O/pairs_${L}_$r.err \
      || { echo "pairs_ab failed"; tail $O/pairs_${L}_$r.err; exit 1; }
    RT_HIP_LIB=$LIB timeout -k 10 300 python tools/pairs_ab.py 7 1 on,on2 64 last_two >> $O/pairs_${L}_$r.jsonl 2>> $O/pairs_${L}_$r.err \
      || { echo "pairs_ab failed"; tail $O/pairs_${L}_$r.err; exit 1; }
    python -c "
import json
for d in map(json.loads, open('$O/pairs_${L}_$r.jsonl')): print('$L', d['world'], d['frames'], d['mode'], d['us_per_frame_q1_med_q3'][1])"
  done
done
