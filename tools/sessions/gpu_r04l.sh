#!/bin/bash
# Round 4, session l: the split schedule's unit order (longest-processing-time-first over
# the units, tiles above alpha x the launch's ideal span split): the whole -m gpu suite,
# the K5 A/B of alpha at 1, 4 and 8 ranks (tools/k5_ab.py), and the K3 A/B of the
# one-frame-kernel variants all3 / all4 / all5, the host cost per call (tools/host_call.py, with
# the bound call of bind_update_frames) (all3 + RT_SINGLE_DIEL; the suite also
# runs on all5).
# Usage: bash tools/sessions/gpu_r04l.sh TAG
set -o pipefail
TAG=${1:-r04l}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
RT_HIP_LIB=$V/librt_hip_all5.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu_all5.log 2>&1 \
  || { tail -20 $O/pytest_gpu_all5.log; exit 1; }
tail -2 $O/pytest_gpu_all5.log
timeout -k 10 400 python tools/k5_ab.py 7 1,4,8 \
  per_wave,split2f100,split2a12,split2a25,split2a50,split2a100,split4a25 > $O/k5_ab.jsonl \
  || { echo k5_ab failed; exit 1; }
cat $O/k5_ab.jsonl | python -c "import json,sys; [print(' ', d['world'], d['mode'], d['median_us'], d['min_us']) for d in map(json.loads, sys.stdin)]"
bash tools/gpu_ab_bench.sh ${TAG}_ab "K3" 3 default $V/librt_hip_all3.so $V/librt_hip_all4.so \
  $V/librt_hip_all5.so $V/librt_hip_ldshit.so $V/librt_hip_all6.so || exit 1
timeout -k 10 120 python tools/host_call.py 20 > $O/host_call.jsonl || { echo host_call failed; exit 1; }
cat $O/host_call.jsonl
