#!/bin/bash
# Round 4, session l: the split schedule's unit order (longest-processing-time-first over
# the units, tiles above alpha x the launch's ideal span split) and the one-frame kernel's new
# defaults (RT_SINGLE_UNIF, RT_SINGLE_AND, RT_SKY_RSQ, RT_SINGLE_CHUNK=1): the whole -m gpu
# suite on the in-tree build and on diellds (RT_SINGLE_DIEL + RT_SINGLE_LDS_HIT), the K5 A/B
# of alpha at 1, 4 and 8 ranks (tools/k5_ab.py), the K3 A/B of and0 / diel / ldshit / diellds
# and spref (RT_SINGLE_SPREF; the suite also runs on it) against the defaults, the host cost per call (tools/host_call.py, with bind_update_frames).
# Usage: bash tools/sessions/gpu_r04l.sh TAG
set -o pipefail
TAG=${1:-r04l}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
RT_HIP_LIB=$V/librt_hip_diellds.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu_diellds.log 2>&1 \
  || { tail -20 $O/pytest_gpu_diellds.log; exit 1; }
tail -2 $O/pytest_gpu_diellds.log
RT_HIP_LIB=$V/librt_hip_spref.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu_spref.log 2>&1 \
  || { tail -20 $O/pytest_gpu_spref.log; exit 1; }
tail -2 $O/pytest_gpu_spref.log
timeout -k 10 400 python tools/k5_ab.py 7 1,4,8 \
  per_wave,split2f100,split2a12,split2a25,split2a50,split2a100,split4a25 > $O/k5_ab.jsonl \
  || { echo k5_ab failed; exit 1; }
cat $O/k5_ab.jsonl | python -c "import json,sys; [print(' ', d['world'], d['mode'], d['median_us'], d['min_us']) for d in map(json.loads, sys.stdin)]"
bash tools/gpu_ab_bench.sh ${TAG}_ab "K3" 3 default $V/librt_hip_and0.so $V/librt_hip_diel.so \
  $V/librt_hip_ldshit.so $V/librt_hip_diellds.so $V/librt_hip_spref.so || exit 1
timeout -k 10 120 python tools/host_call.py 20 > $O/host_call.jsonl || { echo host_call failed; exit 1; }
cat $O/host_call.jsonl
