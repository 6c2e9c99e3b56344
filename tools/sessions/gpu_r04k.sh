#!/bin/bash
# Round 4, session k: the whole -m gpu suite on the in-tree build (partial split schedule)
# and on the all4 variant (RT_SINGLE_UNIF + RT_SINGLE_AND + RT_SKY_RSQ + RT_SINGLE_CHUNK=1),
# an interleaved K3 A/B of the one-frame-kernel variants, and the K5 split-fraction A/B
# (tools/k5_ab.py at 1, 4 and 8 ranks).
# Usage: bash tools/sessions/gpu_r04k.sh TAG
set -o pipefail
TAG=${1:-r04k}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
RT_HIP_LIB=$V/librt_hip_all4.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu_all4.log 2>&1 \
  || { tail -20 $O/pytest_gpu_all4.log; exit 1; }
tail -2 $O/pytest_gpu_all4.log
bash tools/gpu_ab_bench.sh ${TAG}_ab "K3" 3 default $V/librt_hip_unif.so $V/librt_hip_and.so \
  $V/librt_hip_all4.so $V/librt_hip_unifsky.so $V/librt_hip_lds2.so $V/librt_hip_gate.so || exit 1
timeout -k 10 400 python tools/k5_ab.py 7 1,4,8 \
  per_wave,split2,split2f50,split2f25,split2f12,split4f25,split4f12,split3f25 > $O/k5_ab.jsonl \
  || { echo k5_ab failed; exit 1; }
cat $O/k5_ab.jsonl | python -c "import json,sys; [print(' ', d['world'], d['mode'], d['median_us'], d['min_us']) for d in map(json.loads, sys.stdin)]"
