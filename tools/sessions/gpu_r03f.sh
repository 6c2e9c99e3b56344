#!/bin/bash
# Round-3 session f: parity of the bounce-instance candidates, A/B of the bounce
# instance's SGPR plan (K5 and its 8-rank share), the fused trace kernel's disk reciprocal
# (K4), the in-wave seed hash and the one-tile LDS block on rank shares.
# Usage: bash tools/gpu_r03f.sh TAG
set -o pipefail
TAG=${1:-r03f}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 120 ./tools/launch_rate > $O/launch_rate.jsonl 2>&1 || { echo launch_rate failed; cat $O/launch_rate.jsonl; exit 1; }
cat $O/launch_rate.jsonl
for v in breload8 hash3; do
  RT_HIP_LIB=$V/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q \
    --timeout 200 --timeout-method thread > $O/pytest_gpu_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -2 $O/pytest_gpu_$v.log; [ $rc -eq 0 ] || exit 1
done
bash tools/gpu_ab_bench.sh $TAG/ab "K5" 2 default $V/librt_hip_breload.so $V/librt_hip_breload7.so \
  $V/librt_hip_breload8.so $V/librt_hip_bmw7.so || exit 1
for v in default breload7 breload8; do
  E=""; [ $v != default ] && E="RT_HIP_LIB=$V/librt_hip_$v.so"
  env $E timeout -k 10 300 python tools/rank_sim.py K5 64 > $O/rank_k5_$v.jsonl 2>&1 || exit 1
  echo k5 $v; grep '^{' $O/rank_k5_$v.jsonl
done
bash tools/gpu_ab_bench.sh $TAG/ab "K4" 3 default $V/librt_hip_trdisk2.so || exit 1
for v in hash1 hash3 slds0; do
  RT_HIP_LIB=$V/librt_hip_$v.so RT_QUEUES=1 RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 \
    > $O/rank_k3_$v.jsonl 2>&1 || exit 1
  echo k3 $v; grep '^{' $O/rank_k3_$v.jsonl
done
