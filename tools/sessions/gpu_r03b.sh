#!/bin/bash
# Round-3 session b: tests and artifacts of the new one-frame defaults (closed-form disk
# reciprocal, bit-select sincos swap), PMC + stamps of the new build, and A/B of the bounce
# instance's SGPR plan (K5), the fused trace kernel's disk table (K4) and the one-tile
# instance's LDS block (rank shares).  Usage: bash tools/gpu_r03b.sh TAG
set -o pipefail
TAG=${1:-r03b}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench.err \
  || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); print('driver', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['image_ok'])"
RT_HIP_LIB=$V/librt_hip_sst.so timeout -k 10 200 python tools/stamps_single.py K3 1,8,135 \
  > $O/stamps_K3.jsonl 2>&1 || { echo "stamps failed"; tail $O/stamps_K3.jsonl; exit 1; }
grep '^{' $O/stamps_K3.jsonl | cut -c1-300
bash tools/pmc_bench.sh $TAG "K3 K2" || exit 1
RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_dispatch.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k3_dispatch.jsonl
RT_HIP_LIB=$V/librt_hip_slds0.so RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 \
  > $O/rank_k3_dispatch_slds0.jsonl 2>&1 || exit 1
echo slds0; grep '^{' $O/rank_k3_dispatch_slds0.jsonl
bash tools/gpu_ab_bench.sh $TAG/ab "K5" 2 default $V/librt_hip_breload.so $V/librt_hip_breload7.so \
  $V/librt_hip_breload8.so $V/librt_hip_bmw7.so || exit 1
bash tools/gpu_ab_bench.sh $TAG/ab "K4" 3 default $V/librt_hip_trdisk2.so || exit 1
for v in default breload7 breload8; do
  E=""; [ $v != default ] && E="RT_HIP_LIB=$V/librt_hip_$v.so"
  env $E timeout -k 10 300 python tools/rank_sim.py K5 64 > $O/rank_k5_$v.jsonl 2>&1 || exit 1
  echo k5 $v; grep '^{' $O/rank_k5_$v.jsonl
done
