#!/bin/bash
# Round-3 first session: -m gpu tests (incl. the C-ABI RCCL gather), VALU issue rates of the
# remaining forms, per-phase stamps of the one-frame kernel (whole image and rank shares),
# the driver's bench command, PMC with the VALU instruction classes (K3, K2), per-rank
# prediction.  Usage: bash tools/gpu_r03a.sh TAG
set -o pipefail
TAG=${1:-r03a}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/valu_rates > $O/valu_rates.txt 2>&1 || { echo valu_rates failed; tail $O/valu_rates.txt; exit 1; }
tail -21 $O/valu_rates.txt
for c in K3 K2; do
  RT_HIP_LIB=gpu-ray-tracing_amd/build/variants/librt_hip_sst.so timeout -k 10 200 \
    python tools/stamps_single.py $c 1,2,4,8,135 > $O/stamps_$c.jsonl 2>&1 \
    || { echo "stamps $c failed"; tail $O/stamps_$c.jsonl; exit 1; }
  grep '^{' $O/stamps_$c.jsonl | cut -c1-400
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench.err \
  || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['image_ok'], d['candidate_lists'])"
bash tools/pmc_bench.sh $TAG "K3 K2" || exit 1
RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_dispatch.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k3_dispatch.jsonl
# A/B of the one-frame kernel variants (bench.py lines, interleaved) and their rank shares
V=gpu-ray-tracing_amd/build/variants
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 3 default $V/librt_hip_disk2.so $V/librt_hip_sinbits.so \
  $V/librt_hip_snake256.so $V/librt_hip_wg8.so $V/librt_hip_combo.so $V/librt_hip_combowg8.so || exit 1
for v in disk2 snake256 combo wg8; do
  RT_HIP_LIB=$V/librt_hip_$v.so RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 \
    > $O/rank_k3_dispatch_$v.jsonl 2>&1 || exit 1
  echo $v; grep '^{' $O/rank_k3_dispatch_$v.jsonl
done
