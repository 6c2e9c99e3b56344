#!/bin/bash
# Round 5: frame groups over tile PAIRS (rt_tpair_kernel<2 / 4>, RT_TPAIR=1: two pixels per
# lane, the one-frame kernel's joint list walk) against the one-tile frame groups, on whole-
# image fused launches (one GPU, one process): the GPU suite under RT_TPAIR=1 (parity of every
# frame-group case; tests that assert the instance name are expected to differ), the 64-frame
# fused launch per frame (tools/ab_variants.py k3: tree, tree + RT_TPAIR=1, variant tp7 =
# 7 waves per SIMD without scratch), and bench.py --config K4 with and without RT_TPAIR.
# Usage: bash tools/sessions/gpu_r05af.sh TAG
set -o pipefail
TAG=${1:-r05af}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
RT_TPAIR=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu_tpair.log 2>&1; rc=$?
tail -1 $O/pytest_gpu_tpair.log; grep -E "^FAILED" $O/pytest_gpu_tpair.log | head -40
[ $rc -le 1 ] || { echo "pytest rc $rc"; exit 1; }
TREE=gpu-ray-tracing_amd/build/librt_hip.so
TP7=gpu-ray-tracing_amd/build/variants/librt_hip_tp7.so
timeout -k 10 600 python tools/ab_variants.py k3 4 $TREE:RT_TPAIR=0 $TREE:RT_TPAIR=1 $TP7:RT_TPAIR=1 > $O/ab_k3_fused.log 2>&1 \
  || { echo "ab failed"; tail $O/ab_k3_fused.log; exit 1; }
tail -3 $O/ab_k3_fused.log
for r in 1 2; do
  for t in 0 1; do
    RT_TPAIR=$t timeout -k 10 300 python bench.py --config K4 --cpu-seconds 0 > $O/bench_k4_tpair${t}_$r.json 2> $O/bench_k4_tpair${t}_$r.err \
      || { echo "bench failed"; tail $O/bench_k4_tpair${t}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_k4_tpair${t}_$r.json')); print('K4 tpair=$t', d['value'], d['ms_per_step'], d.get('image_ok'), d['roofline'].get('kernel'))"
  done
done
