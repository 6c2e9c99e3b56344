#!/bin/bash
# Round-3 session zb: the AQL tests with per-part queues created on first use, and the
# per-phase stamps of the one-frame kernel at warm clocks (whole image, 8-rank share, one
# band; cold for comparison).  Usage: bash tools/gpu_r03zb.sh TAG
set -o pipefail
TAG=${1:-r03zb}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "submit or queues or dispatch_chain" > $O/pytest_aql.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_aql.log; [ $rc -eq 0 ] || exit 1
RT_HIP_LIB=$V/librt_hip_sst.so timeout -k 10 300 python tools/stamps_single.py K3 1,8,135 \
  > $O/stamps_K3_warm.jsonl 2>&1 || { echo "stamps failed"; tail $O/stamps_K3_warm.jsonl; exit 1; }
grep '^{' $O/stamps_K3_warm.jsonl | cut -c1-330
RT_WARM_MS=0 RT_HIP_LIB=$V/librt_hip_sst.so timeout -k 10 300 python tools/stamps_single.py K3 1,8,135 \
  > $O/stamps_K3_cold.jsonl 2>&1 || { echo "stamps failed"; tail $O/stamps_K3_cold.jsonl; exit 1; }
grep '^{' $O/stamps_K3_cold.jsonl | cut -c1-330
