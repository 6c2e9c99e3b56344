#!/bin/bash
# Round-3 session e: -m gpu suite (incl. concurrent update parts), then A/B of one-frame
# updates as 1-4 concurrent parts (rt_set_update_queues) on K3 / K2 and their rank shares,
# and of the one-frame kernel's instruction-level switches (seed hash in the wave, the
# bit-compare count check, VGPR-resident camera constants, 8-wave plan).
# Usage: bash tools/gpu_r03e.sh TAG
set -o pipefail
TAG=${1:-r03e}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_bench.sh $TAG/abq "K3 K2" 3 default:RT_QUEUES=1 default:RT_QUEUES=2 \
  default:RT_QUEUES=3 default:RT_QUEUES=4 || exit 1
for q in 1 2 3; do
  RT_QUEUES=$q RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 100 > $O/rank_k3_q$q.jsonl 2>&1 || exit 1
  echo k3 q$q; grep '^{' $O/rank_k3_q$q.jsonl
done
bash tools/gpu_ab_bench.sh $TAG/ab "K3 K2" 2 default:RT_QUEUES=1 $V/librt_hip_hash3.so:RT_QUEUES=1 \
  $V/librt_hip_nchk.so:RT_QUEUES=1 $V/librt_hip_vconst.so:RT_QUEUES=1 $V/librt_hip_mw8.so:RT_QUEUES=1 || exit 1
