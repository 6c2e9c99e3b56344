#!/bin/bash
# Round 5, session h: frame-group kernels (the rank shares' frame chains) — the all-f32 lens
# normalisation without the workgroup's LDS table and barrier (disk3: -DRT_TRACE_DISK=3), and
# each frame traced by the one-frame kernel's sample (gsingle: + -DRT_GROUP_SINGLE=1), against
# the committed build (base): the GPU suite on gsingle, then rank 0's K3 chain share at
# 8 / 4 / 2 / 1 ranks (tools/share_region.py), the variants interleaved per rank count, twice.
# Usage: bash tools/sessions/gpu_r05h.sh TAG
set -o pipefail
TAG=${1:-r05h}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_gsingle.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu_gsingle.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu_gsingle.log; exit 1; }
tail -2 $O/pytest_gpu_gsingle.log
for r in 1 2; do
  for n in 8 4 2 1; do
    for lib in base disk3 gsingle; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/share_region.py $n 0 15 20 \
        > $O/share_${lib}_n${n}_$r.json 2> $O/share_${lib}_n${n}_$r.err || { tail $O/share_${lib}_n${n}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/share_${lib}_n${n}_$r.json')); print('$lib', 'n$n', d['kernel'], 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
  done
done
timeout -k 10 60 gpu-ray-tracing_amd/build/launch_cost > $O/launch_cost.jsonl 2>&1 || { cat $O/launch_cost.jsonl; exit 1; }
cat $O/launch_cost.jsonl
