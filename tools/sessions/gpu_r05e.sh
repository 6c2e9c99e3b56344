#!/bin/bash
# Round 5, session e: Markstein divisions (the accumulator's division by n + 1 and the
# normal's division by the radius, y = RN32(1 / b) from the host) — GPU parity suite (the
# fast-math self-test replays them), then the driver's region A/B against the previous build
# (build/variants/librt_hip_base.so, both through ctypes: RT_HIP_LIB), alternating processes,
# then the driver's command on the new build.
# Usage: bash tools/sessions/gpu_r05e.sh TAG
set -o pipefail
TAG=${1:-r05e}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
V=gpu-ray-tracing_amd/build/variants
for r in 1 2 3; do
  for lib in base mk; do
    RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/driver_region.py 15 K3 $lib= \
      > $O/region_${lib}_$r.json 2> $O/region_${lib}_$r.err || { tail $O/region_${lib}_$r.err; exit 1; }
    cat $O/region_${lib}_$r.json
  done
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], 'k2', d['k2']['us_per_step'])"
done
