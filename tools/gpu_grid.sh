#!/bin/bash
# Grid walk for wide-cone bounce rays: parity suite, then K5 A/B against the no-grid build.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/grid; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
NOGRID=gpu-ray-tracing_amd/build/variants/librt_hip_nogrid.so
for r in 1 2; do
  for lib in default $NOGRID; do
    if [ $lib = default ]; then E=""; else E="RT_HIP_LIB=$lib"; fi
    env $E timeout -k 10 300 python bench.py --config K5 --steps 10 --warmup 2 --cpu-seconds 0 \
      > $O/k5_${r}_$(basename $lib).json 2>> $O/bench.err || exit 1
    echo "$r $lib $(python -c "import json,sys; d=json.load(open('$O/k5_${r}_$(basename $lib).json')); print(d['ms_per_step'], d['value'])")"
  done
done
