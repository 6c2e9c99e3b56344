#!/bin/bash
# Round 5, session t: the cone cull's rigorous margin tightened — dist > sqrt(R^2 + m^2)
# instead of R + m (this tree, librt_hip_tight.so) against round 4's (librt_hip_r4cull.so,
# -DRT_CULL_ROUND4=1): the GPU suite on the tree, the candidate lists' size, the driver's
# region (K3, K2), the 8-rank chain share and K5's 64-spp step, interleaved, three rounds.
# Usage: bash tools/sessions/gpu_r05t.sh TAG
set -o pipefail
TAG=${1:-r05t}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for lib in r4cull tight; do
  RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --side 0 --cpu-seconds 0 > $O/bench_${lib}.json 2> $O/bench_${lib}.err || { tail $O/bench_${lib}.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_${lib}.json')); print('$lib', 'lists', d['candidate_lists'], d['roofline']['kernel_avg_us'], d['image_ok'])"
done
for r in 1 2 3; do
  for lib in r4cull tight; do
    for cfg in K3 K2; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/driver_region.py 25 $cfg $lib= \
        > $O/region_${cfg}_${lib}_$r.json 2> $O/region_${cfg}_${lib}_$r.err || { tail $O/region_${cfg}_${lib}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/region_${cfg}_${lib}_$r.json')); print('$cfg', '$lib', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
    RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/share_region.py 8 0 15 20 > $O/share_${lib}_n8_$r.json 2> $O/share_${lib}_n8_$r.err || { tail $O/share_${lib}_n8_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/share_${lib}_n8_$r.json')); print('$lib', 'n8', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
  done
done
for r in 1 2; do
  for lib in r4cull tight; do
    RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 300 python bench.py --config K5 --side 0 --cpu-seconds 0 > $O/bench_K5_${lib}_$r.json 2> $O/bench_K5_${lib}_$r.err || { tail $O/bench_K5_${lib}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_K5_${lib}_$r.json')); print('K5', '$lib', d['ms_per_step'], d['image_ok'])"
  done
done
