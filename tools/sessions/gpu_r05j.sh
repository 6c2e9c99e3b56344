#!/bin/bash
# Round 5, session j: the tree with the Markstein normal — GPU suite, smoke, the driver's command twice (the
# side lines now warmed 50 ms, median of five), and bench.py --config K2 as a main line.
# Then the hit normal's Markstein division (normal_rn, on) against div_core's two steps
# (RT_NORMAL_RN=0): the driver's region (K3, K2), the 8-rank chain share, three rounds.
# Usage: bash tools/sessions/gpu_r05j.sh TAG
set -o pipefail
TAG=${1:-r05j}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; s=d['rank_shares']['K3']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], 'k2', d['k2']['us_per_step'], 'chain', {k: (v['us_per_step'], v['efficiency_vs_1gpu_step']) for k, v in s['chain'].items()}, 'k5', {k: v['us_per_step'] for k, v in d['rank_shares']['K5']['fused_64'].items()})"
  echo "bench run $r: $(python -c "print(round($(date +%s.%N) - $t0, 1))") s"
done
timeout -k 10 300 python bench.py --config K2 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 > $O/bench_k2.json 2> $O/bench_k2.err || { tail $O/bench_k2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_k2.json')); r=d['roofline']; print('K2', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
for r in 1 2 3; do
  for v in on off; do
    if [ $v = off ]; then export RT_NORMAL_RN=0; else unset RT_NORMAL_RN; fi
    for cfg in K3 K2; do
      timeout -k 10 120 python tools/driver_region.py 25 $cfg $v= \
        > $O/region_${cfg}_${v}_$r.json 2> $O/region_${cfg}_${v}_$r.err || { tail $O/region_${cfg}_${v}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/region_${cfg}_${v}_$r.json')); print('$cfg', '$v', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
    timeout -k 10 120 python tools/share_region.py 8 0 15 20 > $O/share_${v}_n8_$r.json 2> $O/share_${v}_n8_$r.err || { tail $O/share_${v}_n8_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/share_${v}_n8_$r.json')); print('$v', 'n8', d['kernel'], 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
  done
done
unset RT_NORMAL_RN
# the hinted path's count check as a range test (librt_hip_pend.so, -DRT_PEND_RANGE=1)
# against the tree's build (librt_hip_cur.so), both through ctypes (RT_HIP_LIB)
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_pend.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "bench or golden or queues or normal" > $O/pytest_gpu_pend.log 2>&1 || { echo "pytest pend failed"; tail -30 $O/pytest_gpu_pend.log; exit 1; }
tail -1 $O/pytest_gpu_pend.log
for r in 1 2 3; do
  for lib in cur pend; do
    for cfg in K3 K2; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/driver_region.py 25 $cfg $lib= \
        > $O/region_${cfg}_${lib}_$r.json 2> $O/region_${cfg}_${lib}_$r.err || { tail $O/region_${cfg}_${lib}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/region_${cfg}_${lib}_$r.json')); print('$cfg', '$lib', 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
  done
done
# frame groups at small shares: two (on) against four (quad, AUTO's choice there) waves per tile
for r in 1 2; do
  for n in 8 4; do
    for m in quad on; do
      timeout -k 10 120 python tools/share_region.py $n 0 15 20 $m > $O/share_${m}_n${n}_$r.json 2> $O/share_${m}_n${n}_$r.err || { tail $O/share_${m}_n${n}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/share_${m}_n${n}_$r.json')); print('$m', 'n$n', d['kernel'], 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
  done
done
# frame groups with a dedicated accumulating wave (librt_hip_gacc.so, -DRT_GROUP_ACC=1: every
# group's samplers all trace, one more wave accumulates and stores) against the tree's build
RT_HIP_LIB=$V/librt_hip_gacc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "chain or pair or share or frames" > $O/pytest_gpu_gacc.log 2>&1 || { echo "pytest gacc failed"; tail -30 $O/pytest_gpu_gacc.log; exit 1; }
tail -1 $O/pytest_gpu_gacc.log
for r in 1 2; do
  for n in 8 4 1; do
    for lib in cur gacc; do
      RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/share_region.py $n 0 15 20 > $O/share_${lib}_n${n}_$r.json 2> $O/share_${lib}_n${n}_$r.err || { tail $O/share_${lib}_n${n}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/share_${lib}_n${n}_$r.json')); print('$lib', 'n$n', d['kernel'], 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'])"
    done
  done
done
