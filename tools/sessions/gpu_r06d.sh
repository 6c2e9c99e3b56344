#!/bin/bash
# Round 6: the exhaustive radius check + accumulator gate (ADVICE), and the new bench.py
# (one launch structure at every N, CLOCK_MONOTONIC job time, wall-clock rank shares).
set -o pipefail
TAG=${1:-r06d}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "selftest or markstein or normal or k5 or bench_dispatch" > $O/pytest_sel.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_sel.log; exit 1; }
tail -2 $O/pytest_sel.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "bench failed"; tail $O/bench_driver.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r06d/bench_driver.json'))
r=d['roofline']
print('K3', d['value'], d['ms_per_step'], r['bound'], r['kernel'], r['kernel_avg_us'], r['frac'], r.get('hbm',{}).get('frac'), d['image_ok'], d['image_check'], d['share_ok'], d.get('side_error'))
print('dispatch', {k: d['dispatch'][k] for k in ('us_per_step','events_us_per_step','hbm_frac_events','image_ok','kernel')})
print('k2', {k: d['k2'][k] for k in ('us_per_step','events_us_per_step','hbm_frac_events','image_ok')})
rs=d['rank_shares']
for s in (20,200):
    print(s, {k:(v['us_per_step'], v['efficiency'], v['image_ok'], v.get('rank_spread')) for k,v in rs[f'K3_chain_{s}_steps'].items()})
print(rs['K3_call_model'], rs['runtime_floor_us'])
print({k:(v['us_per_step'], v['efficiency'], v['image_ok']) for k,v in rs['K5_fused_64'].items()})
print('k5', d['k5']['us_per_step'], d['k5']['segments_per_s'], 'k4', d['k4']['us_per_step'], d['k4']['image_ok'])
PY
