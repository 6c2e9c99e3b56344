#!/bin/bash
# Round 4, session n: after AUTO runs a share's first (cost-measuring) launch per wave — the
# -m gpu suite and smoke(), the K5 AUTO / per-wave A/B at 4 and 8 ranks, the driver's bench
# command twice and the default bench line (reading the round-4 PMC and weighted files).
# Usage: bash tools/sessions/gpu_r04n.sh TAG
set -o pipefail
TAG=${1:-r04n}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python tools/k5_ab.py 7 4,8 per_wave,auto > $O/k5_ab.jsonl || { echo k5_ab failed; exit 1; }
cat $O/k5_ab.jsonl | python -c "import json,sys; [print(' ', d['world'], d['mode'], d['median_us'], d['min_us']) for d in map(json.loads, sys.stdin)]"
for r in 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  echo "$(date +%s.%N) $t0" | awk '{printf "%.1f s\n", $1 - $2}' > $O/bench_driver_$r.time
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; k=d['rank_shares']['K5']['fused_64']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r['binding_frac'], d['image_ok'], {w: (v['us_per_step'], v['predicted_efficiency']) for w, v in k.items()})"
  cat $O/bench_driver_$r.time
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo bench failed; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r['binding_frac'], d['image_ok'])"
