#!/bin/bash
# Round 5, session d: the driver's command after the StripeRenderer binding fix (both
# ping-pong directions bound at the first call: the timed call no longer binds), three runs;
# the rank-share region (tools/share_region.py) at 8 ranks under a kernel trace, to attribute
# the chain share's fixed cost; rank shares at 2 / 4 / 8 unprofiled.
# Usage: bash tools/sessions/gpu_r05d.sh TAG
set -o pipefail
TAG=${1:-r05d}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; s=d['rank_shares']['K3']['chain']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['timed_breakdown_ms'], 'k2', d['k2']['us_per_step'], 'chain', {k: v['us_per_step'] for k, v in s.items()}, 'k5', {k: v['us_per_step'] for k, v in d['rank_shares']['K5']['fused_64'].items()})"
done
for n in 2 4 8; do
  timeout -k 10 120 python tools/share_region.py $n 0 15 20 > $O/share_n${n}.json 2> $O/share_n$n.err || { tail $O/share_n$n.err; exit 1; }
  cat $O/share_n${n}.json | python -c "import json,sys; d=json.load(sys.stdin); d.pop('timeline_host'); print(d)"
done
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/tl_s8 -o tl -- python3 tools/share_region.py 8 0 5 20 \
  > $O/tl_s8_line.json 2> $O/tl_s8.err || { echo "rocprof s8 failed"; tail $O/tl_s8.err; exit 1; }
python tools/timeline.py $O/tl_s8 $O/tl_s8_line.json > $O/timeline_s8.json || exit 1
python -c "import json; d=json.load(open('$O/timeline_s8.json')); [d.pop(k) for k in ('hip_calls',)]; print(json.dumps(d))"
