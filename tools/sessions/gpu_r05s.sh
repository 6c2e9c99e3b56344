#!/bin/bash
# Round 5, session s: the committed tree's other lines — bench.py --config K2 / K4 / K5 as
# main lines, bench.py --gpus 2 / 4 rehearsed over gloo on this one GPU (per_rank_ms,
# barrier_ms, the gathered image), and the driver's command five more times (its spread on
# one box).
# Usage: bash tools/sessions/gpu_r05s.sh TAG
set -o pipefail
TAG=${1:-r05s}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for c in K2 K4 K5; do
  timeout -k 10 300 python bench.py --config $c --side 0 --cpu-seconds 0 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['unit'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
done
for n in 2 4; do
  RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
    > $O/rehearse_k3_n$n.json 2> $O/rehearse_k3_n$n.err || { echo "rehearse $n failed"; tail $O/rehearse_k3_n$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/rehearse_k3_n$n.json').read().strip().splitlines()[-1]); print('n$n', d['value'], d['ms_per_step'], d['image_ok'], d['timed_breakdown_ms'])"
done
for r in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], d['image_ok'])"
done
