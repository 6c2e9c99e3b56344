#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: ranks share the GPU, gloo carries the
# barriers, the timing all-reduce and the gather (staged through host memory).  Checks the
# multi-rank control flow and the gathered image against the fixtures; its timings are not
# measurements.  Usage: bash tools/gpu_rehearse.sh TAG
set -o pipefail
TAG=${1:-rehearse}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export RT_BENCH_BACKEND=gloo
run() {  # nproc port args...
  local n=$1 port=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n "$@" --cpu-seconds 0
}
run 2 29511 --steps 20 --warmup 5 > $O/k3_n2_driver.json 2> $O/k3_n2_driver.err || { tail $O/k3_n2_driver.err; exit 1; }
run 3 29512 --side 0 > $O/k3_n3.json 2> $O/k3_n3.err || { tail $O/k3_n3.err; exit 1; }
run 2 29513 --config K2 --side 0 > $O/k2_n2.json 2> $O/k2_n2.err || { tail $O/k2_n2.err; exit 1; }
run 4 29514 --config K4 --steps 2 --warmup 1 > $O/k4_n4.json 2> $O/k4_n4.err || { tail $O/k4_n4.err; exit 1; }
run 2 29515 --config K5 --steps 1 --warmup 1 > $O/k5_n2.json 2> $O/k5_n2.err || { tail $O/k5_n2.err; exit 1; }
for f in k3_n2_driver k3_n3 k2_n2 k4_n4 k5_n2; do
  python -c "import json; d=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', d['n_gpus'], d['value'], d['image_ok'], d.get('share_ok'), d['image_check'], d['timed_breakdown_ms'], d['data'][-40:])"
done
