#!/bin/bash
# Round-3 session zf: bench.py's N > 1 path rehearsed over gloo on one GPU with the AUTO
# submission (N = 4: every rank's share is 6 000-11 999 tiles, so AQL packets), K3 driver
# command and default length, K2.  Usage: bash tools/gpu_r03zf.sh TAG
set -o pipefail
TAG=${1:-r03zf}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export RT_BENCH_BACKEND=gloo
run() {  # nproc port args...
  local n=$1 port=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n "$@" --cpu-seconds 0
}
run 4 29521 --steps 20 --warmup 5 > $O/k3_n4_driver.json 2> $O/k3_n4_driver.err || { tail $O/k3_n4_driver.err; exit 1; }
run 4 29522 --side 0 > $O/k3_n4.json 2> $O/k3_n4.err || { tail $O/k3_n4.err; exit 1; }
run 4 29523 --config K2 --side 0 > $O/k2_n4.json 2> $O/k2_n4.err || { tail $O/k2_n4.err; exit 1; }
for f in k3_n4_driver k3_n4 k2_n4; do
  python -c "import json; d=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); r=d['roofline']; print('$f', d['n_gpus'], d['value'], d['image_ok'], d['image_check'], r['submit'], r['queues'], d['data'][-40:])"
done
