#!/bin/bash
# Round 4, session w: bench.py --gpus N rehearsed on the one-GPU box with the final build
# (RT_BENCH_BACKEND=gloo: ranks share the GPU, gloo carries barriers, timing and the gather):
# K3 at N = 2 and 4 (the driver's --steps 20 --warmup 5) and K5 at N = 4 — the multi-rank flow
# and its gathered image, not a measurement.
# Usage: bash tools/sessions/gpu_r04w.sh TAG
set -o pipefail
TAG=${1:-r04w}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export RT_BENCH_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29520 + n)) bench.py --gpus $n --steps 20 --warmup 5 --cpu-seconds 0 \
    > $O/rehearse_k3_n$n.json 2> $O/rehearse_k3_n$n.err || { echo "rehearse $n failed"; tail $O/rehearse_k3_n$n.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/rehearse_k3_n$n.json') if l.startswith('{')][-1]); print('rehearse K3', d['n_gpus'], d['value'], d['image_ok'], d['config']['frame_launch'], d['roofline']['kernel'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29530 bench.py --gpus 4 --config K5 --steps 1 --warmup 1 --cpu-seconds 0 \
  > $O/rehearse_k5_n4.json 2> $O/rehearse_k5_n4.err || { echo "rehearse k5 failed"; tail $O/rehearse_k5_n4.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/rehearse_k5_n4.json') if l.startswith('{')][-1]); print('rehearse K5', d['n_gpus'], d['value'], d['image_ok'], d['roofline']['kernel'])"
