#!/bin/bash
# Round 4, session b: the driver's bench command (twice; new side lines: cold_start, k2, k5,
# rank_shares), the host cost of one rt_update_frames call, the N = 2 / 4 / 8 rehearsal of the
# chain-mode rank shares (gloo, ranks sharing the GPU: control flow + gathered image only),
# and the rocprofv3 kernel trace of the driver's command.
# Usage: bash tools/sessions/gpu_r04b.sh TAG
set -o pipefail
TAG=${1:-r04b}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  /usr/bin/time -f "%e s" -o $O/bench_driver_$r.time timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], d['config']['frame_launch'])"
  cat $O/bench_driver_$r.time
done
timeout -k 10 120 python tools/host_call.py 20 > $O/host_call.jsonl || { echo host_call failed; exit 1; }
cat $O/host_call.jsonl
export RT_BENCH_BACKEND=gloo
for n in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29520 + n)) bench.py --gpus $n --steps 20 --warmup 5 --cpu-seconds 0 \
    > $O/rehearse_k3_n$n.json 2> $O/rehearse_k3_n$n.err || { echo "rehearse $n failed"; tail $O/rehearse_k3_n$n.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/rehearse_k3_n$n.json') if l.startswith('{')][-1]); print('rehearse', d['n_gpus'], d['value'], d['image_ok'], d['config']['frame_launch'], d['roofline']['kernel'])"
done
unset RT_BENCH_BACKEND
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > $O/prof_driver.log 2>&1 || { echo "rocprof failed"; tail $O/prof_driver.log; exit 1; }
echo rocprof done
