#!/bin/bash
# Round 4, session d = c + b: the -m gpu suite (split bounce mode, chain hardening), the
# driver's bench command twice (new
# side lines), the host cost of one rt_update_frames call, the N = 2 / 4 / 8 gloo rehearsal
# of chain-mode shares, the driver command's rocprofv3 kernel trace.
# Usage: bash tools/sessions/gpu_r04d.sh TAG
set -o pipefail
TAG=${1:-r04d}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  echo "$(date +%s.%N) $t0" | awk '{printf "%.1f s\n", $1 - $2}' > $O/bench_driver_$r.time
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
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29530 bench.py --gpus 4 --config K5 --steps 1 --warmup 1 --cpu-seconds 0 \
  > $O/rehearse_k5_n4.json 2> $O/rehearse_k5_n4.err || { echo "rehearse k5 failed"; tail $O/rehearse_k5_n4.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/rehearse_k5_n4.json') if l.startswith('{')][-1]); print('rehearse K5', d['n_gpus'], d['value'], d['image_ok'], d['roofline']['kernel'])"
unset RT_BENCH_BACKEND
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > $O/prof_driver.log 2>&1 || { echo "rocprof failed"; tail $O/prof_driver.log; exit 1; }
echo rocprof done
