#!/bin/bash
# Round 4, session v: the bound call passing the camera blob itself and a cached sphere
# pointer: the -m gpu suite, the host cost per call, the K3 frame-chain rank shares, and the
# driver's bench command twice.
# Usage: bash tools/sessions/gpu_r04v.sh TAG
set -o pipefail
TAG=${1:-r04v}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python tools/host_call.py 20 > $O/host_call.jsonl || { echo host_call failed; exit 1; }
cat $O/host_call.jsonl
RT_FPL=0 RT_IMAGES=every RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py K3 20 > $O/rank_K3_chain.jsonl 2> $O/rank.err \
  || { echo rank_sim failed; tail -5 $O/rank.err; exit 1; }
python -c "import json; [print('chain', d['world'], d['us_per_step'], d['predicted_efficiency'], d.get('host_issue_us_per_step')) for d in map(json.loads, open('$O/rank_K3_chain.jsonl'))]"
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; c=d['rank_shares']['K3']['chain']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], d['image_ok'], {w: v['us_per_step'] for w, v in c.items()})"
done
