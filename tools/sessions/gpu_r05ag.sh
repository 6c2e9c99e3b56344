#!/bin/bash
# Round 5: frame groups over tile pairs adopted for AUTO's two-wave groups (rt_tpair_kernel<2>,
# RT_FRAME_PAIRS_ON2; 7 waves per SIMD): the GPU suite (every frame-group case under on / quad
# / on2 / quad2), then tools/pairs_ab.py on one GPU — rank 0's chain share at world sizes
# 1 / 2 / 4 (20-frame calls, every frame's image) and the whole image at K4's structure
# (64-frame calls), 'on' (one tile per group) against 'on2' alternating — and
# bench.py --config K4 twice.
# Usage: bash tools/sessions/gpu_r05ag.sh TAG
set -o pipefail
TAG=${1:-r05ag}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python tools/pairs_ab.py 9 1,2,4 on,on2 20 every > $O/pairs_chain.jsonl 2> $O/pairs_chain.err \
  || { echo "pairs_ab failed"; tail $O/pairs_chain.err; exit 1; }
cat $O/pairs_chain.jsonl
timeout -k 10 300 python tools/pairs_ab.py 7 1 on,on2 64 last_two > $O/pairs_k4.jsonl 2> $O/pairs_k4.err \
  || { echo "pairs_ab failed"; tail $O/pairs_k4.err; exit 1; }
cat $O/pairs_k4.jsonl
for r in 1 2; do
  timeout -k 10 300 python bench.py --config K4 --cpu-seconds 0 > $O/bench_k4_$r.json 2> $O/bench_k4_$r.err \
    || { echo "bench failed"; tail $O/bench_k4_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_k4_$r.json')); print('K4', d['value'], d['ms_per_step'], d.get('image_ok'), d['roofline'].get('kernel'))"
done
