#!/bin/bash
# Round 4, sessions f + g in one call: the split-schedule parity tests after the chunk-0
# register change, the knock-out PMC passes (gpu_r04g.sh), the variant A/B (gpu_r04f.sh),
# a K5 per-wave / split-2 A/B at 1, 4 and 8 ranks, and the driver's bench command timed.
# Usage: bash tools/sessions/gpu_r04fg.sh TAG
set -o pipefail
TAG=${1:-r04fg}
cd $GRAFT_REPO_ROOT; O=gpurun_out/${TAG}_h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "bounce_launches or k5_shares or update_frames_equals" > $O/pytest_split.log 2>&1 \
  || { tail -20 $O/pytest_split.log; exit 1; }
tail -2 $O/pytest_split.log
bash tools/sessions/gpu_r04g.sh ${TAG}_g || exit 1
bash tools/sessions/gpu_r04f.sh ${TAG}_f || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/k5_ab.py 7 1,4,8 per_wave,split2 > $O/k5_ab.jsonl || { echo k5_ab failed; exit 1; }
cat $O/k5_ab.jsonl | python -c "import json,sys; [print(' ', d['world'], d['mode'], d['median_us'], d['min_us']) for d in map(json.loads, sys.stdin)]"
# the driver's bench command once more, timed end to end (native-thread CPU baseline)
t0=$(date +%s.%N)
timeout -k 10 300 python bench.py > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
t1=$(date +%s.%N); awk -v a=$t0 -v b=$t1 'BEGIN{printf "%.1f s\n", b-a}' | tee $O/bench_driver.time
head -c 600 $O/bench_driver.json; echo
