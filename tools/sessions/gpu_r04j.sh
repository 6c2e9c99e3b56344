#!/bin/bash
# Round 4, session j: the partial split schedule (only the costliest tiles of the cost order
# split, RT_SPLIT_FRAC): bounce parity tests, then a K5 A/B of split fractions at 1, 4 and 8
# ranks (tools/k5_ab.py, 7 interleaved launches per mode).
# Usage: bash tools/sessions/gpu_r04j.sh TAG
set -o pipefail
TAG=${1:-r04j}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "bounce_launches or k5_shares or update_frames_equals" > $O/pytest_split.log 2>&1 \
  || { tail -20 $O/pytest_split.log; exit 1; }
tail -2 $O/pytest_split.log
timeout -k 10 400 python tools/k5_ab.py 7 1,4,8 \
  per_wave,split2,split2f50,split2f25,split2f12,split4f25,split4f12,split3f25 > $O/k5_ab.jsonl \
  || { echo k5_ab failed; exit 1; }
cat $O/k5_ab.jsonl | python -c "import json,sys; [print(' ', d['world'], d['mode'], d['median_us'], d['min_us']) for d in map(json.loads, sys.stdin)]"
