#!/bin/bash
# Round 4, session e2: K5 rank shares, the unit order with 8 chunks (alpha 0.25 / 0.5) and with
# 4 chunks at alpha 0.125 / 0.5, against AUTO (4 chunks, alpha 0.25) and per wave, at 1 and 8
# ranks, the modes interleaved launch by launch (tools/k5_ab.py, 7 launches each).
# Usage: bash tools/sessions/gpu_r04e2.sh TAG
set -o pipefail
TAG=${1:-r04e2}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 500 python tools/k5_ab.py 7 1,8 per_wave,auto,split8a25,split8a50,split4a12,split4a50 \
  > $O/k5_ab.jsonl || { echo k5_ab failed; exit 1; }
cat $O/k5_ab.jsonl | python -c "import json,sys; [print(' ', d['world'], d['mode'], d['median_us'], d['min_us']) for d in map(json.loads, sys.stdin)]"
