#!/bin/bash
# Round 6: fixed cost of one timed call (tools/call_latency.py) for the 8-rank and 1-rank K3
# chain shares.
set -o pipefail
TAG=${1:-r06b}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for n in 8 1; do
  timeout -k 10 200 python tools/call_latency.py $n 0 15 > $O/call_latency_n$n.json 2> $O/call_latency_n$n.err \
    || { echo "failed"; tail $O/call_latency_n$n.err; exit 1; }
  cat $O/call_latency_n$n.json
done
