#!/bin/bash
# Round 6: launch timing carried by the dispatch packets (rt_set_launch_timing) — its test,
# and its cost against no events / marker events on the 8- and 1-rank K3 chain calls.
set -o pipefail
TAG=${1:-r06i}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "launch_timing or band_set" > $O/pytest_sel.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_sel.log; exit 1; }
tail -1 $O/pytest_sel.log
for n in 8 1; do
  timeout -k 10 300 python tools/call_latency.py $n 0 15 > $O/call_latency_n$n.json 2> $O/call_latency_n$n.err \
    || { echo "failed"; tail $O/call_latency_n$n.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/call_latency_n$n.json'))
for v in ('ev','noev','stream','ext','noev_again'):
    print($n, v, d[v]['fit'], d[v]['20'])
print('floor', d['tiny_kernel_region_us_med'])"
done
