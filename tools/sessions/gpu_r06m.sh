#!/bin/bash
# Round 6: does the idle GPU's wake-up add to a timed call? tools/idle_latency.py at 8 and
# 1 ranks: idle, after a 1-ms pause, and beside a 1-wave spin kernel on another stream.
set -o pipefail
TAG=${1:-r06m}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/idle_latency.py 8 25 > $O/idle_n8.txt 2>&1 || { echo "n8 failed"; tail $O/idle_n8.txt; exit 1; }
timeout -k 10 300 python tools/idle_latency.py 1 15 > $O/idle_n1.txt 2>&1 || { echo "n1 failed"; tail $O/idle_n1.txt; exit 1; }
grep -v "^{" $O/idle_n8.txt; grep -v "^{" $O/idle_n1.txt
