#!/bin/bash
# Interleaved kernel timings of library builds (no tests).
# Usage: bash tools/run_abonly.sh TAG "k3 k2" ROUNDS lib1 lib2 ...
set -o pipefail
TAG=$1; CFGS=$2; ROUNDS=$3; shift 3
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for c in $CFGS; do
  timeout -k 10 600 python tools/ab_variants.py $c $ROUNDS "$@" > $O/ab_$c.log 2>&1 || { echo "ab $c failed"; tail -5 $O/ab_$c.log; exit 1; }
  tail -$# $O/ab_$c.log
done
