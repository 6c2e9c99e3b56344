#!/bin/bash
# GPU session: -m gpu tests on the product build, then interleaved kernel timings of
# library builds on configs.  Usage: bash tools/gpu_ab.sh TAG "k3 k2" ROUNDS lib1 lib2 ...
set -o pipefail
TAG=$1; CFGS=$2; ROUNDS=$3; shift 3
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log | grep -v "^$"; [ $rc -eq 0 ] || exit 1
for c in $CFGS; do
  timeout -k 10 600 python tools/ab_variants.py $c $ROUNDS "$@" > $O/ab_$c.log 2>&1 \
    || { echo "ab $c failed"; tail -5 $O/ab_$c.log; exit 1; }
  tail -$# $O/ab_$c.log
done
