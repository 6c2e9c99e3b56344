#!/bin/bash
# -m gpu tests, single-frame A/B against a baseline build, and a kernel-trace profile of
# bench.py K3 (side lines on: cold-camera frames rebuild the candidate lists).
# Usage: bash tools/gpu_cand.sh TAG baseline.so
set -o pipefail
TAG=$1; BASE=$2
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for c in k3 k2; do
  timeout -k 10 600 python tools/ab_variants.py $c 5 $BASE gpu-ray-tracing_amd/build/librt_hip.so \
    > $O/ab_$c.log 2>&1 || { echo "ab $c failed"; tail -5 $O/ab_$c.log; exit 1; }
  tail -2 $O/ab_$c.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k3 -- python3 bench.py --config K3 \
  --cpu-seconds 0 > $O/bench_k3.json 2> $O/bench_k3.err || { echo "prof failed"; tail -3 $O/bench_k3.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/k3_kernel_stats.csv
python3 -c "
import csv,sys
for r in csv.DictReader(open('$O/k3_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'])"
python3 -c "import json; d=json.loads(open('$O/bench_k3.json').read()); print(d['value'], d['roofline']['kernel_avg_us'], d.get('cold_camera'))"
