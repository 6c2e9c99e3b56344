#!/bin/bash
# Round-3 session zn: the one-tile instance (rank shares) with the seed hashes computed in the wave (RT_SINGLE_HASH=1: no table loads behind the order entry)
# against the tables, per-rank K3 / K2, three interleaved rounds.
# Usage: bash tools/gpu_r03zn.sh TAG
set -o pipefail
TAG=${1:-r03zn}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_hash1.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "single or update_queues_match or bench_dispatch_chain or aql or stripe" > $O/pytest_hash1.log 2>&1
rc=$?; echo "pytest hash1 rc=$rc"; tail -2 $O/pytest_hash1.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in default $V/librt_hip_hash1.so; do
    for c in K3 K2; do
      n=$(basename $lib .so)
      if [ $lib = default ]; then E=""; else E="RT_HIP_LIB=$lib"; fi
      env $E RT_FPL=1 RT_REPS=7 timeout -k 10 300 python tools/rank_sim.py $c 50 > $O/rank_${c}_${n}_$r.jsonl || exit 1
      python -c "import json,sys; print(sys.argv[2], sys.argv[3], sys.argv[4], ' '.join('%d:%s:%s' % (d['world'], d['us_per_step'], d['submit']) for d in map(json.loads, open(sys.argv[1]))))" $O/rank_${c}_${n}_$r.jsonl $c $n $r
    done
  done
done
