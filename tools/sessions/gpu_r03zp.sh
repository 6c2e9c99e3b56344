#!/bin/bash
# Round-3 A/B: waves per workgroup of the one-frame kernel (RT_SINGLE_WG 1 / 2 against 4) on
# rank shares, K3 / K2, parity subset on each variant first, three interleaved rounds.
# Usage: bash tools/gpu_r03zp.sh TAG
set -o pipefail
TAG=${1:-r03zp}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
for t in 1 2; do
  RT_HIP_LIB=$V/librt_hip_swg$t.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "single or update_queues_match or bench_dispatch_chain or aql" > $O/pytest_swg$t.log 2>&1
  rc=$?; echo "pytest swg$t rc=$rc"; tail -1 $O/pytest_swg$t.log; [ $rc -eq 0 ] || exit 1
done
for r in 1 2 3; do
  for lib in default $V/librt_hip_swg1.so $V/librt_hip_swg2.so; do
    for c in K3 K2; do
      n=$(basename $lib .so)
      if [ $lib = default ]; then E=""; else E="RT_HIP_LIB=$lib"; fi
      env $E RT_FPL=1 RT_REPS=5 timeout -k 10 300 python tools/rank_sim.py $c 50 > $O/rank_${c}_${n}_$r.jsonl 2> $O/rank.err \
        || { echo "rank_sim failed"; tail $O/rank.err; exit 1; }
      python -c "import json,sys; print(sys.argv[2], sys.argv[3], sys.argv[4], ' '.join('%d:%s:%s' % (d['world'], d['us_per_step'], d['submit']) for d in map(json.loads, open(sys.argv[1]))))" $O/rank_${c}_${n}_$r.jsonl $c $n $r
    done
  done
done
