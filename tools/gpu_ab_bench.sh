#!/bin/bash
# Interleaved bench.py A/B of library builds: gpu_ab_bench.sh CONFIG STEPS ROUNDS lib...
# ("default" = the in-tree build).  Prints ms_per_step per (round, lib).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/ab_bench; mkdir -p $O
CFG=$1; STEPS=$2; ROUNDS=$3; shift 3
for r in $(seq $ROUNDS); do
  for lib in "$@"; do
    if [ $lib = default ]; then E=""; else E="RT_HIP_LIB=$lib"; fi
    f=$O/${CFG}_${r}_$(basename $lib).json
    env $E timeout -k 10 300 python bench.py --config $CFG --steps $STEPS --warmup 2 \
      --cpu-seconds 0 --exhaustive-steps 0 --per-frame-steps 0 > $f 2>> $O/bench.err || exit 1
    echo "$r $(basename $lib) $(python -c "import json; d=json.load(open('$f')); print(d['ms_per_step'])")"
  done
done
