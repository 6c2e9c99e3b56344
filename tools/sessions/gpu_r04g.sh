#!/bin/bash
# Round 4, session g: VALU instructions per wave of the one-frame kernel with each phase
# knocked out (RT_SKO builds: 1 no accumulator load, 2 no sphere scan (so no hit shading),
# 4 no random camera ray, 8 no hit shading) against the in-tree build, one PMC pass each
# (SQ_WAVES, SQ_INSTS_VALU, SQ_INSTS_SALU) over bench.py K3 with one launch per update.
# Usage: bash tools/sessions/gpu_r04g.sh TAG
set -o pipefail
TAG=${1:-r04g}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
ARGS="--config K3 --side 0 --cpu-seconds 0 --queues 1 --steps 20 --warmup 5"
for lib in default sko1 sko2 sko4 sko8; do
  E=""; [ $lib != default ] && E="RT_HIP_LIB=$V/librt_hip_$lib.so"
  env $E timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv \
    -d $O/raw -o $lib -- python3 bench.py $ARGS > $O/pmc_$lib.log 2>&1 \
    || { echo "pmc $lib failed"; tail -5 $O/pmc_$lib.log; exit 1; }
  python3 tools/pmc_bench_summary.py $O/pmc_$lib.json "rt_single_kernel<2>" 1 $O/raw/${lib}_counter_collection.csv | head -c 400; echo
done
