#!/bin/bash
# Single-frame launch diagnosis: dispatch-rate microbench, wave traces of one rt_update
# (K3, K2), and issue/stall PMC groups of the single-frame kernel over time_kernel.py.
set -o pipefail
TAG=${1:-diag}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/dispatch_rate > $O/dispatch_rate.jsonl 2>&1 || { echo dispatch failed; tail $O/dispatch_rate.jsonl; exit 1; }
cat $O/dispatch_rate.jsonl
for c in K3 K2; do
  RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_wt.so timeout -k 10 180 \
    python tools/wave_trace_single.py $c > $O/wt_single_$c.json 2>&1 || { echo wt failed; tail $O/wt_single_$c.json; exit 1; }
  grep '^{' $O/wt_single_$c.json
done
bash tools/pmc_kernel.sh $TAG "k3 k2"
