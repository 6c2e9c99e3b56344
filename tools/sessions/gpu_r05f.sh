#!/bin/bash
# Round 5, session f: the Markstein divisions split — the accumulator's alone
# (librt_hip_acc.so: -DRT_NORMAL_RN=0) and with the normal's (librt_hip_mk.so, the default)
# against the previous build (librt_hip_base.so), the driver's region, three interleaved
# rounds of separate processes; then bench.py --gpus 2 / 4 rehearsed on this one GPU over
# gloo (per_rank_ms, barrier_ms).
# Usage: bash tools/sessions/gpu_r05f.sh TAG
set -o pipefail
TAG=${1:-r05f}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
for r in 1 2 3; do
  for lib in base acc mk; do
    RT_HIP_LIB=$V/librt_hip_$lib.so timeout -k 10 120 python tools/driver_region.py 25 K3 $lib= \
      > $O/region_${lib}_$r.json 2> $O/region_${lib}_$r.err || { tail $O/region_${lib}_$r.err; exit 1; }
    cat $O/region_${lib}_$r.json
  done
done
for n in 2 4; do
  RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
    > $O/rehearse_k3_n$n.json 2> $O/rehearse_k3_n$n.err || { echo "rehearse $n failed"; tail $O/rehearse_k3_n$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/rehearse_k3_n$n.json').read().strip().splitlines()[-1]); print('n$n', d['value'], d['ms_per_step'], d['image_ok'], d['timed_breakdown_ms'])"
done
