#!/bin/bash
# Round 6: VALU attribution of the camera-ray sample (verdict item 3) — one PMC pass
# (SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_WAVES) of the driver's K3 command per knock-out build
# (build/variants/librt_hip_skoK.so from tools/patches/single_knockouts.patch), in the
# reference's dispatch structure (rt_single_kernel<2>) and the main line's frame chain
# (rt_tpair_kernel<2>); then the driver's command twice more on the product build.
set -o pipefail
TAG=${1:-r06h}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for mode in dispatch chain; do
  for b in base sko0 sko1 sko2 sko4 sko8 sko14; do
    if [ $b = base ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_$b.so; fi
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/raw -o ${mode}_$b -- \
      python3 bench.py --frame-launch $mode --side 0 --cpu-seconds 0 --steps 20 --warmup 5 > $O/${mode}_$b.log 2>&1 \
      || { echo "pmc $mode $b failed"; tail -5 $O/${mode}_$b.log; exit 1; }
  done
done
unset RT_HIP_LIB
python3 tools/valu_attribution.py $O/raw > $O/valu_attribution_r06.json || exit 1
cat $O/valu_attribution_r06.json | python3 -c "import json,sys; d=json.load(sys.stdin); [print(m, json.dumps(v.get('attribution'))) for m,v in d.items()]"
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo "bench failed"; tail $O/bench_driver_$r.err; exit 1; }
  python tools/summarize_bench.py $O/bench_driver_$r.json
done
