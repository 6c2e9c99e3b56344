cd $GRAFT_REPO_ROOT
for c in k3 k2; do
timeout -k 10 500 python tools/ab_variants.py $c 2 gpu-ray-tracing_amd/build/variants/librt_hip_g0.so gpu-ray-tracing_amd/build/variants/librt_hip_h0.so gpu-ray-tracing_amd/build/variants/librt_hip_h0.so:RT_PERSISTENT=1 > gpurun_out/ab9_$c.log 2>&1; tail -3 gpurun_out/ab9_$c.log
done
