cd $GRAFT_REPO_ROOT
for c in k3 k2; do
timeout -k 10 500 python tools/ab_variants.py $c 2 gpu-ray-tracing_amd/build/variants/librt_hip_w8.so gpu-ray-tracing_amd/build/variants/librt_hip_w7.so gpu-ray-tracing_amd/build/variants/librt_hip_w6.so gpu-ray-tracing_amd/build/variants/librt_hip_w8.so:RT_GRID=tiles gpu-ray-tracing_amd/build/variants/librt_hip_w6.so:RT_GRID=tiles > gpurun_out/ab4_$c.log 2>&1; tail -5 gpurun_out/ab4_$c.log
done
