cd $GRAFT_REPO_ROOT
for c in k3 k2; do
timeout -k 10 500 python tools/ab_variants.py $c 2 gpu-ray-tracing_amd/build/variants/librt_hip_b8.so gpu-ray-tracing_amd/build/variants/librt_hip_b7.so gpu-ray-tracing_amd/build/variants/librt_hip_b6.so gpu-ray-tracing_amd/build/variants/librt_hip_d1.so gpu-ray-tracing_amd/build/variants/librt_hip_d2.so gpu-ray-tracing_amd/build/variants/librt_hip_d3.so > gpurun_out/ab5_$c.log 2>&1; tail -6 gpurun_out/ab5_$c.log
done
