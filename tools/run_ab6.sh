cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest6.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest6.log
for c in k3 k2; do
timeout -k 10 500 python tools/ab_variants.py $c 2 gpu-ray-tracing_amd/build/variants/librt_hip_b8.so gpu-ray-tracing_amd/build/variants/librt_hip_e8.so gpu-ray-tracing_amd/build/variants/librt_hip_e7.so > gpurun_out/ab6_$c.log 2>&1; tail -3 gpurun_out/ab6_$c.log
done
