cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest8.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest8.log
RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_gst.so timeout -k 10 120 python tools/time_kernel.py k3
timeout -k 10 500 python tools/ab_variants.py k3 2 gpu-ray-tracing_amd/build/variants/librt_hip_b8.so gpu-ray-tracing_amd/build/variants/librt_hip_g0.so gpu-ray-tracing_amd/build/variants/librt_hip_g1.so > gpurun_out/ab8_k3.log 2>&1; tail -3 gpurun_out/ab8_k3.log
