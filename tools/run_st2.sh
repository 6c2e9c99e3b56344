cd $GRAFT_REPO_ROOT
for c in k3 k2; do RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_gst.so timeout -k 10 120 python tools/time_kernel.py $c; done
