set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
export RT_HIP_LIB=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants/librt_hip_v1noslpw8.so
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc -o p1 -- python tools/time_kernel.py k3 > gpurun_out/pmc/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc -o p2 -- python tools/time_kernel.py k3 > gpurun_out/pmc/p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o p3 -- python tools/time_kernel.py k3 > gpurun_out/pmc/p3.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o p4 -- python tools/time_kernel.py k3 > gpurun_out/pmc/p4.log 2>&1
ls -R gpurun_out/pmc | head -30
