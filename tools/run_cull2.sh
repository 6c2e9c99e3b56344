cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cull2
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/cull2/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/cull2/pytest.log
for m in exhaustive culled; do for c in k3 k2; do RT_SCAN_MODE=$m timeout -k 10 120 python tools/time_kernel.py $c; done; done
export TMPDIR=/tmp
for c in k3 k2; do
RT_SCAN_MODE=culled timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/cull2/pmc -o ${c}_p1 -- python tools/time_kernel.py $c > /dev/null 2>&1
RT_SCAN_MODE=culled timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/cull2/pmc -o ${c}_p2 -- python tools/time_kernel.py $c > /dev/null 2>&1
done
ls gpurun_out/cull2/pmc
