cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cull1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/cull1/pytest.log 2>&1; echo "pytest rc=$?"; tail -15 gpurun_out/cull1/pytest.log
for m in exhaustive culled; do for c in k3 k2; do RT_SCAN_MODE=$m timeout -k 10 120 python tools/time_kernel.py $c; done; done
