cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pcs; export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1
grep -i -B2 -A8 "pc_sampling\|PC Sampling" gpurun_out/pcs/list.txt | head -40
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d gpurun_out/pcs -o k3 -- python3 tools/time_kernel.py k3 > gpurun_out/pcs/k3.log 2>&1; echo "rc=$?"; tail -5 gpurun_out/pcs/k3.log; ls -la gpurun_out/pcs
