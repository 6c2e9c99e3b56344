set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/s3scan; mkdir -p $O
B=gpu-ray-tracing_amd/build; V=$B/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py k3 3 $B/librt_hip.so $V/librt_hip_g1.so $V/librt_hip_g1s1.so $V/librt_hip_g1s2.so $V/librt_hip_s1.so > $O/ab_scan_k3.log 2>&1 || exit 1
timeout -k 10 600 python tools/ab_variants.py k2 2 $B/librt_hip.so $V/librt_hip_g1.so $V/librt_hip_g1s1.so $V/librt_hip_g1s2.so $V/librt_hip_s1.so > $O/ab_scan_k2.log 2>&1 || exit 1
for m in pair one; do RT_SINGLE=$m RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 > $O/rank_sim_k3_$m.jsonl 2>&1 || exit 1; done
