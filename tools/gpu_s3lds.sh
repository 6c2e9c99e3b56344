# One-frame kernel session: -m gpu tests, A/B against build/variants (K3, K2), rank shares
# of the per-dispatch K3 step with each one-frame instance.  Usage: bash tools/gpu_s3lds.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
B=gpu-ray-tracing_amd/build; V=$(ls $B/variants/*.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py k3 3 $B/librt_hip.so $V > $O/ab_k3.log 2>&1 || exit 1
timeout -k 10 600 python tools/ab_variants.py k2 2 $B/librt_hip.so $V > $O/ab_k2.log 2>&1 || exit 1
for m in pair one; do RT_SINGLE=$m RT_FPL=1 timeout -k 10 300 python tools/rank_sim.py K3 > $O/rank_sim_k3_$m.jsonl 2>&1 || exit 1; done
