#!/bin/bash
# Round 6: which of the bounce instance's last three changes pays — the dielectric's
# divisions and square roots on the fast cores (diel), fast roots in the cone scan (cone),
# the all-f32 defocus disk (disk) — each alone on the hint-table build (hr2), against all
# three (the tree); K5 step and 8-rank share (tools/k5_ab.py).
set -o pipefail
TAG=${1:-r06p}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/gpu-ray-tracing_amd/build/variants
timeout -k 10 900 python tools/k5_ab.py 3 $V/librt_hip_hr2.so $V/librt_hip_diel.so $V/librt_hip_cone.so \
  $V/librt_hip_disk.so tree > $O/k5_ab.jsonl 2> $O/k5_ab.err \
  || { echo "ab failed"; tail $O/k5_ab.err; tail -3 $O/k5_ab.jsonl; exit 1; }
tail -1 $O/k5_ab.jsonl
