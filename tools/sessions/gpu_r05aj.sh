#!/bin/bash
# Round 5: tile-pair groups of four (quad2) against two (on2) and the one-tile groups (on) on
# one GPU: whole-image 64-frame launches (K4's structure) and 20-frame chains at the whole
# image and a 2-rank share (tools/pairs_ab.py, modes alternating call by call).
# Usage: bash tools/sessions/gpu_r05aj.sh TAG
set -o pipefail
TAG=${1:-r05aj}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/pairs_ab.py 9 1 on,on2,quad2 64 last_two > $O/pairs_k4.jsonl 2> $O/pairs_k4.err \
  || { echo "pairs_ab failed"; tail $O/pairs_k4.err; exit 1; }
cat $O/pairs_k4.jsonl
timeout -k 10 300 python tools/pairs_ab.py 9 1,2 on,on2,quad2 20 every > $O/pairs_chain.jsonl 2> $O/pairs_chain.err \
  || { echo "pairs_ab failed"; tail $O/pairs_chain.err; exit 1; }
cat $O/pairs_chain.jsonl
